"""Recorded-IQ file formats, host side: the .sdr WAV header check
of wavFiles (wavfiles.cpp:56-69: 2 channels at 2048000 Hz, else "not a recorded dab
file") and the .raw byte stream of rawFiles (rawfiles.cpp:100-118).  The GPU
conversion itself is tested in test_gpu_formats.py."""
import os
import wave

import numpy as np
import pytest


def test_sdr_roundtrip(tmp_path):
    import dabamd
    rng = np.random.default_rng(3)
    iq = rng.integers(-32768, 32768, 2 * 1001, dtype=np.int16)
    p = str(tmp_path / "x.sdr")
    dabamd.write_sdr(p, iq)
    got = dabamd.read_sdr(p)
    assert got.dtype == np.dtype("<i2") and np.array_equal(np.asarray(got), iq)


@pytest.mark.parametrize("ch,rate,width", [(1, 2048000, 2), (2, 48000, 2), (2, 2048000, 1)])
def test_sdr_rejects_other_layouts(tmp_path, ch, rate, width):
    import dabamd
    p = str(tmp_path / "bad.wav")
    with wave.open(p, "wb") as w:
        w.setnchannels(ch)
        w.setsampwidth(width)
        w.setframerate(rate)
        w.writeframes(b"\0" * (ch * width * 16))
    with pytest.raises(ValueError):
        dabamd.read_sdr(p)


def test_sdr_skips_unknown_chunks(tmp_path):
    """a LIST chunk between fmt and data (common in recorder output) is skipped"""
    import dabamd
    import struct
    iq = np.arange(-8, 8, dtype=np.int16)
    fmt = struct.pack("<HHIIHH", 1, 2, 2048000, 2048000 * 4, 4, 16)
    lst = b"INFOtest!"                                       # odd size: padded
    data = iq.tobytes()
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"LIST" + struct.pack("<I", len(lst)) + lst + b"\0" \
        + b"data" + struct.pack("<I", len(data)) + data
    p = str(tmp_path / "list.sdr")
    with open(p, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)
    assert np.array_equal(np.asarray(dabamd.read_sdr(p)), iq)


def test_raw_drops_odd_byte(tmp_path):
    import dabamd
    p = str(tmp_path / "x.raw")
    b = np.arange(11, dtype=np.uint8)
    b.tofile(p)
    got = dabamd.read_raw(p)
    assert got.size == 10 and np.array_equal(np.asarray(got), b[:10])


def test_ringbuffer_and_sdr_dump_standin(tmp_path):
    """the drop-in RingBuffer (ringbuffer.h:127-319 contract, SPSC stress under TSan) and
    the libsndfile stand-in behind ofdmProcessor::startDumping(SNDFILE *): the .sdr it
    writes is what gui.cpp:879-883 asks sf_open for (WAV, PCM16, 2 channels, 2.048 MHz)"""
    import subprocess
    import wave
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-f", os.path.join(root, "tests", "cpp", "Makefile")], check=True)
    out = tmp_path / "dump.sdr"
    r = subprocess.run([os.path.join(root, "tests", "cpp", "build", "test_ringbuffer"), str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "RINGBUFFER OK" in r.stdout, r.stdout + r.stderr
    with wave.open(str(out)) as w:
        assert (w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()) == (2, 2, 2048000, 3 * 4096)
        d = np.frombuffer(w.readframes(3 * 4096), "<i2").reshape(-1, 2)
    k = np.arange(3 * 4096)
    assert np.array_equal(d[:, 0], (k - 6000).astype(np.int16)) and np.array_equal(d[:, 1], (-k).astype(np.int16))


def test_dropin_binds_libsndfile_when_built_with_it():
    """built with -DDABGPU_HAVE_SNDFILE the drop-ins take
    libsndfile's own SNDFILE / SF_INFO / sf_* (the stand-in steps aside), so gui.cpp's
    set_dumping (gui.cpp:861-893) hands its ::SNDFILE* to ofdmProcessor::startDumping
    unchanged.  libsndfile is absent here: compiled against its API declarations
    (tests/cpp/sndfile_api/sndfile.h), not linked."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    inc = ["-I" + os.path.join(root, "tests", "cpp", "sndfile_api"), "-I" + os.path.join(root, "include"),
           "-I" + os.path.join(root, "sdr-j-dab_amd", "host")]
    for src in (os.path.join(root, "sdr-j-dab_amd", "host", "dabgpu_frontend.cpp"),
                os.path.join(root, "tests", "cpp", "gui_dump_sndfile.cpp")):
        r = subprocess.run([gxx, "-std=c++17", "-fsyntax-only", "-Wall", "-DDABGPU_HAVE_SNDFILE"] + inc + [src],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-2000:]
