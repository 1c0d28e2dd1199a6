"""The C++ drop-in classes (sdr-j-dab_amd/host/dabgpu_dropin.h: viterbi,
uep_/eep_deconvolve, reedSolomon, phaseReference, ficHandler, mscHandler,
ofdmProcessor and the streaming ensembleDecoder) on the GPU, checked by
tests/cpp/test_dropin.cpp against the CPU oracle and the transmitter's truth, and by
tests/cpp/test_gui.cpp, which replays gui.cpp's call sequence (service lookups on the
ficHandler, set_audioChannel / set_dataChannel, setFiles, stop, clearEnsemble) and
whose MPEG layer II file and MSC data groups are compared here with the oracle's
mp2Processor / mscDatagroup restatements run on the oracle's MSC bits of the same IQ."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_dropin")
GUI = os.path.join(ROOT, "tests", "cpp", "build", "test_gui")


def _make():
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "tests", "cpp", "Makefile")], check=True)


@pytest.mark.gpu
def test_cpp_dropin_classes():
    _make()
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=600)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and "DROPIN OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_gui_sequence_and_msc_consumers_match_oracle(tmp_path):
    _make()
    r = subprocess.run([GUI, str(tmp_path)], capture_output=True, text=True, timeout=600)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and "GUI OK" in r.stdout, r.stdout + r.stderr
    sys.path[:0] = [os.path.join(ROOT, "sdr-j-dab_amd"), os.path.join(ROOT, "tests")]
    import oracle_py as orc
    from dabamd.synth import Ensemble, MP2, PACKET
    # the ensemble of test_gui.cpp (NF, SC, cfg, seed)
    NF = 28
    sub = [(0, 96, 128, 0o103, 0, 0, MP2), (96, 48, 64, 0o103, 0, 1, 0), (144, 24, 32, 0o103, 0, 0, PACKET)]
    ens = Ensemble(NF, subch=sub, pre_offset=50000, snr_db=25.0, cfo_hz=50.0, amplitude=1.0, figs=True)
    g = ens.generate(2024, truth=False)
    ref = orc.decode_stream(g["iq"], NF + 1, [s[:5] for s in sub])
    n = ref["n"]
    assert n >= NF - 1
    # mp2Processor with the mp2 file set: lf bytes per frame (lf = the frame's bit count)
    m = orc.MP2(128)
    d = orc.Datagroups(60, 0)
    for c in range(16, 4 * n):
        m.add(ref["msc"][c, 0, :24 * 128])
        d.add(ref["msc"][c, 2, :24 * 32])
    lf = 24 * 128
    want = b"".join(f + bytes(lf - len(f)) for f, rate in m.frames)
    got = open(tmp_path / "mp2.bin", "rb").read()
    assert len(m.frames) >= 4 * n - 16 - 2
    assert got[:len(want)] == want                       # the oracle's frames, in order
    assert 0 <= len(got) - len(want) <= 8 * lf           # (the drop-in may decode the stream's last frame too)
    raw = open(tmp_path / "datagroups.bin", "rb").read()
    groups, o = [], 0
    while o < len(raw):
        nb = int(np.frombuffer(raw[o:o + 4], "<u4")[0])
        groups.append(list(raw[o + 4:o + 4 + nb]))
        o += 4 + nb
    assert d.crc_errors == 0 and len(d.groups) >= 10
    assert groups[:len(d.groups)] == d.groups
    assert len(groups) - len(d.groups) <= 16
    # the OFDM classes' display feeds (ofdm-processor.h:49-59, ofdm-decoder.h:40-44):
    # iqBuffer (ofdm-decoder.cpp:192-206) -- every 8th frame's symbol-2 carriers, within
    # 1e-5 of the spectrum's RMS of the oracle's FFT of the same (NCO-mixed) samples;
    # spectrumBuffer (ofdm-processor.cpp:161-180,220-238) -- 32768 raw input samples per
    # emission, at the reference's positions, bit for bit
    _, _, _, disp, dfr, spec = orc.ofdm_run_display(g["iq"], NF + 1, max_disp=16, max_spec=64)
    iqd = np.fromfile(tmp_path / "iq_display.bin", np.complex64).reshape(-1, 1536)
    k = min(len(iqd), len(disp))
    assert k >= 3 and list(dfr[:3]) == [7, 15, 23]
    for i in range(k):
        rms = np.sqrt(np.mean(np.abs(disp[i]) ** 2))
        err = np.abs(iqd[i] - disp[i]).max() / rms
        assert err <= 1e-5, (i, err)
    spd = np.fromfile(tmp_path / "spectrum.bin", np.complex64).reshape(-1, 32768)
    x = g["iq"].view(np.complex64)
    k = min(len(spd), len(spec))
    assert k >= 10 and len(spec) - len(spd) <= 2, (len(spd), len(spec))
    for i in range(k):
        assert np.array_equal(spd[i].view(np.uint64), x[spec[i]:spec[i] + 32768].view(np.uint64)), (i, spec[i])


def test_cpp_dropin_builds():
    """the drop-in library and its tests link on a host without a GPU"""
    _make()
    assert os.path.exists(EXE) and os.path.exists(GUI)
