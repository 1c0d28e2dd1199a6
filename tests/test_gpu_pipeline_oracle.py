"""The GPU streaming pipeline against the reference CPU path (oracle), end to end, where
decoded-bit parity can fail: near the decoding threshold (11-12 dB SNR), under carrier
frequency offsets (the general NCO path: per-sample oscillator indices, coarse and fine
AFC), at the full sizes of configs C3 (64 ensembles x 9 UEP-3 subchannels = 864 CUs)
and C5 (256 DAB+ subchannels), with a signal dropout (sync loss and re-acquisition
inside a run, ofdm-processor.cpp:354-357) and with streams out of lockstep.

The oracle decodes the SAME IQ sequentially (oracle_py.decode_stream: ofdmProcessor::run
-> processToken soft bits -> ficHandler / dabConcurrent -> Viterbi), so FIC/MSC bits are
compared with what the reference's own decoding of its own soft bits gives.  Bar:
frame placement and correctors identical; decoded FIC/MSC bits and CRC flags
identical (0 mismatches); int16 soft bits identical except +-1 where the FFT rounding
(FFTW3f in the reference, absent here: unpinned) moves q*127 across an integer.

Every pipeline test runs on cf32 streams and on the same streams stored as .sdr PCM16
samples (dabgpu_pipe_set_iq_format(DABGPU_IQ_S16): the kernels convert x / 32768 in their
loads); the quantised floats are what the oracle decodes, so the bar is unchanged.  A
subset also runs on .raw u8 samples (rawfiles.cpp:115-117).  The synthetic transmitter's
amplitude is 0.25 for the recorded formats (peaks inside +-1, as a recording's gain
would set them)."""
import numpy as np
import pytest

import oracle_py as orc
import pipeline_check as pc

pytestmark = pytest.mark.gpu

SOFT_BOUNDARY_RATE = 1e-4       # int16 soft bits that may differ by 1 (FFT rounding)


@pytest.fixture(scope="module")
def ctx():
    import dabamd
    c = dabamd.Context(0)
    yield c
    c.close()


F32, S16, U8 = pc.IQ_F32, pc.IQ_S16, pc.IQ_U8
FMTS = pytest.mark.parametrize("fmt", [F32, S16], ids=["f32", "s16"])


def _amp(fmt):
    return 1.0 if fmt == F32 else 0.25


def _gen(subch, frames, seeds, snr, cfo=0.0, fmt=F32):
    """synthetic streams as the format carries them (pc.quantize)"""
    from dabamd.synth import Ensemble
    e = Ensemble(frames, subch=subch, snr_db=snr, cfo_hz=cfo, amplitude=_amp(fmt))
    if len(seeds) > 4:
        iq = e.generate_many(len(seeds), seed0=seeds[0], threads=16)
        return [pc.quantize(iq[i], fmt) for i in range(len(seeds))]
    return [pc.quantize(e.generate(s, truth=False)["iq"], fmt) for s in seeds]


def _check(stats, what, soft=True):
    for s, r in enumerate(stats):
        assert r["frames"] > 0, (what, s, r)
        assert r["placement"] == 0, (what, s, r)
        assert r["fic_bad"] == 0 and r["crc_bad"] == 0, (what, s, r)
        assert r["msc_bad"] == 0, (what, s, r)
        if soft and r["soft"]:
            assert r["soft_offby1_only"], (what, s, r)
            assert r["soft_bad"] <= SOFT_BOUNDARY_RATE * r["soft"], (what, s, r)


MIXED = [(0, 96, 128, 3, 1), (96, 48, 64, 0o103, 0), (144, 24, 32, 0o104, 0), (168, 84, 96, 2, 1),
         (768, 96, 128, 3, 1)]


@FMTS
@pytest.mark.parametrize("snr,cfo,runs", [(11.0, 0.0, 3), (8.0, 0.0, 3), (12.0, 300.0, 8), (12.0, 800.0, 8),
                                          (11.5, -1700.0, 8), (25.0, 2300.0, 3), (20.0, -9700.0, 4),
                                          (20.0, 6400.0, 4)])
def test_pipeline_bits_match_reference_path(ctx, snr, cfo, runs, fmt):
    """two ensembles, 5 subchannels (UEP-3/-2, EEP-3A/-4A, one above CU 511), runs of 4
    frames: every committed frame's placement/correctors, soft bits, FIC bits + CRCs and
    MSC bits against the oracle run on the same IQ.  8 dB is at the FIC's decoding
    threshold for this transmitter (CRC failures in both); with a CFO the fine AFC
    converges by 10% per frame (ofdm-processor.cpp:445-446), hence 32 frames.  -9.7 and
    +6.4 kHz are several carriers off: the coarse corrector (processBlock_0's offset,
    ofdm-processor.cpp:395-406) has to move first."""
    F = 4
    iqs = _gen(MIXED, F * runs + 1, [31, 32], snr, cfo, fmt)
    refs = orc.decode_streams(iqs, F * runs, MIXED)
    gpu = pc.gpu_decode(ctx, iqs, F, runs, MIXED, soft_streams=(0, 1), iq_format=fmt)
    stats = [pc.compare(gpu[s], refs[s], MIXED) for s in range(2)]
    print(f"snr {snr} cfo {cfo} fmt {fmt}:", stats)
    _check(stats, (snr, cfo, fmt))
    if abs(cfo) > 2000.0:
        return                        # the reference's AFC may wander here; parity is what counts
    for s in range(2):
        # the same frames as the reference (a stream that loses sync under a large
        # offset re-acquires inside the run and delivers fewer frames -- in both)
        assert stats[s]["frames"] == stats[s]["oracle_frames"] >= F * runs - 4
        assert stats[s]["msc_cw"] >= (4 * stats[s]["frames"] - 16) * len(MIXED)
    ctx.check()


@FMTS
def test_pipeline_corrector_sequence_under_drifting_cfo(ctx, fmt):
    """the AFC loop over a long run (40 frames) under a carrier offset that DRIFTS from +900
    to +1,150 Hz (a linear chirp applied to the transmitted signal, 6 Hz per frame: the
    loop's 10 % gain lags it by ~60 Hz, within DQPSK's reach): the fine corrector
    (ofdm-processor.cpp:445-446, int16 truncation of 0.1 arg(FreqCorr) / pi * 500) steps
    every frame and wraps into the coarse one past +-500 Hz (:458-466), and FreqCorr is
    accumulated by the GPU in its own order (raw samples, rotated once) -- the
    per-frame (coarse, fine) sequence, frame placement and decoded bits must equal the
    oracle's ofdmProcessor::run frame for frame"""
    from dabamd.synth import Ensemble
    sub = MIXED[:2]
    F, runs = 4, 10
    e = Ensemble(F * runs + 2, subch=sub, snr_db=15.0, amplitude=_amp(fmt))
    g = e.generate(81, truth=False)
    x = g["iq"].reshape(-1, 2).astype(np.float64)
    n = np.arange(len(x), dtype=np.float64)
    f0, f1 = 900.0, 1150.0
    rate = (f1 - f0) / (len(x) / 2048000.0)                 # Hz per second
    ph = 2 * np.pi * (f0 * n + 0.5 * rate * n * n / 2048000.0) / 2048000.0
    z = (x[:, 0] + 1j * x[:, 1]) * np.exp(1j * ph)
    iq = pc.quantize(np.stack([z.real, z.imag], axis=1).astype(np.float32).reshape(-1), fmt)
    ref = orc.decode_stream(iq, F * runs, sub)
    gpu = pc.gpu_decode(ctx, [iq], F, runs, sub, soft_streams=(0,), iq_format=fmt)
    st = pc.compare(gpu[0], ref, sub)
    seq = [(fi.coarse, fi.fine) for fi in gpu[0]["info"]]
    print("drifting CFO:", st, "correctors", seq[::4])
    _check([st], ("drift", fmt))
    assert st["frames"] == ref["n"] >= F * runs - 2
    assert seq == [(fi.coarse, fi.fine) for fi in ref["info"][:len(seq)]]
    fines = [f for _, f in seq]
    assert len(set(fines)) > 10 and len({c for c, _ in seq}) >= 2     # the loop moved, coarse included


@FMTS
@pytest.mark.parametrize("method", [0, 2])
def test_pipeline_freq_sync_methods(ctx, method, fmt):
    """freqSyncMethod 0 (getMiddle) and 2 (pattern match) in processBlock_0
    (ofdm-decoder.cpp:103-104,128-161,233-258) through the pipeline under CFO"""
    F, runs = 3, 2
    sub = MIXED[:2]
    iqs = _gen(sub, F * runs + 1, [41], 20.0, 1200.0, fmt)
    ref = orc.decode_stream(iqs[0], F * runs, sub, method=method)
    gpu = pc.gpu_decode(ctx, iqs, F, runs, sub, method=method, iq_format=fmt)
    st = pc.compare(gpu[0], ref, sub, check_soft=False)
    print("method", method, st)
    _check([st], method, soft=False)
    assert st["frames"] == ref["n"]


@FMTS
def test_pipeline_dropout_reacquires_like_reference(ctx, fmt):
    """1.5 frames of the signal replaced by an interferer (a carrier at +100 kHz: its
    PRS correlation is flat, so findIndex fails -- Max < 3 * mean): the stream goes back
    to the null search from where it is (goto notSynced), which finds the next null once
    the signal returns -- frame for frame the oracle's ofdmProcessor::run, inside ONE
    pipeline run (DABGPU_CTL_ACQ_SYNC, as every test here that counts frames: the reference's
    in-run search; the engine's default searches in the background,
    test_pipeline_background_reacquisition_like_reference)"""
    from dabamd.synth import Ensemble
    sub = MIXED[:2]
    F, runs = 4, 3
    e = Ensemble(F * runs + 4, subch=sub, snr_db=20.0, amplitude=_amp(fmt))
    g = e.generate(51, truth=False)
    iq = g["iq"].reshape(-1, 2).copy()
    a = g["frame0"] + 3 * 196608 + 40000
    b = a + 300000
    # (plus a noise floor 20 dB below it: without one, the FFT bins next to the carrier
    # hold only rounding noise and the soft bits of the half-jammed frame are arbitrary)
    level = float(np.sqrt((iq[:200000] ** 2).sum(1).mean()))
    ph = 2 * np.pi * 100e3 / 2048000 * np.arange(b - a)
    rng = np.random.default_rng(5)
    iq[a:b, 0] = level * np.cos(ph) + rng.normal(0, level / 10, b - a)
    iq[a:b, 1] = level * np.sin(ph) + rng.normal(0, level / 10, b - a)
    iq = pc.quantize(np.ascontiguousarray(iq.reshape(-1)), fmt)
    ref = orc.decode_stream(iq, F * runs, sub)
    gpu = pc.gpu_decode(ctx, [iq], F, runs, sub, soft_streams=(0,), iq_format=fmt)
    st = pc.compare(gpu[0], ref, sub)
    print("dropout:", st, [(x.resyncs, x.acquisitions, x.frames_run) for x in gpu[0]["states"]])
    _check([st], "dropout")
    assert st["frames"] == ref["n"] >= F * runs - 2
    last = gpu[0]["states"][-1]
    assert last.resyncs >= 1 and last.acquisitions >= 2
    wins = [fi.window_start for fi in ref["info"]]
    assert any(w2 - w1 != 196608 for w1, w2 in zip(wins, wins[1:]))    # the dropout broke the frame grid


@FMTS
def test_pipeline_digital_silence_like_reference(ctx, fmt):
    """exact zero samples over six data symbols of a frame (a recording's digital
    silence): their spectra are 0, so r = X conj(P) = 0 and q = -re / (|re| + |im|) is
    0 / 0 in the reference (ofdm-decoder.cpp:185-189) -- the soft-bit fast path must hand
    those bins to the exact path (NaN -> the same int16 as the reference's conversion) on
    both formats (the bounded formats decide it without the range compare), and the frame
    after them decodes as the reference's"""
    from dabamd.synth import Ensemble
    sub = MIXED[:3]
    F, runs = 4, 2
    e = Ensemble(F * runs + 4, subch=sub, snr_db=25.0, amplitude=_amp(fmt))
    g = e.generate(53, truth=False)
    iq = g["iq"].reshape(-1, 2).copy()
    a = g["frame0"] + 2 * 196608 + 20000           # data symbols ~7..13 of the third frame
    iq[a:a + 6 * 2552] = 0.0
    iq = pc.quantize(np.ascontiguousarray(iq.reshape(-1)), fmt)
    ref = orc.decode_stream(iq, F * runs, sub)
    gpu = pc.gpu_decode(ctx, [iq], F, runs, sub, soft_streams=(0,), iq_format=fmt)
    st = pc.compare(gpu[0], ref, sub)
    print("silence:", st)
    _check([st], "silence")
    assert st["frames"] == ref["n"] >= F * runs - 1
    ctx.check()


@FMTS
def test_pipeline_background_reacquisition_like_reference(ctx, fmt):
    """The engine's default re-acquisition (DABGPU_CTL_ACQ_ASYNC, round 6), and the same
    mode set explicitly: stream 0 loses sync in a dropout (as above); its null search runs
    in the background while stream 1 keeps decoding n_frames per run, and the runs after
    the search continue stream 0 from the null it found -- both streams' frames (placement,
    FIC, MSC, soft bits) equal the oracle's ofdmProcessor::run frame for frame, stream 0's
    delivered later"""
    from dabamd.synth import Ensemble
    sub = MIXED[:2]
    F, runs = 4, 7
    e = Ensemble(F * runs + 4, subch=sub, snr_db=20.0, amplitude=_amp(fmt))
    g0, g1 = e.generate(51, truth=False), e.generate(52, truth=False)
    iq = g0["iq"].reshape(-1, 2).copy()
    a = g0["frame0"] + 3 * 196608 + 40000
    b = a + 300000
    level = float(np.sqrt((iq[:200000] ** 2).sum(1).mean()))
    ph = 2 * np.pi * 100e3 / 2048000 * np.arange(b - a)
    rng = np.random.default_rng(5)
    iq[a:b, 0] = level * np.cos(ph) + rng.normal(0, level / 10, b - a)
    iq[a:b, 1] = level * np.sin(ph) + rng.normal(0, level / 10, b - a)
    iqs = [pc.quantize(np.ascontiguousarray(iq.reshape(-1)), fmt), pc.quantize(g1["iq"], fmt)]
    refs = orc.decode_streams(iqs, F * runs, sub)
    for acq in ("default", "async"):
        gpu = pc.gpu_decode(ctx, iqs, F, runs, sub, soft_streams=(0, 1), acq=acq, iq_format=fmt)
        runs0 = [(x.frames_run, x.acquiring, x.resyncs) for x in gpu[0]["states"]]
        print("background re-acquisition", acq, runs0)
        assert all(x.frames_run == F for x in gpu[1]["states"])          # stream 1 never waits
        assert any(fr < F for fr, _, _ in runs0)                          # stream 0 missed runs while searching
        assert gpu[0]["states"][-1].resyncs >= 1 and gpu[0]["states"][-1].acquisitions >= 2
        for s in range(2):
            st = pc.compare(gpu[s], refs[s], sub)
            print("stream", s, st)
            _check([st], ("background", acq, s))
        st0 = pc.compare(gpu[0], refs[0], sub)
        assert st0["frames"] > 4                   # frames after the dropout were decoded too


def test_background_search_flag_clears_without_a_run(ctx):
    """dabgpu_stream_state.acquiring tells a caller when the background null
    search (DABGPU_CTL_ACQ_ASYNC) no longer reads iq_d -- it clears once the search is done,
    seen through dabgpu_pipe_state alone (no further run); dabgpu_pipe_acquire_wait waits
    for it; a RESYNC issued while a search is in flight waits for it and wins (the stream
    searches again from its new position at the next run)"""
    import time
    import dabamd
    from dabamd.synth import Ensemble
    sub = MIXED[:1]
    F = 4
    e = Ensemble(6 * F + 4, subch=sub, snr_db=20.0)
    g = e.generate(51, truth=False)
    iq = g["iq"].reshape(-1, 2).copy()
    a = g["frame0"] + 3 * 196608 + 40000
    b = a + 300000
    level = float(np.sqrt((iq[:200000] ** 2).sum(1).mean()))
    ph = 2 * np.pi * 100e3 / 2048000 * np.arange(b - a)
    iq[a:b, 0] = level * np.cos(ph)
    iq[a:b, 1] = level * np.sin(ph)
    x = np.ascontiguousarray(iq.reshape(-1))
    n = len(x) // 2
    diq = ctx.put(x[None, :])

    def until_loss(pipe):
        pipe.acquire(diq, n, [0], [n])
        pipe.control(dabamd.CTL_ACQ_ASYNC)
        for r in range(5):
            pipe.run(diq, n, [n], partial=True)
            if pipe.state(0).frames_run < F:          # the sync loss: a search was launched
                return True
        return False
    try:
        for mode in ("poll", "resync"):
            pipe = dabamd.Pipeline(ctx, 1, F, [dabamd.Subch(*sub[0][:4], 0, 0)])
            try:
                assert until_loss(pipe)
                if mode == "poll":
                    t0 = time.time()
                    while pipe.state(0).acquiring and time.time() - t0 < 5.0:
                        time.sleep(0.001)
                    assert pipe.state(0).acquiring == 0        # cleared without another run
                    pipe.acquire_wait()                         # nothing in flight: at once
                else:
                    pipe.control(dabamd.CTL_RESYNC)             # at once: the search may be in flight
                    st = pipe.state(0)
                    assert st.acquiring == 0 and st.synced == 0  # it waited, and RESYNC won
                pipe.run(diq, n, [n], partial=True)             # decodes on from there
                pipe.acquire_wait()
                pipe.sync()
                ctx.check()
            finally:
                pipe.close()
    finally:
        diq.free()


@FMTS
def test_pipeline_streams_out_of_lockstep(ctx, fmt):
    """stream 1 gets fewer samples in run 1 (it commits fewer frames, DABGPU_E_STATE),
    then all of them: its CIF count, 16-CIF de-interleaver and warm-up follow its own
    frames, and run 2's MSC bits of BOTH streams equal the reference path's"""
    sub = MIXED[:3]
    F = 3
    iqs = _gen(sub, 3 * F + 1, [61, 62], 30.0, fmt=fmt)
    n = len(iqs[0]) // 2
    refs = orc.decode_streams(iqs, 3 * F, sub)
    fi = refs[1]["info"][1]                    # stream 1 gets samples up to the end of its 2nd frame
    short = fi.window_start + fi.start_index + 2048 + 75 * 2552 + 10
    gpu = pc.gpu_decode(ctx, iqs, F, 3, sub, n_avail=[[n, short], [n, n], [n, n]], iq_format=fmt)
    assert gpu[1]["states"][0].frames_run < F and gpu[0]["states"][0].frames_run == F
    for s in range(2):
        st = pc.compare(gpu[s], refs[s], sub, check_soft=False)
        print("lockstep", s, st)
        _check([st], ("lockstep", s), soft=False)
        assert st["msc_cw"] > 0


@pytest.mark.parametrize("fmt", [F32, S16, U8], ids=["f32", "s16", "u8"])
def test_c3_full_size_bits_match_reference_path(ctx, fmt):
    """config C3 at its size: 64 ensembles x 9 UEP-3 128 kbit/s subchannels (all 864
    CUs), 3 runs of 3 frames (36 CIFs: 20 past the 16-CIF warm-up), 12 dB SNR.  Every
    ensemble's FIC and MSC bits against the reference path; soft bits of 4 ensembles."""
    sub = [(96 * i, 96, 128, 3, 1) for i in range(9)]
    F, runs, E = 3, 3, 64
    iqs = _gen(sub, F * runs + 1, list(range(7000, 7000 + E)), 12.0, fmt=fmt)
    refs = orc.decode_streams(iqs, F * runs, sub)
    gpu = pc.gpu_decode(ctx, iqs, F, runs, sub, soft_streams=(0, 21, 42, 63), iq_format=fmt)
    stats = [pc.compare(gpu[s], refs[s], sub) for s in range(E)]
    tot = {k: sum(r[k] for r in stats) for k in ("frames", "fic_cw", "msc_cw", "fic_bad", "msc_bad", "soft", "soft_bad")}
    print("C3 fmt", fmt, tot)
    _check(stats, "C3")
    assert tot["msc_cw"] == E * 9 * (4 * F * runs - 16)


@FMTS
def test_c5_full_size_superframes_match_reference_path(ctx, fmt):
    """config C5 at its size: 16 ensembles x 16 DAB+ 64 kbit/s EEP-3A subchannels = 256,
    3 runs of 3 frames at 11 dB: MSC bits and every superframe record (fire code, RS
    corrections, AU table, AU CRCs, bytes) against the oracle's mp4Processor fed with
    the ORACLE's own MSC bits"""
    sub = [(48 * i, 48, 64, 0o103, 0, 1) for i in range(16)]
    F, runs, E = 3, 3, 16
    iqs = _gen(sub, F * runs + 1, list(range(8000, 8000 + E)), 11.0, fmt=fmt)
    refs = orc.decode_streams(iqs, F * runs, sub)
    gpu = pc.gpu_decode(ctx, iqs, F, runs, sub, dabplus=True, iq_format=fmt)
    n = bad = ok3 = 0
    for s in range(E):
        st = pc.compare(gpu[s], refs[s], sub, check_soft=False)
        _check([st], ("C5", s), soft=False)
        a, b, c = pc.compare_dabplus(gpu[s], refs[s], sub)
        n, bad, ok3 = n + a, bad + b, ok3 + c
    print("C5 superframe records:", n, "mismatches:", bad, "decoded:", ok3)
    assert bad == 0 and ok3 > 0


@pytest.mark.parametrize("pad,fmt,packed", [(0, F32, True), (1, F32, True), (0, S16, True), (0, U8, True),
                                            (0, S16, "fic"), (1, U8, "fic")])
def test_packed_msc_output_and_dabplus_match_reference_path(ctx, pad, fmt, packed):
    """dabgpu_pipe_set_packed: the traceback writes the MSC bits 8 per byte (msb first,
    mp4processor.cpp:115-121's packing) and the DAB+ layer reads those bytes -- FIC, MSC
    and every superframe record equal the reference path, with UEP/EEP and DAB+
    subchannels side by side, near the decoding threshold.  pad 1: an odd row stride (the
    traceback's byte stores instead of 16-bit ones, the DAB+ layer's byte-wise window
    copy instead of 4-byte loads).  "fic": DABGPU_PACK_FIC as well -- the FIBs as bytes
    (CRC bytes inverted in place, as check_CRC_bits leaves the bits) and the CRC flags of
    the packed-byte check, both equal the reference path's"""
    sub = [(0, 96, 128, 3, 1, 0), (96, 48, 64, 0o103, 0, 1), (144, 24, 32, 0o104, 0, 0), (168, 36, 48, 0o103, 0, 1),
           (768, 96, 128, 3, 1, 0)]
    F, runs = 4, 5
    iqs = _gen(sub, F * runs + 1, [61, 62], 11.0, fmt=fmt)
    refs = orc.decode_streams(iqs, F * runs, sub)
    gpu = pc.gpu_decode(ctx, iqs, F, runs, sub, dabplus=True, packed=packed, packed_pad=pad, iq_format=fmt)
    ok3 = 0
    for s in range(2):
        st = pc.compare(gpu[s], refs[s], sub, check_soft=False)
        _check([st], ("packed", s), soft=False)
        assert st["msc_cw"] == len(sub) * (4 * st["frames"] - 16)
        n, bad, c = pc.compare_dabplus(gpu[s], refs[s], sub)
        assert bad == 0, (s, n, bad)
        ok3 += c
    assert ok3 > 0


@pytest.mark.parametrize("packed", [False, "fic"], ids=["bits", "fib_bytes"])
def test_fic_only_pipeline_matches_reference_path(ctx, packed):
    """a pipeline that decodes no subchannel: the FIC alone through its own ACS and
    traceback launches (not the MSC's shared ones) and k_fic_post -- FIC bits (or, with
    DABGPU_PACK_FIC, FIB bytes: the traceback's packed stores at a 96-byte row stride and the
    CRC check on bytes) and CRC flags equal the reference path's, near the threshold"""
    F, runs = 4, 3
    iqs = _gen(MIXED, F * runs + 1, [41, 42], 9.0, fmt=S16)
    refs = orc.decode_streams(iqs, F * runs, MIXED)
    gpu = pc.gpu_decode(ctx, iqs, F, runs, [], packed=packed, iq_format=S16)
    for s in range(2):
        st = pc.compare(gpu[s], refs[s], [], check_soft=False)
        _check([st], ("fic only", packed, s), soft=False)
        assert st["fic_cw"] == 4 * st["frames"] and st["msc_cw"] == 0


def test_pipeline_null_lock_like_reference(ctx):
    """the stream on which the reference's null search locks onto the frame period after a
    sync loss (tests/null_lock.py, test_null_search_locks_onto_frame_period_like_reference):
    with the reference's in-run search (ACQ_SYNC) the pipeline decodes the same 229 frames
    as the oracle's ofdmProcessor::run -- placement, FIC bits, CRCs -- and is still not
    synchronised when the stream's samples end"""
    import null_lock as nl
    _, x = nl.stream()
    ref = orc.decode_streams([x], nl.FRAMES, [])[0]
    assert ref["n"] == 229
    gpu = pc.gpu_decode(ctx, [x], 8, 32, [], iq_format=S16, acq="sync")[0]
    st = pc.compare(gpu, ref, [], check_soft=False)
    _check([st], "null lock", soft=False)
    assert st["frames"] == 229 and gpu["info"][-1].window == nl.LAST_WINDOW
    assert not gpu["states"][-1].synced


@pytest.mark.parametrize("fmt", [S16, U8], ids=["s16", "u8"])
def test_recorded_format_decodes_like_converted_cf32(ctx, fmt):
    """the pipeline reading .sdr / .raw samples straight from HBM (the conversion inside
    the kernels' loads) against the same pipeline reading those samples converted to cf32
    by dabgpu_iq_convert: frame placement, correctors, every int16 soft bit, FIC and MSC
    bits identical -- the format is a transport, not an approximation -- under a carrier
    offset (the NCO path) and noise"""
    import dabamd
    sub = MIXED[:3]
    F, runs = 4, 4
    iqs = _gen(sub, F * runs + 1, [71, 72], 12.0, 800.0, fmt)
    raw = [pc.to_raw(x, fmt) for x in iqs]
    conv = []
    for r in raw:                                      # dabgpu_iq_convert on the device
        src = ctx.put(r)
        dst = ctx.buf(4 * len(r))
        ctx.iq_convert(fmt, src, len(r) // 2, dst)
        ctx.sync()
        conv.append(dst.download(np.float32, (len(r),)))
        src.free(); dst.free()
        assert np.array_equal(conv[-1], iqs[len(conv) - 1])
    a = pc.gpu_decode(ctx, conv, F, runs, sub, soft_streams=(0, 1))
    b = pc.gpu_decode(ctx, iqs, F, runs, sub, soft_streams=(0, 1), iq_format=fmt)
    for s in range(2):
        assert len(a[s]["info"]) == len(b[s]["info"]) >= F * runs - 4
        for x, y in zip(a[s]["info"], b[s]["info"]):
            assert (x.window, x.start_index, x.coarse, x.fine, x.correction, x.snr) == \
                   (y.window, y.start_index, y.coarse, y.fine, y.correction, y.snr)
        assert np.array_equal(a[s]["fic"], b[s]["fic"]) and np.array_equal(a[s]["crc"], b[s]["crc"])
        assert sorted(a[s]["msc"]) == sorted(b[s]["msc"]) and len(a[s]["msc"]) > 0
        assert all(np.array_equal(a[s]["msc"][c], b[s]["msc"][c]) for c in a[s]["msc"])
        assert sorted(a[s]["soft"]) == sorted(b[s]["soft"])
        assert all(np.array_equal(a[s]["soft"][g], b[s]["soft"][g]) for g in a[s]["soft"])


@pytest.mark.parametrize("fmt", [S16, U8], ids=["sdr", "raw"])
def test_recording_file_decodes_from_hbm_like_reference(ctx, fmt, tmp_path):
    """a recording file (.sdr WAV PCM16, gui.cpp:880-883, or .raw u8) read into HBM as
    the file holds it (Context.load_recording: 4 / 2 bytes per pair, memory-mapped and
    streamed) and decoded by the pipeline straight from those bytes: the bytes equal the
    file's, and placement, soft bits, FIC and MSC equal the oracle's decode of the samples
    the reference's reader would hand over"""
    import dabamd
    sub = MIXED[:2]
    F, runs = 4, 2
    iq = _gen(sub, F * runs + 1, [81], 15.0, 600.0, fmt)[0]
    raw = pc.to_raw(iq, fmt)
    path = tmp_path / ("rec.sdr" if fmt == S16 else "rec.raw")
    if fmt == S16:
        dabamd.write_sdr(str(path), raw)
    else:
        raw.tofile(str(path))
    buf, n, got_fmt = ctx.load_recording(str(path), chunk_pairs=1 << 20)
    try:
        assert got_fmt == fmt and n == len(iq) // 2
        assert np.array_equal(buf.download(raw.dtype, raw.shape), raw)
        ref = orc.decode_stream(iq, F * runs, sub)
        gpu = pc.gpu_decode(ctx, [iq], F, runs, sub, soft_streams=(0,), iq_format=fmt, dev_iq=(buf, n))
        st = pc.compare(gpu[0], ref, sub)
        print("recording:", fmt, st)
        _check([st], "recording")
        assert st["frames"] == ref["n"] >= F * runs - 1
    finally:
        buf.free()


def _profile_mix():
    """subchannels covering the depuncturing kinds the pipeline's input-major ACS loader
    meets (k_viterbi.hip acs_tiles_in): UEP rows with rate-1/4 segments (PI 24: 240
    inputs per 60-step tile), every UEP level of one bitrate, EEP-A 1-4 incl. the 8 kbit/s
    special case, EEP-B 1-4 (deconvolve.cpp:39-114,244-314); lengths from the decoder's
    own fragment sizes, packed into ensembles of <= 864 CUs"""
    import dabamd
    kinds = [(384, 1, 1), (192, 1, 1), (32, 1, 1), (80, 1, 1)] + [(96, l, 1) for l in range(1, 6)] + \
            [(8, 0o101, 0), (8, 0o102, 0), (48, 0o101, 0), (16, 0o102, 0), (24, 0o103, 0), (40, 0o104, 0)] + \
            [(32, 0o201, 0), (64, 0o202, 0), (96, 0o203, 0), (128, 0o204, 0)]
    ens, cur, start = [], [], 0
    for br, prot, uep in kinds:
        _, frag, _, _ = dabamd.subch_profile(dabamd.Subch(0, 864, br, prot, 0 if uep else 1, 0))
        n = (frag + 63) // 64
        if start + n > 864:
            ens.append(cur)
            cur, start = [], 0
        cur.append((start, n, br, prot, uep))
        start += n
    ens.append(cur)
    return ens


@FMTS
def test_pipeline_every_profile_kind_matches_reference_path(ctx, fmt):
    """every depuncturing kind through the streaming pipeline at 9 dB (Viterbi decisions
    that matter): MSC bits of every subchannel and the FIC against the reference path"""
    F, runs = 4, 5
    for g, sub in enumerate(_profile_mix()):
        iqs = _gen(sub, F * runs + 1, [900 + g], 9.0, fmt=fmt)
        ref = orc.decode_stream(iqs[0], F * runs, sub)
        gpu = pc.gpu_decode(ctx, iqs, F, runs, sub, iq_format=fmt)
        st = pc.compare(gpu[0], ref, sub, check_soft=False)
        print("profiles", g, [s[2:] for s in sub], st)
        _check([st], ("profiles", g), soft=False)
        assert st["msc_cw"] == len(sub) * (4 * F * runs - 16)


def test_pipeline_solo_profiling_leaves_outputs_unchanged(ctx):
    """profiling mode 3 (every stage alone on the device, bench.py's solo steps) times the
    stages without changing what the pipeline decodes: FIC bits + CRCs, MSC bits and DAB+
    superframe records of the same IQ with profiling off and in mode 3 are identical, and
    every stage that ran has a positive time"""
    import dabamd
    sub = [(0, 96, 128, 3, 1), (96, 48, 64, 0o103, 0, 1), (144, 48, 64, 0o103, 0, 1)]
    F, runs = 3, 4
    iqs = _gen(sub, F * runs + 1, [61, 62], 20.0)
    S = len(iqs)
    stride = max(len(x) // 2 for x in iqs)
    buf = np.zeros((S, 2 * stride), np.float32)
    for s, x in enumerate(iqs):
        buf[s, :len(x)] = x
    diq = ctx.put(buf)
    subs = [dabamd.Subch(sc[0], sc[1], sc[2], sc[3], 0 if sc[4] else 1,
                         dabamd.SUBCH_DABPLUS if (len(sc) > 5 and sc[5]) else 0) for sc in sub]
    outs = []
    try:
        for mode in (0, 3):
            pipe = dabamd.Pipeline(ctx, S, F, subs)
            try:
                pipe.set_profiling(mode)
                got = []
                for r in range(runs):
                    fic, crc, msc, valid = pipe.run(diq, stride, [stride] * S, download=True)
                    info, sfb = pipe.dabplus(download=True)
                    got.append((fic.copy(), crc.copy(), msc.copy(), valid.copy(), info.copy(), sfb.copy()))
                pipe.sync()
                if mode == 3:
                    t = pipe.timing()
                    for k in ("demod", "msc_acs", "msc_traceback", "dabplus"):
                        assert t[k][1] > 0 and t[k][0] > 0.0, (k, t)
                outs.append(got)
            finally:
                pipe.close()
    finally:
        diq.free()
    for r in range(runs):
        (fa, ca, ma, va, ia, sa), (fb, cb, mb, vb, ib, sb) = outs[0][r], outs[1][r]
        assert np.array_equal(fa, fb) and np.array_equal(ca, cb) and np.array_equal(va, vb), r
        v = va.astype(bool)                 # CIF slots a run did not deliver hold old contents
        for k, sc in enumerate(sub):        # and a row past its subchannel's 24 * bitRate bits
            nb = 24 * sc[2]
            assert np.array_equal(ma[v][:, k, :nb], mb[v][:, k, :nb]), (r, k)
        assert np.array_equal(ia, ib), r
        d = ia["status"] == 3
        assert np.array_equal(sa[d], sb[d]), r
    assert outs[0][-1][3].any() and (outs[0][-1][4]["status"] == 3).any()


def test_scan_mode_counts_attempts_like_reference(ctx):
    """scanMode on a stream with no DAB signal (noise only), handed over in growing pieces
    across several dabgpu_pipe_run calls: the null search gives up every T_F samples,
    `attempts` counts the searches and No_Signal_Found fires after more than 5 of them
    (ofdm-processor.cpp:274-315).  After every call the stream's attempts / no_signal
    equal the reference's counters at the sample where its getSample would block
    (oracle_py.null_scan), including an attempt cut in the middle by the end of the
    available samples and resumed by the next call."""
    import dabamd
    rng = np.random.default_rng(7)
    n = 3_400_000
    iq = rng.normal(0.0, 0.3, 2 * n).astype(np.float32)
    diq = ctx.put(iq)
    pipe = dabamd.Pipeline(ctx, 1, 2, [])
    try:
        pipe.control(dabamd.CTL_SCAN_ON)
        seen = []
        for m in (200_000, 700_000, 1_250_000, 1_251_000, 1_600_000, 2_300_000, 3_000_000, 3_400_000):
            pipe.run(diq, n, [m], partial=True)
            st = pipe.state(0)
            found, att, ns, pos = orc.null_scan(iq, m)
            assert not found and not st.synced
            assert (st.attempts, st.no_signal) == (att, ns), (m, st.attempts, st.no_signal, att, ns)
            seen.append((att, ns))
        assert seen[-1][1] >= 2 and any(a > 0 for a, _ in seen)   # the counters did move
    finally:
        pipe.close()
        diq.free()


@pytest.mark.parametrize("scan", [False, True])
def test_null_search_matches_reference_on_random_streams(ctx, scan):
    """k_acquire against the reference's null search (ofdm-processor.cpp:274-338,
    oracle_py.null_scan) on 48 streams cut from a DAB signal at random offsets: some
    behind a noise prefix (the search gives up after T_F samples and starts over, scan
    mode counting the attempts), some with a quiet gap (a dip whose end does not come
    within T_null + 50 samples: notSynced from SyncOnEndNull), some ending early (out of
    samples inside an attempt).  Every stream's outcome -- synchronised or not, the sample
    where SyncOnPhase starts, attempts, No_Signal_Found -- equals the reference's, which
    pins where the 64-sample groups cut: at the first failing threshold test, at the
    counter limits and at the 1024-sample block ends."""
    import dabamd
    from dabamd.synth import Ensemble
    rng = np.random.default_rng(11 if scan else 12)
    e = Ensemble(5, snr_db=15.0)
    sig = e.generate(77, truth=False)["iq"].view(np.complex64)
    rms = float(np.sqrt(np.mean(np.abs(sig) ** 2)))
    S, L = 48, 1_300_000
    streams = np.zeros((S, L), np.complex64)
    n_avail = []
    for s in range(S):
        kind = s % 4
        off = int(rng.integers(0, 196_608))
        parts = []
        if kind == 1:                                 # noise first: at least one give-up
            z = int(rng.integers(260_000, 520_000))
            parts.append((rms * (rng.normal(size=z) + 1j * rng.normal(size=z)) / np.sqrt(2)).astype(np.complex64))
        if kind == 2:                                 # a quiet gap longer than a null
            g0 = int(rng.integers(60_000, 200_000))
            gap = int(rng.integers(3_000, 9_000))
            parts.append(sig[off:off + g0])
            parts.append((0.01 * rms * rng.normal(size=gap)).astype(np.complex64))
            off += g0
        parts.append(sig[off:])
        x = np.concatenate(parts)[:L]
        streams[s, :len(x)] = x
        n = len(x) if kind != 3 else int(rng.integers(40_000, 260_000))
        n_avail.append(n)
    iq = streams.view(np.float32)
    diq = ctx.put(iq)
    pipe = dabamd.Pipeline(ctx, S, 1, [])
    try:
        if scan:
            pipe.control(dabamd.CTL_SCAN_ON)
        missing = None
        try:
            pipe.acquire(diq, L, [0] * S, n_avail)
        except dabamd.DabError as ex:              # DABGPU_E_STATE: streams still searching
            assert "found no null symbol" in str(ex), ex
            missing = int(str(ex).split(": ")[-1].split()[0])
        synced = 0
        for s in range(S):
            found, att, ns, pos = orc.null_scan(iq[s], n_avail[s], scan)
            st = pipe.state(s)
            assert bool(st.synced) == bool(found), (s, st.synced, found)
            assert (st.attempts, st.no_signal) == (att, ns), (s, st.attempts, st.no_signal, att, ns)
            if found:
                assert st.next_pos == pos, (s, st.next_pos, pos)
            synced += bool(found)
        assert missing == (S - synced if synced < S else None), (missing, synced)
        assert synced >= S // 2, synced                 # most streams found a null
    finally:
        pipe.close()
        diq.free()


@pytest.mark.parametrize("token", [2, 5])
def test_pipeline_iq_display_matches_reference_feed(ctx, token):
    """the constellation feed (ofdmDecoder::processToken, ofdm-decoder.cpp:192-206): the
    pipeline's display-token carriers of every 8th frame equal the oracle's iqBuffer
    pushes (fft_buffer[0, K/2) and [T_u-1-K/2, T_u-1) of the same frame) within 1e-5 of
    the spectrum's RMS, under a carrier offset (the NCO-mixed samples' FFT); token 5 via
    set_displayToken (ofdm-decoder.h:50; dabgpu_pipe_set_display_token)"""
    import dabamd
    from dabamd.synth import Ensemble
    F, runs = 8, 2
    sub = [(0, 96, 128, 3, 1)]
    e = Ensemble(F * runs + 1, subch=[s + (0,) for s in sub], snr_db=20.0, cfo_hz=1300.0)
    iq = e.generate(55, truth=False)["iq"]
    n, info, _, disp, dfr, _ = orc.ofdm_run_display(iq, F * runs, token=token)
    assert n == F * runs and list(dfr) == [7, 15]
    diq = ctx.put(iq[None, :])
    subs = [dabamd.Subch(s[0], s[1], s[2], s[3], 0 if s[4] else 1, 0) for s in sub]
    pipe = dabamd.Pipeline(ctx, 1, F, subs)
    pipe.set_display(True)
    if token != 2:
        pipe.set_display_token(token)
    got = {}
    try:
        for r in range(runs):
            pipe.run(diq, e.length, [e.length])
            frames, si = pipe.frames()
            for f in range(F):
                assert frames[f].window == info[r * F + f].window_start
                got[r * F + f] = pipe.iq_display(0, f)
    finally:
        pipe.close()
        diq.free()
    for k, fidx in enumerate(dfr):
        want = disp[k]
        rms = np.sqrt(np.mean(np.abs(want) ** 2))
        err = np.abs(got[int(fidx)] - want).max() / rms
        print("frame", fidx, "max |gpu - oracle| / rms", err)
        assert err <= 1e-5, (fidx, err)


def test_pipeline_back_end_bounds_error_reported_once(ctx):
    """the back-end streams' error path: an MSC job handed a subchannel offset
    past the soft-bit ring (DABGPU_CTL_INJECT_BOUNDS) is refused by the Viterbi loader; the
    pipeline reports DABGPU_E_BOUNDS exactly once (at dabgpu_pipe_sync), and the next run
    and sync succeed with correct FIC/MSC bits.  The refused subchannel is decoded from
    erasures (the RING8 loader substitutes the erasure byte 127 where the int16
    form reads 0), i.e. exactly the reference's Viterbi of an all-zero soft block, and the
    other subchannel of the same run is unaffected"""
    import dabamd
    sub = MIXED[:2]
    F = 2
    iqs = _gen(sub, 5 * F + 1, [71], 30.0)
    ref = orc.decode_stream(iqs[0], 5 * F, sub)
    diq = ctx.put(iqs[0][None, :])
    subs = [dabamd.Subch(s[0], s[1], s[2], s[3], 0 if s[4] else 1, 0) for s in sub]
    pipe = dabamd.Pipeline(ctx, 1, F, subs)
    n = len(iqs[0]) // 2
    try:
        for _ in range(3):                             # clean, past the 16-CIF warm-up
            pipe.run(diq, n, [n])
        pipe.control(dabamd.CTL_INJECT_BOUNDS)
        valid1 = pipe.run(diq, n, [n], download=False)  # the faulty back end runs behind this call
        with pytest.raises(dabamd.DabError, match="out-of-bounds"):
            pipe.sync()
        pipe.sync()                                    # reported once
        st = pipe.state(0)
        cif0 = st.cif_count - 4 * st.frames_run
        msc1 = pipe.msc_d.download(np.uint8, (1, 4 * F, len(sub), pipe.msc_stride))
        nb0 = 24 * sub[0][2]
        erased = orc.viterbi(np.zeros(4 * (nb0 + 6), np.int16), nb0) ^ orc.prbs(nb0)
        nvalid = 0
        for c in range(4 * F):
            if valid1[0, c]:
                nvalid += 1
                assert np.array_equal(msc1[0, c, 0, :nb0], erased)                  # refused: erasures
                nb1 = 24 * sub[1][2]
                assert np.array_equal(msc1[0, c, 1, :nb1], ref["msc"][cif0 + c, 1, :nb1])
        assert nvalid > 0
        fic, crc, msc, valid = pipe.run(diq, n, [n])   # and the pipeline goes on
        pipe.sync()
        st = pipe.state(0)
        cif0 = st.cif_count - 4 * st.frames_run
        assert st.frames_run == F and crc.all()
        for c in range(4 * F):
            if valid[0, c]:
                for k, sc in enumerate(sub):
                    nb = 24 * sc[2]
                    assert np.array_equal(msc[0, c, k, :nb], ref["msc"][cif0 + c, k, :nb])
        ctx.check()
    finally:
        pipe.close()
        diq.free()


def test_fetch_to_host_equals_download(ctx):
    """dabgpu_pipe_fetch: a run's FIC bits, CRC flags and packed MSC reach pinned host
    memory behind its channel decoding -- through k_to_host at a 16-byte aligned offset and
    through the runtime's copy at an odd one -- equal to a synchronous download of the same
    device buffers, while the next run decodes"""
    import dabamd
    sub = MIXED[:3]
    F, runs = 4, 4
    iqs = _gen(sub, F * runs + 1, [71, 72], 20.0)
    S = len(iqs)
    lens = [len(x) // 2 for x in iqs]
    stride = max(lens)
    buf = np.zeros((S, 2 * stride), np.float32)
    for s, x in enumerate(iqs):
        buf[s, :len(x)] = x
    diq = ctx.put(buf)
    subs = [dabamd.Subch(sc[0], sc[1], sc[2], sc[3], 0 if sc[4] else 1, 0) for sc in sub]
    pipe = dabamd.Pipeline(ctx, S, F, subs)
    pipe.set_packed(True)
    n_fic, n_crc = S * F * 4 * 768, S * F * 12
    n_msc = S * 4 * F * len(sub) * pipe.msc_stride_packed
    total = n_fic + n_crc + n_msc
    hb = [dabamd.HostBuf(ctx, total + 64) for _ in range(2)]
    try:
        for r in range(runs):
            pipe.run(diq, stride, lens, download=False, partial=True)
            h, base = hb[r & 1], (1 if r & 1 else 0)          # odd runs: unaligned -> runtime copy
            o = base
            for src, n in ((pipe.fic_d, n_fic), (pipe.crc_d, n_crc), (pipe.msc_d, n_msc)):
                pipe.fetch(h, src, n, o)
                o += n
            if r >= 1:                                        # the previous run's copy, after this run's
                pipe.sync()
                prev = hb[(r - 1) & 1]
                pb = 1 if (r - 1) & 1 else 0
                got = prev.view(np.uint8, (total,), pb).copy()
                exp = np.concatenate([d.download(np.uint8, (n,)) for d, n in
                                      ((fic_prev, n_fic), (crc_prev, n_crc), (msc_prev, n_msc))])
                assert np.array_equal(got, exp), r
                assert got[:n_fic].any()                      # real decoded bits, not an empty buffer
            fic_prev, crc_prev, msc_prev = pipe.fic_d, pipe.crc_d, pipe.msc_d
    finally:
        for b in hb:
            b.free()


def test_outputs_in_pinned_host_memory_equal_device_outputs(ctx):
    """dabgpu_pipe_run's FIC / CRC / MSC outputs may be dabgpu_host_alloc memory (zero copy:
    the traceback and k_fic_post write across PCIe, bench.py --delivered-mode direct): over
    runs with packed MSC and FIB bytes, the bytes equal a second pipeline's device outputs"""
    import ctypes as C
    import dabamd
    sub = MIXED[:3]
    F, runs = 4, 3
    iqs = _gen(sub, F * runs + 1, [81, 82], 15.0)
    S = len(iqs)
    lens = [len(x) // 2 for x in iqs]
    stride = max(lens)
    buf = np.zeros((S, 2 * stride), np.float32)
    for s, x in enumerate(iqs):
        buf[s, :len(x)] = x
    diq = ctx.put(buf)
    subs = [dabamd.Subch(sc[0], sc[1], sc[2], sc[3], 0 if sc[4] else 1, 0) for sc in sub]
    pa, pb = dabamd.Pipeline(ctx, S, F, subs), dabamd.Pipeline(ctx, S, F, subs)
    hip = C.CDLL("libamdhip64.so")

    class Out:                      # a pinned host buffer through its device address
        def __init__(self, n):
            self.hb = dabamd.HostBuf(ctx, n)
            d = C.c_void_p()
            assert hip.hipHostGetDevicePointer(C.byref(d), self.hb.ptr, 0) == 0 and d.value
            self.ptr = d
    n_fic, n_crc = S * F * 4 * 96, S * F * 12
    n_msc = S * 4 * F * len(sub) * pa.msc_stride_packed
    outs = [(Out(n_fic), Out(n_crc), Out(n_msc)) for _ in range(2)]
    dev = pb._outs                  # pb's own device buffers, freed by close()
    try:
        for p in (pa, pb):
            p.set_packed(dabamd.PACK_MSC | dabamd.PACK_FIC)
        pb._outs = outs
        for r in range(runs):
            pa.run(diq, stride, lens, download=False, partial=True)
            pb.run(diq, stride, lens, download=False, partial=True)
            pa.sync()
            pb.sync()
            for d, h, n in ((pa.fic_d, pb.fic_d, n_fic), (pa.crc_d, pb.crc_d, n_crc), (pa.msc_d, pb.msc_d, n_msc)):
                assert np.array_equal(d.download(np.uint8, (n,)), h.hb.view(np.uint8, (n,))), r
            assert pb.fic_d.hb.view(np.uint8, (n_fic,)).any()
    finally:
        pb._outs = dev
        pa.close()
        pb.close()
        for o in outs:
            for b in o:
                b.hb.free()
        diq.free()


def test_dabplus_compact_output_equals_sparse(ctx):
    """dabgpu_pipe_set_dabplus_compact: the run's decoded superframes in CIF order, slot k
    of the k-th, the record's `reserved` = k -- the same bytes and records as the sparse
    layout, over runs that carry superframes across their seams (11 dB: RS corrections)"""
    import dabamd
    sub = [(0, 48, 64, 0o103, 0, 1), (48, 36, 48, 0o103, 0, 1), (84, 96, 128, 3, 1, 0)]
    F, runs = 4, 6
    iqs = _gen(sub, F * runs + 1, [91, 92], 11.0)
    S = len(iqs)
    lens = [len(x) // 2 for x in iqs]
    stride = max(lens)
    buf = np.zeros((S, 2 * stride), np.float32)
    for s, x in enumerate(iqs):
        buf[s, :len(x)] = x
    diq = ctx.put(buf)
    subs = [dabamd.Subch(sc[0], sc[1], sc[2], sc[3], 0 if sc[4] else 1, dabamd.SUBCH_DABPLUS if sc[5] else 0)
            for sc in sub]
    pa, pb = dabamd.Pipeline(ctx, S, F, subs), dabamd.Pipeline(ctx, S, F, subs)
    for p in (pa, pb):
        p.set_packed(True)
    pb.set_dabplus_compact(True)
    nd, decoded = len(pa.dp), 0
    for r in range(runs):
        pa.run(diq, stride, lens, download=False, partial=True)
        pb.run(diq, stride, lens, download=False, partial=True)
        ia, ba = pa.dabplus()
        ib, bb = pb.dabplus()
        for name in ("status", "num_aus", "n_corrected", "au_start", "au_crc_ok"):
            assert np.array_equal(ia[name], ib[name]), (r, name)
        for s in range(S):
            for d in range(nd):
                end = 110 * (pa.dp[d].bitRate // 8)
                k = 0
                for c in range(4 * F):
                    if ia["status"][s, c, d] == 3:
                        assert ib["reserved"][s, c, d] == k, (r, s, c, d)
                        assert np.array_equal(bb[s, d, k, :end], ba[s, c, d, :end]), (r, s, c, d)
                        k += 1
                        decoded += 1
                    else:
                        assert ib["reserved"][s, c, d] == 0xFF
                assert k <= pb.sf_slots
    assert decoded >= S * nd * 2
