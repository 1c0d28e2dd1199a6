"""TEST INFRASTRUCTURE: the stream on which ofdmProcessor::run's null search locks onto the
frame period after a sync loss (found by bench.py's four-rank rehearsal),
and a restatement of that search (ofdm-processor.cpp:272-327) that reports every attempt.

The stream: bench.py's C3 ensemble for rank 3 of a 4-rank run with 8 ensembles and 8
frames per step -- stream 1 (synthetic seed 1025), cyclic with a 16-frame period, 353 frames
long, stored as .sdr PCM16 -- with the sync_loss leg's interferer (a +100 kHz carrier plus
noise over 300,000 samples) from sample 45,015,888, in the data symbols of the frame whose
window starts at 44,975,888."""
import numpy as np

TF, TS, TNULL = 196608, 2552, 2656
C3_SUBCH = [(96 * i, 96, 128, 3, 1, 0) for i in range(9)]
FRAMES, PERIOD, SEED = 353, 16, 1025
JAM_AT, JAM_N = 45_015_888, 300_000
LAST_WINDOW = 44_975_888                 # the jammed frame: the last one decoded


def jam(n=JAM_N, amplitude=0.25):
    """the sync_loss leg's interferer as PCM16 (bench.py sync_loss_leg)"""
    rng = np.random.default_rng(11)
    ph = 2 * np.pi * 100e3 / 2048000 * np.arange(n)
    j = np.empty((n, 2), np.float32)
    j[:, 0] = amplitude * (np.cos(ph) + rng.normal(0, 0.1, n))
    j[:, 1] = amplitude * (np.sin(ph) + rng.normal(0, 0.1, n))
    return np.clip(np.rint(j.reshape(-1) * 32768.0), -32768, 32767).astype(np.int16)


def stream():
    """(PCM16 samples [2 n], the same as cf32 x / 32768)"""
    from dabamd.synth import Ensemble
    ens = Ensemble(FRAMES, subch=C3_SUBCH, snr_db=30.0, cfo_hz=1300.0, amplitude=0.25)
    per = ens.period_many(1, seed0=SEED, period=PERIOD, threads=8)[0]
    r = np.clip(np.rint(per * 32768.0), -32768, 32767).astype(np.int16)
    raw = np.zeros(2 * ens.length, np.int16)
    for p, q, m in ens.stream_pieces(PERIOD):
        raw[2 * p:2 * (p + m)] = r[2 * q:2 * (q + m)]
    raw[2 * JAM_AT:2 * (JAM_AT + JAM_N)] = jam()
    return raw, raw.astype(np.float32) / 32768.0


def trace_null_search(x, start, attempts):
    """notSynced -> SyncOnNull -> SyncOnEndNull from sample `start` of cf32 x (no NCO:
    coarse + fine = 0), `attempts` times or until the end of a null is found.  Returns
    [(dip position or None, end position or None, sLevel at the dip)]."""
    z = x.reshape(-1, 2).astype(np.float64)
    out, pos, sl = [], start, 0.0
    n = len(z)

    def ja(i):
        return abs(z[i, 0]) + abs(z[i, 1])
    for _ in range(attempts):
        sl = 0.0
        for i in range(pos, pos + 20 * TS):
            sl = 0.00001 * ja(i) + (1 - 0.00001) * sl
        pos += 20 * TS
        env = [ja(i) for i in range(pos, pos + 50)]
        for i in range(pos, pos + 50):
            sl = 0.00001 * ja(i) + (1 - 0.00001) * sl
        cur, pos, c, dip = sum(env), pos + 50, 0, None
        while pos < n:
            v = ja(pos)
            sl = 0.00001 * v + (1 - 0.00001) * sl
            cur += v - env[-50]
            env.append(v)
            pos += 1
            c += 1
            if not cur / 50 > 0.40 * sl:
                dip = pos
                break
            if c > TF:
                break
        if dip is None:
            out.append((None, None, sl))
            continue
        c, end, sl_dip = 0, None, sl
        while pos < n:
            v = float(np.hypot(z[pos, 0], z[pos, 1]))
            sl = 0.00001 * ja(pos) + (1 - 0.00001) * sl
            cur += v - env[-50]
            env.append(v)
            pos += 1
            c += 1
            if not cur / 50 < 0.75 * sl:
                end = pos
                break
            if c > TNULL + 50:
                break
        out.append((dip, end, sl_dip))
        if end is not None:
            break
    return out
