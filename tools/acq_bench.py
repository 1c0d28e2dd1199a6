"""The null-symbol search alone (k_acquire through dabgpu_pipe_acquire, host-timed):
E streams from their first sample, clean or with an interferer over the first 1.5
frames (the bench's sync-loss case: two give-ups before the signal returns), at the
bench's 1300 Hz carrier offset.  DABGPU_LIB selects a library build (A/B).
  python tools/acq_bench.py [--ensembles 64] [--jam] [--reps 3]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sdr-j-dab_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ensembles", type=int, default=64)
    ap.add_argument("--jam", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import dabamd
    from dabamd.synth import Ensemble
    E = a.ensembles
    ens = Ensemble(6, subch=[(0, 96, 128, 3, 1, 0)], snr_db=30.0, cfo_hz=1300.0)
    iq = ens.generate_many(E, seed0=300, threads=16)
    if a.jam:
        n = 300000
        rng = np.random.default_rng(3)
        ph = 2 * np.pi * 100e3 / 2048000 * np.arange(n)
        v = iq.reshape(E, -1, 2)
        v[:, 1000:1000 + n, 0] = np.cos(ph) + rng.normal(0, 0.1, n)
        v[:, 1000:1000 + n, 1] = np.sin(ph) + rng.normal(0, 0.1, n)
    ctx = dabamd.Context(0)
    diq = ctx.put(iq)
    stride = iq.shape[1] // 2
    ts, wins = [], None
    for r in range(a.reps):
        pipe = dabamd.Pipeline(ctx, E, 1, [])
        pipe.sync()
        t0 = time.perf_counter()
        pipe.acquire(diq, stride, [0] * E, [stride] * E)
        pipe.sync()
        ts.append((time.perf_counter() - t0) * 1e3)
        wins = [pipe.state(s).next_pos for s in range(E)]
        pipe.close()
    print(f"acquire E={E} jam={a.jam}: ms {['%.2f' % t for t in ts]} windows {wins[:4]}", flush=True)


if __name__ == "__main__":
    main()
