"""Front-end kernel timing on the C3 batch (64 ensembles x 24 frames): the fused
findIndex + processToken kernel (dabgpu_ofdm_sync_demod), the demod alone with
explicit frames (dabgpu_ofdm_demod) and findIndex alone (dabgpu_prs_sync), each
timed with HIP events on the context stream (median of REPS launches).  HBM
fraction from the algorithmic bytes (8 T_s + 2 * 3072 per symbol, + 8 T_u of the
sync window).  DABGPU_LIB=path selects a library build (A/B of variants).

  python tools/demod_bench.py [--ensembles 64] [--frames 24] [--reps 10]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sdr-j-dab_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ensembles", type=int, default=64)
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--cfo", type=float, default=0.0)
    ap.add_argument("--phase", type=int, default=0, help="NCO phase step of every frame (!= 0: the per-sample NCO)")
    a = ap.parse_args()
    import dabamd
    from dabamd.synth import Ensemble
    E, F = a.ensembles, a.frames
    ens = Ensemble(F + 1, snr_db=30.0, cfo_hz=a.cfo)
    iq = ens.generate_many(E, seed0=77, threads=16)
    f0 = ens.generate(77, truth=False)["frame0"]
    stride = ens.length
    ctx = dabamd.Context(0)
    L = dabamd.lib()
    diq = ctx.put(iq)
    del iq
    frames = []
    for e in range(E):
        for k in range(F):
            b0 = f0 + k * 196608 + 2656 + 504
            frames.append(dabamd.Frame(iq_base=e * stride, n_samples=stride, window=b0 - 504, block0=b0,
                                       out_slot=len(frames), flags=0, lp_window=123457 if a.phase else 0,
                                       lp_data=654321 if a.phase else 0, phase_a=a.phase, phase_b=a.phase))
    n = len(frames)
    fa = (dabamd.Frame * n)(*frames)
    dfr = dabamd.DevBuf(ctx, C.sizeof(fa)).upload(np.frombuffer(fa, dtype=np.uint8))
    soft = ctx.buf(2 * n * 75 * 3072)
    si, snr, fc = ctx.buf(4 * n), ctx.buf(2 * n), ctx.buf(8 * n)
    sym_bytes = n * 75 * (8 * 2552 + 2 * 3072)
    res = {}

    fns = {
        "sync_demod": (lambda: L.dabgpu_ofdm_sync_demod(ctx.h, diq.ptr, dfr.ptr, n, 3, si.ptr, snr.ptr, soft.ptr,
                                                        None, fc.ptr), sym_bytes + n * 8 * 2048),
        "sync_demod_nosnr": (lambda: L.dabgpu_ofdm_sync_demod(ctx.h, diq.ptr, dfr.ptr, n, 3, si.ptr, None, soft.ptr,
                                                              None, fc.ptr), sym_bytes + n * 8 * 2048),
        "demod": (lambda: L.dabgpu_ofdm_demod(ctx.h, diq.ptr, dfr.ptr, n, soft.ptr, None, fc.ptr), sym_bytes),
        "prs_sync": (lambda: L.dabgpu_prs_sync(ctx.h, diq.ptr, dfr.ptr, n, 3, si.ptr, None, None), n * 8 * 2048),
    }
    # clocks up first (~0.5 s of back-to-back launches), then the variants interleaved
    t_end = time.time() + 0.5
    while time.time() < t_end:
        fns["demod"][0]()
        ctx.sync()
    ts = {k: [] for k in fns}
    for r in range(a.reps):
        for k, (fn, nb) in fns.items():
            L.dabgpu_event_record(ctx.h, 0)
            fn()
            L.dabgpu_event_record(ctx.h, 1)
            ms = C.c_float()
            L.dabgpu_event_elapsed(ctx.h, 0, 1, C.byref(ms))
            ts[k].append(ms.value)
    for k, (fn, nb) in fns.items():
        v = sorted(ts[k])
        med = v[len(v) // 2]
        res[k] = {"median_ms": med, "min_ms": v[0], "GBps": nb / med / 1e6, "frac_hbm": nb / med / 1e6 / 8000}
        print(k, json.dumps(res[k]), flush=True)
    s = si.download(np.int32, n)
    print("startIndex values:", np.unique(s)[:8], flush=True)
    ctx.check()
    print(json.dumps({"lib": dabamd.LIB_PATH, "frames": n, **res}))


if __name__ == "__main__":
    main()
