"""Same-box A/B of pipeline settings (not part of the product): generates bench.py's
workload once, then times K steps of a fresh pipeline per configuration, configs
interleaved over several repetitions (box-to-box variance is ~5 %, so A/B across
gpurun calls is not reliable).  A configuration is a set of environment variables read
at dabgpu_pipe_create (e.g. DABGPU_TB_DEFER, DABGPU_NO_SPECULATE).

  python tools/ab_pipe.py --configs "base:" "nodefer:DABGPU_TB_DEFER=0" [--reps 3 --steps 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sdr-j-dab_amd"))
import numpy as np  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", required=True, help="NAME:VAR=V,VAR=V")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--cfo", type=float, default=1300.0)
    ap.add_argument("--ensembles", type=int, default=0)
    a = ap.parse_args()
    import dabamd
    from dabamd.synth import Ensemble
    SUBCH, E_default, _ = bench.WORKLOADS[a.workload]
    E, F = a.ensembles or E_default, a.frames
    ens = Ensemble(F * (a.warmup + a.steps) + 2, subch=SUBCH, snr_db=30.0, cfo_hz=a.cfo)
    ctx = dabamd.Context(0)
    stride = ens.length
    diq = ctx.buf(E * 2 * stride * 4)
    t0 = time.time()
    for g0 in range(0, E, 8):
        n = min(8, E - g0)
        diq.upload_at(ens.generate_many(n, seed0=1000 + g0, threads=min(16, os.cpu_count() or 1)), g0 * 2 * stride * 4)
    print(f"generated {E} ensembles in {time.time() - t0:.1f}s", flush=True)
    subs = [dabamd.Subch(s[0], s[1], s[2], s[3], 0 if s[4] else 1, dabamd.SUBCH_DABPLUS if s[5] else 0)
            for s in SUBCH]
    dabplus = any(s[5] for s in SUBCH)
    cfgs = []
    for c in a.configs:
        name, _, vs = c.partition(":")
        env = dict(kv.split("=", 1) for kv in vs.split(",") if kv)
        cfgs.append((name, env))
    res = {n: [] for n, _ in cfgs}
    for rep in range(a.reps):
        for name, env in cfgs:
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            pipe = dabamd.Pipeline(ctx, E, F, subs)
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            pipe.acquire(diq, stride, [0] * E, [stride] * E)
            for i in range(a.warmup):
                pipe.run(diq, stride, [stride] * E, download=False)
                if dabplus:
                    pipe.dabplus(download=False)
            pipe.sync()
            t = time.perf_counter()
            for i in range(a.steps):
                pipe.run(diq, stride, [stride] * E, download=False)
                if dabplus:
                    pipe.dabplus(download=False)
            pipe.sync()
            ms = (time.perf_counter() - t) / a.steps * 1e3
            res[name].append(ms)
            print(f"rep {rep} {name}: {ms:.3f} ms/step", flush=True)
            pipe.close() if hasattr(pipe, "close") else None
            del pipe
    out = {n: {"median_ms": float(np.median(v)), "min_ms": float(min(v)), "all": v,
               "msym_per_s": E * F * 76 / float(np.median(v)) / 1e3} for n, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
