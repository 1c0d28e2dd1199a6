"""Time k_acquire (one wave per stream) on a null search that starts inside a 300,000-sample
interferer (the dropout of test_pipeline_dropout_reacquires_like_reference): the reference's
search runs ~1 M samples there.  Prints ms per launch and ns per searched sample."""
import sys, time, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sdr-j-dab_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dabamd
from dabamd.synth import Ensemble
import oracle_py as orc

e = Ensemble(16, subch=[(0, 96, 128, 3, 1, 0)], snr_db=20.0)
g = e.generate(51, truth=False)
iq = g["iq"].reshape(-1, 2).copy()
a = g["frame0"] + 3 * 196608 + 40000
b = a + 300000
level = float(np.sqrt((iq[:200000] ** 2).sum(1).mean()))
ph = 2 * np.pi * 100e3 / 2048000 * np.arange(b - a)
rng = np.random.default_rng(5)
iq[a:b, 0] = level * np.cos(ph) + rng.normal(0, level / 10, b - a)
iq[a:b, 1] = level * np.sin(ph) + rng.normal(0, level / 10, b - a)
x = np.ascontiguousarray(iq.reshape(-1))
ctx = dabamd.Context(0)
for off in (-100000, 150000):
    st = a + off
    seg = np.ascontiguousarray(x[2 * st:])
    n = len(seg) // 2
    found, att, ns, pos = orc.null_scan(seg, n, False)
    for S in (1, 64):
        d = ctx.put(np.tile(seg, S))
        ts = []
        for rep in range(3):                       # a fresh pipeline each time: the search starts over
            pipe = dabamd.Pipeline(ctx, S, 1, [])
            pipe.sync()
            t0 = time.perf_counter()
            pipe.acquire(d, n, [0] * S, [n] * S)
            pipe.sync()
            ts.append(time.perf_counter() - t0)
            st0 = pipe.state(0)
            pipe.close()
        d.free()
        t = min(ts)
        print(f"start {off:+d} S={S}: {t * 1e3:.2f} ms, searched {pos} samples (oracle), "
              f"{t / pos * 1e9:.1f} ns/sample; next_pos {st0.next_pos} == {pos}: {st0.next_pos == pos}", flush=True)
ctx.close()
