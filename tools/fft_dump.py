"""ANALYSIS TOOL: the fused demod's NCO-mixed FFT input and spectrum of 3 frames
(dabgpu_ofdm_demod_mix with the spectrum hook) saved to gpurun_out/<out>/fft_dump.npz, to
compare the GPU transform with tests/gpu_fft_emu.py on the CPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdr-j-dab_amd"), os.path.join(ROOT, "tests")]
import dabamd                                    # noqa: E402
from test_gpu_parity import _cfo_frames, _recorded   # noqa: E402

out = sys.argv[1]
ctx = dabamd.Context(0)
res = {}
for fmt, code in (("f32", None), ("s16", dabamd.IQ_S16)):
    g, x, frs = _cfo_frames(1300.0, amplitude=0.25)
    iq = ctx.put(g["iq"] if code is None else _recorded(g["iq"], code)[0])
    o = ctx.demod_mix(iq, frs, 1, fmt=code, with_spec=True)
    iq.free()
    res[f"{fmt}_mix"] = o[0][:, :8]
    res[f"{fmt}_spec"] = o[-1][:, :8].astype(np.complex64)
os.makedirs(os.path.join(ROOT, "gpurun_out", out), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", out, "fft_dump.npz"), **res)
print("saved", {k: v.shape for k, v in res.items()})
