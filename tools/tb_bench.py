"""Calibration (not part of the product): the Viterbi operator (dabgpu_viterbi: k_acs<0>
+ k_traceback<0>) on a C3-sized batch of mother-code codewords, REPS times, for
rocprofv3 --kernel-trace --stats timing of the traceback alone (DABGPU_LIB selects a
variant build).   python tools/tb_bench.py [N] [REPS]"""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sdr-j-dab_amd"))
import numpy as np
import dabamd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 55296
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nbits = 3072
ctx = dabamd.Context(0)
rng = np.random.default_rng(1)
soft = rng.integers(-127, 128, (n, 4 * (nbits + 6)), dtype=np.int16)
din, dout = ctx.put(soft), ctx.buf(n * nbits)
for _ in range(reps):
    rc = dabamd.lib().dabgpu_viterbi(ctx.h, din.ptr, n, nbits, dout.ptr)
    assert rc == 0, rc
ctx.check()
print(f"{reps} x dabgpu_viterbi: {n} codewords x {nbits + 6} steps")
