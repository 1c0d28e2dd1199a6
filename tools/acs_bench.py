"""Calibration (not part of the product): ACS cost per trellis step for the three
input paths of the Viterbi kernels, to separate the ACS itself from its tile loader.
Run under `rocprofv3 --kernel-trace --stats`; prints the work sizes so the per-step
cycles can be computed from the k_acs<KIND> durations:
  k_acs<0> mother code (contiguous, no depuncturing)   -- dabgpu_viterbi
  k_acs<1> UEP-3 128 kbit/s fragments (depuncturing)    -- dabgpu_msc_deconvolve
"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sdr-j-dab_amd"))
import numpy as np
import dabamd

ctx = dabamd.Context(0)
rng = np.random.default_rng(1)
n, nbits = 16384, 3072
soft = rng.integers(-127, 128, (n, 4 * (nbits + 6)), dtype=np.int16)
for _ in range(3):
    ctx.viterbi(soft, nbits)
print(f"k_acs<0>: {n} codewords x {nbits + 6} steps = {n // 2 * (nbits + 6)} wave-steps")
sub = dabamd.Subch(0, 96, 128, 3, 0, 0)   # UEP (uepFlag 0), protection level 3
frag = 96 * 64
frags = rng.integers(-127, 128, (n, frag), dtype=np.int16)
for _ in range(3):
    ctx.msc_deconvolve(frags, [sub] * n)
print(f"k_acs<1>: {n} codewords x {nbits + 6} steps = {n // 2 * (nbits + 6)} wave-steps")
