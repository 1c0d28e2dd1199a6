#!/bin/bash
# Round 6 final tree: frames per step (batch / latency trade-off) and the recorded formats, one box.
#   tools/r06_sweep.sh OUT
set -o pipefail
O=$1
A="--steps 12 --warmup 3 --no-cpu-baseline --solo-steps 0 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0"
for f in 12 24 32 48; do tools/gpu.sh $O bench frames$f $A --frames $f || exit $?; done
for fmt in u8 f32; do tools/gpu.sh $O bench fmt_$fmt $A --iq-format $fmt || exit $?; done
tools/gpu.sh $O bench c5 --workload c5 --steps 12 --warmup 3 --no-cpu-baseline --solo-steps 0 --sync-loss-steps 0
