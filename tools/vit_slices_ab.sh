#!/bin/bash
# the MSC Viterbi in K slices (DABGPU_VIT_SLICES=K: slice i's traceback reads
# the decisions slice i's ACS has just written, <= 256 MB per slice at K >= 8 for C3) against
# the whole-batch launches (K = 1), interleaved on one box; every run's checked step compares
# ensemble 0's FIC and MSC with the transmitted bits.
#   tools/vit_slices_ab.sh OUT REPS K...
set -o pipefail
O=$1; REPS=$2; shift 2
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/$O
for r in $(seq 1 $REPS); do
  for k in "$@"; do
    DABGPU_VIT_SLICES=$k timeout -k 10 240 python3 bench.py --steps 12 --warmup 3 --no-cpu-baseline --solo-steps 0 \
        --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0 > $R/gpurun_out/$O/slices_${k}_$r.log 2>&1 \
        || { echo "K=$k failed"; tail -5 $R/gpurun_out/$O/slices_${k}_$r.log; exit 1; }
    grep '"value"' $R/gpurun_out/$O/slices_${k}_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_launch']; c=d['checked_step']
print('K=$k rep $r value %.4g M ms/step %.3f acs(+tb) %.3f demod %.3f msc %d/%d fic %s' % (d['value']/1e6, d['ms_per_step'], k['msc_acs'], k['demod'], c['msc_equal_transmitted'], c['msc_codewords'], c['fic_blocks_equal_transmitted']))" | tee -a $R/gpurun_out/$O/slices.txt
  done
done
