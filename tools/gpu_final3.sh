#!/bin/bash
# one GPU call for the round's record: gpu tests, the driver's bench command (C3 with the
# CPU baseline), the C5 bench (CPU baseline incl. RS codewords/s), a C3 rocprofv3
# kernel-stats profile and C3 PMC passes (HBM traffic, SQ issue/LDS counters, TA busy).
#   tools/gpu_final3.sh OUTNAME   ->  gpurun_out/OUTNAME/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c5 > $O/bench_c5.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt3 -o kt3 --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/kt3.log 2>&1 || exit 1
$R/tools/pmc_passes.sh $1/pmc3 "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
    "TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" > $O/pmc3.log 2>&1 || exit 1
echo done
