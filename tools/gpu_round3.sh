#!/bin/bash
# one GPU call: gpu tests, the driver's bench command (C3, with the CPU baseline), the C5 bench
# (with its CPU baseline: RS codewords/s), a C5 kernel-stats profile and C5 PMC traffic
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c5 > $O/bench_c5.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt5 -o kt5 --output-format csv -- python3 $R/bench.py --workload c5 --no-cpu-baseline --steps 8 > $O/kt5.log 2>&1 || exit 1
BENCH_ARGS="--workload c5" $R/tools/pmc_passes.sh $1/pmc5 "FETCH_SIZE" "WRITE_SIZE" > $O/pmc5.log 2>&1 || exit 1
echo done
