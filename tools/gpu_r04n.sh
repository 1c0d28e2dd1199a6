#!/bin/bash
# Round 4: packed-output parity at an odd row stride; C5 kernel stats (rocprofv3) and HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes) with packed MSC and the batched DAB+ loads.
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py -m gpu -x -q --timeout 200 --timeout-method thread -k "packed" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof5 -o c5 -- python3 $R/bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --solo-steps 0 --delivered-steps 0 --sync-loss-steps 0 > $R/$O/prof5.log 2>&1 || { tail -5 $R/$O/prof5.log; exit 1; }
f=$(find $R/$O/prof5 -name "*kernel_stats.csv" | head -1); cp "$f" $R/$O/c5_kernel_stats.csv; cut -c1-140 $R/$O/c5_kernel_stats.csv | head -14
BENCH_ARGS="--workload c5 --solo-steps 0 --delivered-steps 0 --sync-loss-steps 0" $R/tools/pmc_passes.sh r04n/pmc5 "FETCH_SIZE" "WRITE_SIZE" > $R/$O/pmc5.log 2>&1 || { tail -5 $R/$O/pmc5.log; exit 1; }
python3 $R/tools/pmc_traffic.py $(find $R/$O/pmc5/p1 -name '*counter_collection.csv') $(find $R/$O/pmc5/p2 -name '*counter_collection.csv') $R/$O/traffic_c5.json | grep -i "dp_\|acs\|traceback\|demod"
