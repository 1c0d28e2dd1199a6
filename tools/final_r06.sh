#!/bin/bash
# Round 6's final-tree evidence, in two gpurun calls:
#   tools/final_r06.sh OUT a   -m gpu suite, smoke(), the driver's bench command, a kernel trace
#   tools/final_r06.sh OUT b   HBM traffic passes (FETCH_SIZE, WRITE_SIZE -> rNN_traffic_c3.json
#                              via tools/pmc_traffic.py), the ACS clock / issue pass, and the
#                              N = 2 rehearsal on one GPU (gloo-staged, both legs)
set -o pipefail
O=$1; P=$2
R=${GRAFT_REPO_ROOT:-/root/repo}
case $P in
a)
    tools/gpu.sh $O tests tests -s &&
    tools/gpu.sh $O smoke &&
    tools/gpu.sh $O bench c3_driver_cmd --gpus 1 --steps 20 --warmup 5 &&
    tools/gpu.sh $O stats c3 --steps 20 --warmup 5 --no-cpu-baseline --solo-steps 0 --delivered-steps 0 \
        --sync-loss-steps 0 --c5-steps 0 ;;
b)
    BENCH_ARGS="--solo-steps 0 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0" \
        tools/pmc_passes.sh $O "FETCH_SIZE" "WRITE_SIZE" &&
    python3 tools/pmc_traffic.py $(find $R/gpurun_out/$O/p1 -name '*counter_collection.csv') \
        $(find $R/gpurun_out/$O/p2 -name '*counter_collection.csv') $R/gpurun_out/$O/traffic_c3.json &&
    tools/gpu.sh $O pmc clock "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU" \
        --c5-steps 0 &&
    python3 tools/acs_clock_issue.py $R/gpurun_out/$O/pmc_clock "k_acs2" > $R/gpurun_out/$O/acs_clock_issue.json &&
    timeout -k 10 600 python3 -u bench.py --gpus 2 --ensembles 16 --frames 8 --steps 4 --warmup 6 --fed-steps 4 \
        > $R/gpurun_out/$O/bench_local2_one_gpu.log 2>&1 ;;
*)
    echo "usage: tools/final_r06.sh OUT a|b"; exit 2 ;;
esac
