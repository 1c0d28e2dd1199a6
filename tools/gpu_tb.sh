#!/bin/bash
# traceback isolation variants timed by rocprofv3 on the Viterbi operator (tools/tb_bench.py)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/tb; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  DABGPU_LIB=$R/sdr-j-dab_amd/lib/variants/libdabgpu_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$v -o $v --output-format csv -- python3 $R/tools/tb_bench.py 55296 5 > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  echo "$v: $(grep -h 'k_traceback\|k_acs' $f | awk -F'","' '{printf "%s avg %.3f ms  ", substr($1,1,40), $4/1e6}')"
done
