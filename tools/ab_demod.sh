#!/bin/bash
# A/B timing of demod variants (tools/build_variant.sh) with tools/demod_bench.py:
#   tools/ab_demod.sh "ARGS" NAME... (NAME "base" = sdr-j-dab_amd/lib/libdabgpu.so)
args=$1; shift
for n in "$@"; do
    if [ "$n" = base ]; then lib=""; else lib=sdr-j-dab_amd/lib/variants/libdabgpu_$n.so; fi
    echo -n "$n: "
    DABGPU_LIB=$lib timeout -k 10 120 python -u tools/demod_bench.py $args | tail -1 | \
        python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v["median_ms"], 4) for k, v in d.items() if isinstance(v, dict)})' || exit 1
done
