#!/bin/bash
# Build a variant of libdabgpu.so with extra compile flags for A/B timing:
#   tools/build_variant.sh NAME "-DFLAG ..."  ->  sdr-j-dab_amd/lib/variants/libdabgpu_NAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
P=$ROOT/sdr-j-dab_amd
OUT=$P/build/variant_$1
mkdir -p "$OUT" "$P/lib/variants"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -w $2"
for f in k_ofdm.hip k_demod.hip k_viterbi.hip k_dabplus.hip dabgpu_host.cpp; do
    extra=""; [ "$f" = k_demod.hip ] && extra="${DEMOD_FLAGS--fno-slp-vectorize}"    # as the Makefile (env DEMOD_FLAGS: A/B)
    /opt/rocm/bin/hipcc $FLAGS $extra -x hip -c "$P/csrc/$f" -o "$OUT/$f.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$P/lib/variants/libdabgpu_$1.so" "$OUT"/*.o
echo "$P/lib/variants/libdabgpu_$1.so"
