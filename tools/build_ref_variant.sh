#!/bin/bash
# Build libdabgpu.so from a git revision's kernel sources for same-box A/B timing:
#   tools/build_ref_variant.sh NAME [REV]  ->  sdr-j-dab_amd/lib/variants/libdabgpu_NAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=${2:-HEAD}
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" sdr-j-dab_amd/csrc include | tar -x -C "$TMP"
P=$TMP/sdr-j-dab_amd
mkdir -p "$P/build" "$ROOT/sdr-j-dab_amd/lib/variants"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -w"
for f in k_ofdm.hip k_demod.hip k_viterbi.hip k_dabplus.hip dabgpu_host.cpp; do
    extra=""; [ "$f" = k_demod.hip ] && extra="-fno-slp-vectorize"
    /opt/rocm/bin/hipcc $FLAGS $extra -x hip -c "$P/csrc/$f" -o "$P/build/$f.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/sdr-j-dab_amd/lib/variants/libdabgpu_$1.so" "$P"/build/*.o
rm -rf "$TMP"
echo "$ROOT/sdr-j-dab_amd/lib/variants/libdabgpu_$1.so"
