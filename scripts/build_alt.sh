#!/bin/bash
# A/B build of libmog_air.so: the product objects (make -C mog-asr_amd first)
# with ONE source recompiled under other flags, linked into build_alt/ (same
# source hash, so mog_air._lib accepts it through MOG_AIR_LIB).
# usage: scripts/build_alt.sh <csrc file stem> <extra / replaced hipcc flags...>
#   e.g. scripts/build_alt.sh vae_step -fslp-vectorize
set -e
cd "$(dirname "$0")/../mog-asr_amd"
stem=$1; shift
mkdir -p build_alt
cp build/*.o build_alt/
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" \
    -c csrc/$stem.hip -o build_alt/$stem.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-soname,libmog_air.so \
    -o build_alt/libmog_air.so build_alt/*.o
echo "built mog-asr_amd/build_alt/libmog_air.so ($stem: $*)"
