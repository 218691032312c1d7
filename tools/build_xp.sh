#!/bin/bash
# A/B build of the library with extra compile flags (CPU, from the repo root):
#   bash tools/build_xp.sh TAG "-DPM_SOMETHING=1 ..."  ->  halo2-aggregation_amd/lib_xp/libxp_TAG.so
set -e
TAG=$1; shift
FLAGS="$*"
D=halo2-aggregation_amd
B=/tmp/pm_xp_$TAG
mkdir -p $B $D/lib_xp
for S in capi inst_pallas inst_vesta inst_bn254; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function $FLAGS -c -o $B/$S.o $D/csrc/$S.hip &
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o $D/lib_xp/libxp_$TAG.so $B/*.o
ls -la $D/lib_xp/libxp_$TAG.so
