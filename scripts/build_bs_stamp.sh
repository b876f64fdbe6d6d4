#!/bin/bash
# Diagnostic build of the library with the bit-sliced kernel's phase stamps
# (-DRS_BS_STAMP=1) into build/bs_stamp/librs_mi355x.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
B=reedsolomon16_amd/build
OUT=build/bs_stamp
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DRS_BS_STAMP=1 -I$B -c reedsolomon16_amd/csrc/bitslice.hip -o $OUT/bitslice.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/librs_mi355x.so $B/kernels.o $OUT/bitslice.o $B/gf_host.o $B/codec.o
