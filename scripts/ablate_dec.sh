#!/bin/bash
# Lab builds of the bit-sliced decoder (bitslice_dec.hip) into
# build/ablate_dec/<name>/librs_mi355x.so.  The product source carries no
# lab hooks: scripts/lab/bitslice_dec_lab.patch adds them to a copy
# (RS_DEC_ABL: bitmask of steps left out, wrong results -- 1 row loads,
# 2 phase-1 transform, 4 phase 2, 8 phase-3 transform, 16 reveal, 32 scale-in,
# 64 transposes; RS_DEC_STAMP: per-wave s_memtime segment sums printed by the
# launcher; RS_DEC_WAVES: waves per workgroup).
# VARIANTS="name:abl[:flag,flag]", e.g. "stamp:0:-DRS_DEC_STAMP".  Performance
# experiments only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
HIPCC=/opt/rocm/bin/hipcc
SRC=reedsolomon16_amd/csrc
B=reedsolomon16_amd/build
rm -rf build/ablate_dec; mkdir -p build/ablate_dec/src
cp $SRC/*.hip $SRC/*.hpp build/ablate_dec/src/
patch -s build/ablate_dec/src/bitslice_dec.hip scripts/lab/bitslice_dec_lab.patch
VARS=${VARIANTS:-"base:0 load:1 p1:2 phase2:4 p3:8 reveal:16 scale:32 transp:64"}
for v in $VARS; do
  IFS=: read -r name abl flags <<< "$v"
  mkdir -p build/ablate_dec/$name
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$B -Ibuild/ablate_dec/src -DRS_DEC_ABL=$abl ${flags//,/ } -c build/ablate_dec/src/bitslice_dec.hip -o build/ablate_dec/$name/bitslice_dec.o &
done
wait
for v in $VARS; do
  name=${v%%:*}; d=build/ablate_dec/$name
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $d/librs_mi355x.so $B/kernels.o $B/bitslice.o $d/bitslice_dec.o $B/gf_host.o $B/codec.o
done
