#!/bin/bash
# Build variants of the bit-sliced decoder (bitslice_dec.hip) into
# build/ablate_dec/<name>/librs_mi355x.so.  VARIANTS="name:abl[:flag,flag]":
# RS_DEC_ABL bits (steps left out, wrong results) and extra -D flags, e.g.
# "stamp:0:-DRS_DEC_STAMP".  Performance experiments only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
HIPCC=/opt/rocm/bin/hipcc
SRC=reedsolomon16_amd/csrc
B=reedsolomon16_amd/build
rm -rf build/ablate_dec; mkdir -p build/ablate_dec
VARS=${VARIANTS:-"base:0 load:1 p1:2 phase2:4 p3:8 reveal:16 scale:32 transp:64"}
for v in $VARS; do
  IFS=: read -r name abl flags <<< "$v"
  mkdir -p build/ablate_dec/$name
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$B -DRS_DEC_ABL=$abl ${flags//,/ } -c $SRC/bitslice_dec.hip -o build/ablate_dec/$name/bitslice_dec.o &
done
wait
for v in $VARS; do
  name=${v%%:*}; d=build/ablate_dec/$name
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $d/librs_mi355x.so $B/kernels.o $B/bitslice.o $d/bitslice_dec.o $B/bitslice_enc256.o $B/gf_host.o $B/codec.o
done
