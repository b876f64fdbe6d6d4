#!/bin/bash
# Build variants of the bit-sliced decoder (bitslice_dec.hip with RS_DEC_ABL
# bits: steps left out, wrong results) into build/ablate_dec/<name>/librs_mi355x.so.
# Performance experiments only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
HIPCC=/opt/rocm/bin/hipcc
SRC=reedsolomon16_amd/csrc
B=reedsolomon16_amd/build
rm -rf build/ablate_dec; mkdir -p build/ablate_dec
VARS=${VARIANTS:-"base:0 load:1 ifft0:2 planes:4 iffta:8 phase2:16 ffta:32 bytes:64 fft0:128 reveal:256 phase1:512 phase3:1024 p1p3:1536"}
for v in $VARS; do
  name=${v%%:*}; abl=${v#*:}
  mkdir -p build/ablate_dec/$name
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$B -DRS_DEC_ABL=$abl -c $SRC/bitslice_dec.hip -o build/ablate_dec/$name/bitslice_dec.o &
done
wait
for v in $VARS; do
  name=${v%%:*}; d=build/ablate_dec/$name
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $d/librs_mi355x.so $B/kernels.o $B/bitslice.o $d/bitslice_dec.o $B/gf_host.o $B/codec.o
done
