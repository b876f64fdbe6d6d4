#!/bin/bash
# Lab builds of the C3 kernel k_encode_hp (bitslice.hip) with steps left out
# (wrong results; performance experiments only) into
# build/ablate_hp/<name>/librs_mi355x.so.  RS_HP_ABL bitmask: 1 the XOR
# networks (twiddle products, D), 2 the bit-plane transposes and half swaps,
# 4 the LDS exchanges (puts, gets, barriers).  The product source is copied
# and rewritten by scripts/lab/hp_lab.py; it carries no lab hooks itself.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
HIPCC=/opt/rocm/bin/hipcc
SRC=reedsolomon16_amd/csrc
B=reedsolomon16_amd/build
rm -rf build/ablate_hp; mkdir -p build/ablate_hp/src
cp $SRC/*.hip $SRC/*.hpp build/ablate_hp/src/
python3 scripts/lab/hp_lab.py build/ablate_hp/src/bitslice.hip
VARS=${VARIANTS:-"base:0 nonet:1 nonet_notr:3 memonly:7"}
for v in $VARS; do
  IFS=: read -r name abl <<< "$v"
  mkdir -p build/ablate_hp/$name
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$B -Ibuild/ablate_hp/src -DRS_HP_ABL=$abl -c build/ablate_hp/src/bitslice.hip -o build/ablate_hp/$name/bitslice.o &
done
wait
for v in $VARS; do
  name=${v%%:*}; d=build/ablate_hp/$name
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $d/librs_mi355x.so $B/kernels.o $d/bitslice.o $B/bitslice_dec.o $B/gf_host.o $B/codec.o
done
