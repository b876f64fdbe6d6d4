#!/bin/bash
# Build variants of the engine library into build/ablate/<name>/librs_mi355x.so
# (performance experiments only).  VARIANTS="name:flags ..." overrides the set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
HIPCC=/opt/rocm/bin/hipcc
SRC=reedsolomon16_amd/csrc
rm -rf build/ablate
mkdir -p build/ablate/common
$HIPCC -O3 -std=c++17 -fPIC -c $SRC/gf_host.cpp -o build/ablate/common/gf_host.o &
$HIPCC -O3 -std=c++17 -fPIC -c $SRC/codec.cpp -o build/ablate/common/codec.o &
for v in ${VARIANTS:-base: nodma:-DRS_ABL_NO_DMA=1 nomul:-DRS_ABL_NO_MUL=1}; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
  out=build/ablate/$name; mkdir -p $out
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c $SRC/kernels.hip -o $out/kernels.o &
done
wait
for d in build/ablate/*/; do
  [ "$(basename $d)" = common ] && continue
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $d/librs_mi355x.so $d/kernels.o reedsolomon16_amd/build/bitslice.o reedsolomon16_amd/build/bitslice_dec.o build/ablate/common/gf_host.o build/ablate/common/codec.o
done
