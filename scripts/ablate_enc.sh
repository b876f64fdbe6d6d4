#!/bin/bash
# Lab builds of k_enc_lds with the 64-byte-tile (F16<2>) variant compiled for
# N workgroups per CU (__launch_bounds__(256, N)) into
# build/ablate_enc/w<N>/librs_mi355x.so; time them with RS_UNIT_WIDTH=narrow
# (scripts/gpu_r4w.sh).  Performance experiments only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
HIPCC=/opt/rocm/bin/hipcc
SRC=reedsolomon16_amd/csrc
B=reedsolomon16_amd/build
rm -rf build/ablate_enc; mkdir -p build/ablate_enc/src
cp $SRC/*.hip $SRC/*.hpp build/ablate_enc/src/
python3 - <<'PY'
p = "build/ablate_enc/src/kernels.hip"
s = open(p).read()
old = "__global__ void __launch_bounds__(256, 4) k_enc_lds(EncodeArgs a) {"
assert old in s
s = s.replace(old, "__global__ void __launch_bounds__(256, F::W == 2 ? RS_ENC_NARROW_WGS : 4) k_enc_lds(EncodeArgs a) {")
open(p, "w").write(s)
PY
for n in ${WGS:-4 5 6 8}; do
  mkdir -p build/ablate_enc/w$n
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$B -Ibuild/ablate_enc/src -DRS_ENC_NARROW_WGS=$n -c build/ablate_enc/src/kernels.hip -o build/ablate_enc/w$n/kernels.o -Rpass-analysis=kernel-resource-usage 2> build/ablate_enc/w$n/res.txt &
done
wait
for n in ${WGS:-4 5 6 8}; do
  d=build/ablate_enc/w$n
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $d/librs_mi355x.so $d/kernels.o $B/bitslice.o $B/bitslice_dec.o $B/gf_host.o $B/codec.o
  echo "w$n: $(grep -A8 'k_enc_ldsINS0_3F16ILi2EEELi8ELb0ENS0_4F16SILi2EEELb1E' $d/res.txt | grep -E 'VGPRs:|ScratchSize|Occupancy' | sed 's/.*remark: *//' | tr '\n' ' ')"
done
