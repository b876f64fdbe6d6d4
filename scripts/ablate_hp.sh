#!/bin/bash
# Half-plane kernel ablations (performance experiments only; most variants
# compute wrong parity): one library per variant in build/ablate_hp/<name>/,
# C3 geometry only.  VARIANTS="name:-DFLAG,-DFLAG2 ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
HIPCC=/opt/rocm/bin/hipcc
SRC=reedsolomon16_amd/csrc
B=reedsolomon16_amd/build
OUT=build/ablate_hp
rm -rf $OUT; mkdir -p $OUT/common
$B/gen_bs_tables $OUT/common/bs_tables.h ${BS_CHUNKS:-4:12 5:6}
for v in ${VARIANTS:-base: nomul:-DRS_BS_ABL_NOMUL nolds:-DRS_BS_ABL_NOLDS noload:-DRS_BS_ABL_NOLOAD notrans:-DRS_BS_ABL_NOTRANS nostore:-DRS_BS_ABL_NOSTORE memonly:-DRS_BS_ABL_NOMUL,-DRS_BS_ABL_NOTRANS,-DRS_BS_ABL_NOLDS}; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
  mkdir -p $OUT/$name
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -I$OUT/common -c $SRC/bitslice.hip -o $OUT/$name/bitslice.o &
done
wait
for d in $OUT/*/; do
  [ "$(basename $d)" = common ] && continue
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $d/librs_mi355x.so $B/kernels.o $d/bitslice.o $B/bitslice_dec.o $B/gf_host.o $B/codec.o
done
