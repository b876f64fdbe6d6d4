#!/bin/bash
# Host code of the library (codec.cpp, gf_host.cpp, multi.cpp) under AddressSanitizer and
# UBSan, on the CPU: rebuild those two objects instrumented (device code stays
# as built: -fno-gpu-sanitize), link a test copy of the library, and run the
# CPU tests that drive the host paths (C-ABI validation, Split/Join, plans,
# schedule checks, bit-sliced table replays) against it.
set -e
cd "$(dirname "$0")/.."
D=/tmp/rs_asan; mkdir -p $D
B=reedsolomon16_amd/build
for f in gf_host codec multi; do
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC -fno-gpu-sanitize -fsanitize=address,undefined -fno-omit-frame-pointer -pthread \
    -I$B -c reedsolomon16_amd/csrc/$f.cpp -o $D/$f.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -fsanitize=address,undefined -fno-gpu-sanitize -o $D/librs_asan.so \
  $B/kernels.o $B/bitslice.o $B/bitslice_dec.o $D/gf_host.o $D/codec.o $D/multi.o -pthread
RT=$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.asan-x86_64.so)
ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  LD_PRELOAD=$RT RS_MI355X_LIB=$D/librs_asan.so python -m pytest tests/test_capi_cpu.py tests/test_bitslice_cpu.py tests/test_multi_cpu.py -q -x -p no:cacheprovider
