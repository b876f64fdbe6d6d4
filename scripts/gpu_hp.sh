#!/bin/bash
# Half-plane bit-sliced encode: parity (both kernels) then C3 bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bitslice.py tests/test_gpu_parity.py -k "bs_ or bitsliced or c3_full or baseline_config_encode" -x -v --timeout 120 --timeout-method thread > gpurun_out/hp_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/hp_pytest.log; [ $rc -eq 0 ] || exit $rc
for K in 2 1; do
  RS_BS_KERNEL=$K timeout -k 10 120 python bench.py --no-cpu --steps 50 --warmup 10 > gpurun_out/hp_bench16_k$K.log 2>&1 || exit $?
  echo "kernel $K 16 stripes: $(python -c "import json,sys; d=json.loads(open('gpurun_out/hp_bench16_k$K.log').read().strip().splitlines()[-1]); print(d['roofline']['kernel_ms'], d['roofline']['frac'])")"
  RS_BS_KERNEL=$K timeout -k 10 120 python bench.py --no-cpu --steps 200 --warmup 20 --stripes 1 > gpurun_out/hp_bench1_k$K.log 2>&1 || exit $?
  echo "kernel $K 1 stripe: $(python -c "import json,sys; d=json.loads(open('gpurun_out/hp_bench1_k$K.log').read().strip().splitlines()[-1]); print(d['roofline']['kernel_ms'], d['roofline']['frac'])")"
done
