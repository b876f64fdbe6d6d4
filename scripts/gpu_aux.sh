#!/bin/bash
# Cache-policy A/B of the bit-sliced encode (build/ablate_hp/*), twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_ablate_hp.sh && cp gpurun_out/ablate_hp.log gpurun_out/ablate_hp_1.log && bash scripts/gpu_ablate_hp.sh
