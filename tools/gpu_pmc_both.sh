#!/bin/bash
# PMC of the committed kernels at pop 8 (headline, 1 GPU) and pop 1 (per-GPU work at 8 GPUs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
KRE="conv_|slab|head|bn_|weight_prep|fused_opt" BARGS="--steps 6 --warmup 2 --exploit_every 0" bash tools/gpu_pmc_pop.sh || exit 1
mkdir -p gpurun_out/pmc8 && mv gpurun_out/pmc/* gpurun_out/pmc8/
python3 tools/pmc_summary.py gpurun_out/pmc8/counters_*.csv > gpurun_out/pmc8/summary.txt
KRE="conv_|slab|head|bn_|weight_prep|fused_opt" BARGS="--steps 6 --warmup 2 --exploit_every 0 --pop 1" bash tools/gpu_pmc_pop.sh || exit 1
mkdir -p gpurun_out/pmc1 && mv gpurun_out/pmc/* gpurun_out/pmc1/
python3 tools/pmc_summary.py gpurun_out/pmc1/counters_*.csv > gpurun_out/pmc1/summary.txt
cat gpurun_out/pmc8/summary.txt gpurun_out/pmc1/summary.txt
