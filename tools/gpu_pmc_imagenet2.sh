#!/bin/bash
# PMC groups (tools/gpu_pmc_pop.sh) for the ImageNet convg kernels; summary: python tools/pmc_summary.py gpurun_out/pmc/counters_*.csv
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
KRE="convg_" BARGS="--model imagenet --steps 1 --warmup 1 --exploit_every 0" bash tools/gpu_pmc_pop.sh
