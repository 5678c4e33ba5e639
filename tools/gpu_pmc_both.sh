set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
KRE="conv_" BARGS="--pop 1 --steps 2 --warmup 1 --exploit_every 0" bash tools/gpu_pmc_pop.sh || exit 1
mkdir -p gpurun_out/pmc_pop1 && mv gpurun_out/pmc/* gpurun_out/pmc_pop1/
KRE="convg_" BARGS="--model imagenet --steps 1 --warmup 1 --exploit_every 0" bash tools/gpu_pmc_pop.sh || exit 1
mkdir -p gpurun_out/pmc_imagenet && mv gpurun_out/pmc/* gpurun_out/pmc_imagenet/
echo PMC_DONE
