#!/bin/bash
# Diagnostic session: phase stamps at pop 1 (tools/abl/libdtf_stamp.so), kernel traces pop 8 / pop 1
# (tools/gpu_prof_cifar.sh), PMC passes of the pop 8 step (tools/gpu_pmc_pop.sh).  Each step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -f tools/abl/libdtf_stamp.so ]; then
  timeout -k 10 200 python tools/stamps.py run --pop 1 > gpurun_out/stamps_pop1.txt 2>&1 || { tail -20 gpurun_out/stamps_pop1.txt; exit 1; }
  tail -6 gpurun_out/stamps_pop1.txt
fi
bash tools/gpu_prof_cifar.sh || exit 1
python tools/trace_gaps.py gpurun_out/p8/run_kernel_trace.csv > gpurun_out/p8_breakdown.txt 2>&1
python tools/trace_gaps.py gpurun_out/p1/run_kernel_trace.csv > gpurun_out/p1_breakdown.txt 2>&1
head -4 gpurun_out/p8_breakdown.txt gpurun_out/p1_breakdown.txt
if [ -n "$PMC" ]; then
  BARGS="--steps 3 --warmup 2 --exploit_every 0" KRE="conv_|head_|dw_slab" bash tools/gpu_pmc_pop.sh || exit 1
  python tools/pmc_summary.py gpurun_out/pmc/counters_*.csv > gpurun_out/pmc_pop8.txt 2>&1
  head -30 gpurun_out/pmc_pop8.txt
fi
echo DIAG_OK
