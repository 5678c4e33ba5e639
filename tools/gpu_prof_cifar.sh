#!/bin/bash
# Kernel traces of the headline step (pop 8) and of one member per GPU (pop 1) -> gpurun_out/p8, gpurun_out/p1;
# then: python tools/trace_gaps.py gpurun_out/p8/run_kernel_trace.csv ; python tools/kstats.py gpurun_out/p8/run_kernel_stats.csv 13
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/p8 gpurun_out/p1
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p8 -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --exploit_every 0 > "$GRAFT_REPO_ROOT/gpurun_out/p8.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/p8.log"; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p1 -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --pop 1 --steps 30 --warmup 5 --exploit_every 0 > "$GRAFT_REPO_ROOT/gpurun_out/p1.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/p1.log"; exit 1; }
find /tmp/p8 \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/p8/" \;
find /tmp/p1 \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/p1/" \;
echo PROF_OK
