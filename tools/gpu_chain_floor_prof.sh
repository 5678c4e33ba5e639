#!/bin/bash
# Kernel trace of tools/chain_floor.hip: per-dispatch durations vs the per-launch wall time it prints.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/cf
export TMPDIR=/tmp
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/cf -o run -- "$GRAFT_REPO_ROOT/tools/bin/chain_floor" > "$GRAFT_REPO_ROOT/gpurun_out/cf/out.txt" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/cf/out.txt"; exit 1; }
find /tmp/cf -name "*kernel_stats*" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/cf/" \;
find /tmp/cf -name "*kernel_trace*" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/cf/" \;
cat "$GRAFT_REPO_ROOT/gpurun_out/cf/out.txt" | grep us/launch
cat "$GRAFT_REPO_ROOT"/gpurun_out/cf/*kernel_stats*
