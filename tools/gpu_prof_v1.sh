#!/bin/bash
# kernel trace of the ResNet-56 v1 step at pop 8 -> gpurun_out/pv1 (python tools/kstats.py gpurun_out/pv1/run_kernel_stats.csv 30)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pv1
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pv1 -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --resnet_version 1 --steps 10 --warmup 3 --exploit_every 0 > "$GRAFT_REPO_ROOT/gpurun_out/pv1.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/pv1.log"; exit 1; }
find /tmp/pv1 \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pv1/" \;
cd "$GRAFT_REPO_ROOT" && python3 tools/kstats.py gpurun_out/pv1/run_kernel_stats.csv 30 | head -60
