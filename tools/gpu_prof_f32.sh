#!/bin/bash
# Kernel statistics of the fp32 HIP step (bench --dtype fp32, pop 8) -> gpurun_out/pf32
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pf32
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf32 -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --dtype fp32 --steps 6 --warmup 2 --exploit_every 0 > "$GRAFT_REPO_ROOT/gpurun_out/pf32/bench.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/pf32/bench.log"; exit 1; }
find /tmp/pf32 \( -name "*kernel_stats*" \) -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/pf32/" \;
echo PROF_OK
