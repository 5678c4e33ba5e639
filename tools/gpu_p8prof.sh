#!/bin/bash
# pop-N kernel stats of the bench step (default pop 8) -> gpurun_out/p8prof
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
POP=${POP:-8}
mkdir -p gpurun_out/p8prof
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p8prof -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --pop $POP --steps 30 --warmup 5 --exploit_every 0 > "$GRAFT_REPO_ROOT/gpurun_out/p8prof/prof.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/p8prof/prof.log"; exit 1; }
find /tmp/p8prof \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/p8prof/" \;
cd "$GRAFT_REPO_ROOT" && python3 tools/kstats.py gpurun_out/p8prof/run_kernel_stats.csv 35 > gpurun_out/p8prof/kstats.txt && head -30 gpurun_out/p8prof/kstats.txt
