#!/bin/bash
# GPU session 2: HIP ResNet step numerics, HIP-backend bench, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu2.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu2.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit 1; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_hip.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -2 gpurun_out/bench_hip.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_hip -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --exploit_every 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_hip.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_hip.log; exit 1; }
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof_hip && find /tmp/prof_hip -name "*stats*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof_hip/ \;
ls -la $GRAFT_REPO_ROOT/gpurun_out/prof_hip
