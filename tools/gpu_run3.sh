#!/bin/bash
# GPU session: numerics tests, then a bench sweep (SWEEP_FILE), then a rocprof kernel-stats run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu3.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu3.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_gpu3.log; echo "pytest rc=$rc"; exit 1; fi
bash tools/gpu_sweep_noprof.sh || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_hip -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --exploit_every 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_hip.log 2>&1 || { echo "rocprof failed"; exit 1; }
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_hip; mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof_hip && find /tmp/prof_hip -name "*kernel_stats*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof_hip/ \;
