#!/bin/bash
# GPU session 1: kernel tests, torch-backend baseline bench, rocprof stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import torch; print(torch.__version__, torch.cuda.get_device_name(0))" > gpurun_out/env.txt 2>&1
rocm-smi --showtopo > gpurun_out/topo.txt 2>&1 || true
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --backend torch --steps 10 --warmup 3 > gpurun_out/bench_torch.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_torch.log; exit 1; }
tail -2 gpurun_out/bench_torch.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_torch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --backend torch --steps 3 --warmup 1 --exploit_every 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_torch.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_torch.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_torch -name "*stats*" | head
