#!/bin/bash
# trajectory test (tests/test_gpu_trajectory.py) twice with each library: default vs ops/libdtf_kernels_nosplit.so
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/traj
for r in 1 2; do
  for v in default nosplit; do
    L=""; [ $v = nosplit ] && L="$GRAFT_REPO_ROOT/distributedtf_amd/ops/libdtf_kernels_nosplit.so"
    DTF_LIB=$L timeout -k 10 300 python -u -m pytest -q -s --timeout 280 --timeout-method thread tests/test_gpu_trajectory.py > gpurun_out/traj/${v}_$r.log 2>&1
    echo "$v $r rc=$?: $(grep -o 'eval acc ref.*' gpurun_out/traj/${v}_$r.log | head -1)"
  done
done
