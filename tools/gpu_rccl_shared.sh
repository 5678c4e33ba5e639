#!/bin/bash
# RCCL on ONE GPU: 2 ranks share the device (DTF_SHARE_GPU=1 -> per-rank NCCL_HOSTID, socket transport).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DTF_RCCL_DUMP_S=100
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_rccl_shared.py > gpurun_out/pytest_rccl.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_rccl.log | head -20
exit $rc
