#!/bin/bash
# round 5: HIP golden blocks + placement invariance / resume + data tests -> gpurun_out/r5t
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5t
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_gpu_golden_hip.py tests/test_gpu_data.py > gpurun_out/r5t/golden.log 2>&1
rc=$?; grep -E "passed|failed|batch-size|Error" gpurun_out/r5t/golden.log | head -30
[ $rc -ne 0 ] && { tail -50 gpurun_out/r5t/golden.log; exit 1; }
timeout -k 10 1150 python -u -m pytest -x -v -s --timeout 1100 --timeout-method thread tests/test_gpu_placement.py > gpurun_out/r5t/placement.log 2>&1
rc=$?; grep -E "passed|failed|world|Error|assert" gpurun_out/r5t/placement.log | head -30
[ $rc -ne 0 ] && { tail -40 gpurun_out/r5t/placement.log; exit 1; }
exit 0
