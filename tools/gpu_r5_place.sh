#!/bin/bash
# placement invariance + resume (tests/test_gpu_placement.py) and the det-build CIFAR step test -> gpurun_out/r5pl
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5pl
timeout -k 10 1150 python -u -m pytest -x -v -s --timeout 1100 --timeout-method thread tests/test_gpu_placement.py > gpurun_out/r5pl/placement.log 2>&1
rc=$?; grep -E "passed|failed|world|Error|assert" gpurun_out/r5pl/placement.log | head -30
[ $rc -ne 0 ] && { tail -40 gpurun_out/r5pl/placement.log; exit 1; }
DTF_DETERMINISTIC=1 timeout -k 10 300 python -u tools/det_check.py > gpurun_out/r5pl/det_check.log 2>&1
rc=$?; grep -v Warning gpurun_out/r5pl/det_check.log | tail -12; exit $rc
