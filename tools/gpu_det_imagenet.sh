#!/bin/bash
# deterministic build: bitwise replay (tools/det_check.py, CIFAR / MNIST / ImageNet) + ImageNet fixed-point oracle test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/det
if [ "${SKIP_DET_CHECK:-0}" != "1" ]; then
DTF_DETERMINISTIC=1 timeout -k 10 300 python -u tools/det_check.py > gpurun_out/det/det_check.log 2>&1
rc=$?; cat gpurun_out/det/det_check.log | grep -v Warning | tail -12
[ $rc -ne 0 ] && exit 1
fi
DTF_DETERMINISTIC=1 timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_imagenet_step.py > gpurun_out/det/pytest.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert|loss rel|PASS|FAIL" gpurun_out/det/pytest.log | head -30
exit $rc
