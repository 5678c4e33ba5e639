#!/bin/bash
# deterministic build: fp32 ImageNet / MNIST oracle tests + the full det_check replay -> gpurun_out/r5d32
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5d32
DTF_DETERMINISTIC=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagenet_f32.py tests/test_gpu_mnist_f32.py > gpurun_out/r5d32/det_tests.log 2>&1
rc=$?; echo "det build fp32 tests: $(tail -1 gpurun_out/r5d32/det_tests.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r5d32/det_tests.log; exit 1; }
DTF_DETERMINISTIC=1 timeout -k 10 600 python -u tools/det_check.py > gpurun_out/r5d32/det_check.log 2>&1
rc=$?; grep -v Warning gpurun_out/r5d32/det_check.log | tail -15; [ $rc -ne 0 ] && exit 1
DTF_HALF=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fp16.py > gpurun_out/r5d32/half.log 2>&1
rc=$?; echo "half build: $(tail -1 gpurun_out/r5d32/half.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r5d32/half.log; exit 1; }
exit 0
