#!/bin/bash
# ResNet-50 v1 (post-activation bottleneck) on the HIP ImageNet path: oracle step test + bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/in_v1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py > gpurun_out/in_v1/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|rel |passed|failed" gpurun_out/in_v1/pytest.log | head -40
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u bench.py --model imagenet --resnet_version 1 --steps 10 --warmup 3 > gpurun_out/in_v1/bench_v1.log 2>&1 && grep '^{' gpurun_out/in_v1/bench_v1.log
