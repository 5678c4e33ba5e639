#!/bin/bash
# fp32 ImageNet HIP step: oracle tests, bf16 ImageNet regression check, fp32 bench -> gpurun_out/r5i32
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5i32
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_imagenet_f32.py > gpurun_out/r5i32/f32.log 2>&1
rc=$?; grep -E "worst|loss hip|PASS|FAIL|Error|error|passed|failed|rel " gpurun_out/r5i32/f32.log | tail -40; [ $rc -ne 0 ] && { tail -30 gpurun_out/r5i32/f32.log; exit 1; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py tests/test_gpu_f32.py tests/test_gpu_golden_hip.py > gpurun_out/r5i32/bf16.log 2>&1
rc=$?; echo "regression: $(tail -1 gpurun_out/r5i32/bf16.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r5i32/bf16.log; exit 1; }
timeout -k 10 400 python -u bench.py --model imagenet --dtype fp32 --batch 32 --steps 3 --warmup 1 > gpurun_out/r5i32/b.log 2>&1 || { tail -5 gpurun_out/r5i32/b.log; exit 1; }
echo "imagenet fp32: $(grep '^{' gpurun_out/r5i32/b.log)"
timeout -k 10 300 python -u bench.py --model imagenet --steps 10 --warmup 2 > gpurun_out/r5i32/b16.log 2>&1 || { tail -5 gpurun_out/r5i32/b16.log; exit 1; }
echo "imagenet bf16: $(grep '^{' gpurun_out/r5i32/b16.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")"
