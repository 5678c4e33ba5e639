#!/bin/bash
# fp32 MNIST HIP step: oracle tests (release + det builds), det replay, MNIST fp32 bench -> gpurun_out/r5m
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5m
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_mnist_f32.py tests/test_gpu_mnist_step.py > gpurun_out/r5m/rel.log 2>&1
rc=$?; grep -E "rel err|PASS|FAIL|Error|passed|failed" gpurun_out/r5m/rel.log | tail -40; [ $rc -ne 0 ] && { tail -40 gpurun_out/r5m/rel.log; exit 1; }
DTF_DETERMINISTIC=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mnist_f32.py > gpurun_out/r5m/det.log 2>&1
rc=$?; echo "det build: $(tail -1 gpurun_out/r5m/det.log)"; [ $rc -ne 0 ] && { tail -40 gpurun_out/r5m/det.log; exit 1; }
DTF_DETERMINISTIC=1 timeout -k 10 500 python -u tools/det_check.py > gpurun_out/r5m/det_check.log 2>&1
rc=$?; grep -v Warning gpurun_out/r5m/det_check.log | tail -13; [ $rc -ne 0 ] && exit 1
for dt in bf16 fp32; do
  timeout -k 10 300 python -u bench.py --model mnist --dtype $dt --steps 50 --warmup 5 > gpurun_out/r5m/b_$dt.log 2>&1 || { tail -5 gpurun_out/r5m/b_$dt.log; exit 1; }
  echo "mnist $dt: $(grep '^{' gpurun_out/r5m/b_$dt.log)"
done
