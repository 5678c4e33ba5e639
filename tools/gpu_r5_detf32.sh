#!/bin/bash
# deterministic fp32 CIFAR step: det_check (bitwise replay incl. fp32) + fp32 oracle tests in both builds -> gpurun_out/r5df
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5df
DTF_DETERMINISTIC=1 timeout -k 10 400 python -u tools/det_check.py > gpurun_out/r5df/det_check.log 2>&1
rc=$?; grep -v Warning gpurun_out/r5df/det_check.log | tail -12; [ $rc -ne 0 ] && exit 1
DTF_DETERMINISTIC=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py > gpurun_out/r5df/f32_det.log 2>&1
rc=$?; echo "det build fp32 tests: $(tail -1 gpurun_out/r5df/f32_det.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r5df/f32_det.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py tests/test_gpu_det_poison.py tests/test_gpu_resnet_step.py > gpurun_out/r5df/f32_rel.log 2>&1
rc=$?; echo "release build: $(tail -1 gpurun_out/r5df/f32_rel.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r5df/f32_rel.log; exit 1; }
for env in "" "DTF_DETERMINISTIC=1"; do
  env $env timeout -k 10 300 python -u bench.py --dtype fp32 --steps 20 --warmup 3 > gpurun_out/r5df/b.log 2>&1 || { tail -5 gpurun_out/r5df/b.log; exit 1; }
  echo "[$env] fp32 bench: $(grep '^{' gpurun_out/r5df/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")"
done
