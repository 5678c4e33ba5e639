#!/bin/bash
# fp32 paths under the XCD-aware work order: numerics (fp32 tests) + bench A/B DTF_CG_XCD=2 (default) vs 0
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/f32x
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f32.py tests/test_gpu_imagenet_f32.py > gpurun_out/f32x/t.log 2>&1
rc=$?; echo "fp32 tests: $(tail -1 gpurun_out/f32x/t.log)"; [ $rc -ne 0 ] && { tail -20 gpurun_out/f32x/t.log; exit 1; }
: > gpurun_out/f32x/ab.log
for pass in 1 2; do
  for x in 2 0; do
    DTF_CG_XCD=$x timeout -k 10 300 python -u bench.py --dtype fp32 --steps 20 --warmup 3 > gpurun_out/f32x/b.log 2>&1 || { tail -5 gpurun_out/f32x/b.log; exit 1; }
    echo "[cifar fp32 XCD=$x]: $(grep '^{' gpurun_out/f32x/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/f32x/ab.log
    DTF_CG_XCD=$x timeout -k 10 300 python -u bench.py --model imagenet --dtype fp32 --steps 4 --warmup 1 > gpurun_out/f32x/b.log 2>&1 || { tail -5 gpurun_out/f32x/b.log; exit 1; }
    echo "[imagenet fp32 XCD=$x]: $(grep '^{' gpurun_out/f32x/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/f32x/ab.log
  done
done
