#!/bin/bash
# 32x32x16 MFMA tiles A/B (DTF_CG_M32) on the ImageNet ResNet-50 step: oracle test with M32 on, then alternating benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5m32
DTF_CG_M32=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py -k "224 or 64" > gpurun_out/r5m32/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5m32/pytest.log; [ $rc -ne 0 ] && { grep -E "assert|Error" gpurun_out/r5m32/pytest.log | head; tail -30 gpurun_out/r5m32/pytest.log; exit 1; }
for r in 1 2; do for m in 0 1; do
  DTF_CG_M32=$m timeout -k 10 300 python -u bench.py --model imagenet --steps 10 --warmup 3 > gpurun_out/r5m32/one.log 2>&1 || { tail -5 gpurun_out/r5m32/one.log; exit 1; }
  echo "M32=$m: $(grep '^{' gpurun_out/r5m32/one.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/r5m32/ab.log
done; done
