#!/bin/bash
# ImageNet folded forward (DTF_CG_FOLD): v2 step tests with the fold, then ResNet-50 pop 8 bench fold 0 / 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fold
DTF_CG_FOLD=1 timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py -k "not sizes3 and not sizes4 and not sizes5" > gpurun_out/fold/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/fold/pytest.log; [ $rc -ne 0 ] && { grep -E "assert|Error|member" gpurun_out/fold/pytest.log | head -20; exit 1; }
: > gpurun_out/fold/ab.log
for f in 0 1; do
  DTF_CG_FOLD=$f timeout -k 10 300 python -u bench.py --model imagenet --steps 10 --warmup 3 > gpurun_out/fold/bench_$f.log 2>&1 || { tail -5 gpurun_out/fold/bench_$f.log; exit 1; }
  echo "fold $f: $(grep '^{' gpurun_out/fold/bench_$f.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/fold/ab.log
done
