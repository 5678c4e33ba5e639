#!/bin/bash
# round 6: read-once BN1 fold (DTF_CG_FOLD1) -- ImageNet v2 step numerics with the fold, then ResNet-50 pop 8 A/B
# (alternating, two rounds) -> gpurun_out/r6f
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6f
mkdir -p $O
DTF_CG_FOLD1=1 timeout -k 10 400 python3 -u -m pytest -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py > $O/pytest_fold1.log 2>&1
rc=$?; tail -2 $O/pytest_fold1.log; [ $rc -ne 0 ] && { grep -E "assert|Error|member" $O/pytest_fold1.log | head -20; exit 1; }
for r in 1 2; do
  for f in 0 1; do
    DTF_CG_FOLD1=$f timeout -k 10 300 python3 -u bench.py --model imagenet --steps 10 --warmup 3 > $O/bench_${f}_$r.log 2>&1 || { tail -5 $O/bench_${f}_$r.log; exit 1; }
    echo "fold1=$f run $r: $(grep '^{' $O/bench_${f}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
  done
done
exit 0
