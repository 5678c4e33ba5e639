#!/bin/bash
# round 6: parity-class LPT order of the stride-2 3x3 data gradients (ResNet-50) -> gpurun_out/r6l
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6l
mkdir -p $O
DTF_CG_CLASS_LPT=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head; exit 1; }
for r in 1 2 3; do
  for f in 0 1; do
    DTF_CG_CLASS_LPT=$f timeout -k 10 300 python3 -u bench.py --model imagenet --steps 10 --warmup 3 > $O/b_${f}_$r.log 2>&1 || { tail -5 $O/b_${f}_$r.log; exit 1; }
    echo "lpt=$f run $r: $(grep '^{' $O/b_${f}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
  done
done
exit 0
