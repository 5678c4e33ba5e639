#!/bin/bash
# round 6: deferred wgrad jobs with fp32 atomics instead of dW slabs (DTF_DEFER_ATOMIC) -> gpurun_out/r6a
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6a
mkdir -p $O
DTF_DEFER_ATOMIC=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_resnet_step.py > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head; exit 1; }
for r in 1 2; do
  for pop in 8 1 2 4; do
    for f in 0 1; do
      st=$([ $pop = 8 ] && echo 100 || echo 200)
      DTF_DEFER_ATOMIC=$f timeout -k 10 200 python3 -u bench.py --pop $pop --steps $st --warmup 20 > $O/b_${pop}_${f}_$r.log 2>&1 || { tail -5 $O/b_${pop}_${f}_$r.log; exit 1; }
      echo "pop $pop atomic=$f run $r: $(grep '^{' $O/b_${pop}_${f}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
    done
  done
done
exit 0
