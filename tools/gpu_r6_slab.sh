#!/bin/bash
# round 6: grid-strided slab_reduce_all (DTF_SLAB_X_BLOCKS) -- ResNet step numerics, then pop 8 / pop 1 A/B -> gpurun_out/r6s
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_resnet_step.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head -20; exit 1; }
for pop in 8 1; do
  for r in 1 2; do
    for x in 0 16 32; do
      DTF_SLAB_X_BLOCKS=$x timeout -k 10 200 python3 -u bench.py --pop $pop --steps 100 --warmup 20 > $O/b_${pop}_${x}_$r.log 2>&1 || { tail -5 $O/b_${pop}_${x}_$r.log; exit 1; }
      echo "pop $pop xblocks $x run $r: $(grep '^{' $O/b_${pop}_${x}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
    done
  done
done
exit 0
