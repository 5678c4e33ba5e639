#!/bin/bash
# round 6: block-input gradient applied by the previous block's conv3 data gradient (convg MODE 3,
# DTF_CG_GFOLD_MAXF) -- ResNet-50 numerics (release at 64 / 128, det replay), then an interleaved A/B -> gpurun_out/r6g
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6g
mkdir -p $O
for f in 64 128; do
  DTF_CG_GFOLD_MAXF=$f timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py > $O/pytest_$f.log 2>&1
  rc=$?; echo "gfold $f tests: $(tail -1 $O/pytest_$f.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest_$f.log | head; exit 1; }
done
DTF_DETERMINISTIC=1 timeout -k 10 300 python3 -u tools/det_check.py > $O/det.log 2>&1; rc=$?
grep -E "image 64|DET_" $O/det.log; [ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for f in 0 64 128; do
    DTF_CG_GFOLD_MAXF=$f timeout -k 10 300 python3 -u bench.py --model imagenet --steps 10 --warmup 3 > $O/b_${f}_$r.log 2>&1 || { tail -5 $O/b_${f}_$r.log; exit 1; }
    echo "gfold_maxf=$f run $r: $(grep '^{' $O/b_${f}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
  done
done
exit 0
