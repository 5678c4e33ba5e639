#!/bin/bash
# round 6: conv1 read-once BN fold up to width 256 (default) -- ResNet-50 numerics (release, det replay),
# then an interleaved A/B against the fold1 width 128 (DTF_CG_FOLD1_MAXC) -> gpurun_out/r6x2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6x2
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py tests/test_gpu_golden_hip.py > $O/pytest.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head; exit 1; }
DTF_DETERMINISTIC=1 timeout -k 10 300 python3 -u tools/det_check.py > $O/det.log 2>&1; rc=$?
grep -E "image 64|DET_" $O/det.log; [ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for f in 128 256; do
    DTF_CG_FOLD1_MAXC=$f timeout -k 10 300 python3 -u bench.py --model imagenet --steps 10 --warmup 3 > $O/b_${f}_$r.log 2>&1 || { tail -5 $O/b_${f}_$r.log; exit 1; }
    echo "fold1_maxc=$f run $r: $(grep '^{' $O/b_${f}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
  done
done
exit 0
