#!/bin/bash
# round 6: MX-1 wide-wgrad BN coefficients hoisted per thread (XCOL) -- ResNet-50 numerics (release, det replay),
# then an interleaved A/B against the previous library (DTF_LIB=libdtf_kernels_old.so) -> gpurun_out/r6x
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py tests/test_gpu_golden_hip.py > $O/pytest.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head; exit 1; }
DTF_DETERMINISTIC=1 timeout -k 10 300 python3 -u tools/det_check.py > $O/det.log 2>&1; rc=$?
grep -E "image 64|DET_" $O/det.log; [ $rc -ne 0 ] && exit 1
OLD=$GRAFT_REPO_ROOT/distributedtf_amd/ops/libdtf_kernels_old.so
for r in 1 2 3; do
  for f in old new; do
    if [ $f = old ]; then L=$OLD; else L=""; fi
    DTF_LIB=$L timeout -k 10 300 python3 -u bench.py --model imagenet --steps 10 --warmup 3 > $O/b_${f}_$r.log 2>&1 || { tail -5 $O/b_${f}_$r.log; exit 1; }
    echo "lib=$f run $r: $(grep '^{' $O/b_${f}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
  done
done
exit 0
