#!/bin/bash
# round 6: vectorised BN-transform coefficient reads in the generic ResNet-50 conv (CG_XF_VEC) and the fold variants
# re-measured with it -> gpurun_out/r6x
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6x
mkdir -p $O
DTF_CG_FOLD=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py > $O/pytest_fold.log 2>&1
rc=$?; echo "full fold tests: $(tail -1 $O/pytest_fold.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest_fold.log | head; exit 1; }
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py > $O/pytest_default.log 2>&1
rc=$?; echo "default tests: $(tail -1 $O/pytest_default.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest_default.log | head; exit 1; }
L0=$GRAFT_REPO_ROOT/distributedtf_amd/ops/libdtf_kernels_xfvec0.so
b() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --model imagenet --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "$tag: $(grep '^{' $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for r in 1 2; do
  b "vec0_default_$r" DTF_LIB=$L0
  b "vec1_default_$r" X=1
  b "vec1_maxc256_$r" DTF_CG_FOLD1_MAXC=256
  b "vec1_fold2_$r" DTF_CG_FOLD2=1
  b "vec1_fullfold_$r" DTF_CG_FOLD=1
done
exit 0
