#!/bin/bash
# round 6: (1) conv_fwd_s1<16> staging coefficients in VGPRs: A/B against libdtf_kernels_old.so (pop 8, pop 1);
# (2) selective BN3 fold into conv3 (DTF_CG_FOLD3_MAXC): ResNet-50 numerics with every block folded, then a sweep
# -> gpurun_out/r6f3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_ab_lib.sh r6cr tests/test_gpu_resnet_step.py "--steps 100 --warmup 10" "--pop 1 --steps 200 --warmup 20" || exit 1
O=gpurun_out/r6f3
mkdir -p $O
DTF_CG_FOLD3_MAXC=2048 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py > $O/pytest.log 2>&1
rc=$?; echo "fold3 tests: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head; exit 1; }
for r in 1 2; do
  for f in 0 256 512 1024 2048; do
    DTF_CG_FOLD3_MAXC=$f timeout -k 10 300 python3 -u bench.py --model imagenet --steps 10 --warmup 3 > $O/b_${f}_$r.log 2>&1 || { tail -5 $O/b_${f}_$r.log; exit 1; }
    echo "fold3_maxc=$f run $r: $(grep '^{' $O/b_${f}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
  done
done
exit 0
