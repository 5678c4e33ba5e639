#!/bin/bash
# round 6: table-free stride-1 1x1 wide weight gradients (convg_wgrad_wide P1) -- numerics (release, det replay),
# then an A/B against libdtf_kernels_old.so -> gpurun_out/$1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6p1}
mkdir -p $O
DTF_DETERMINISTIC=1 timeout -k 10 300 python3 -u tools/det_check.py > $O/det.log 2>&1; rc=$?
grep -E "image 64|DET_" $O/det.log; [ $rc -ne 0 ] && exit 1
bash tools/gpu_ab_lib.sh $1 "tests/test_gpu_imagenet_step.py tests/test_gpu_golden_hip.py" "--model imagenet --steps 10 --warmup 3"
