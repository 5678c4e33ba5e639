#!/bin/bash
# GPU: numerics tests ($TESTS), benches ($BENCHES, gpu_quick format), stamps at pop 1 ($STAMP_ENV)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${TESTS:-tests/test_gpu_resnet_step.py} > gpurun_out/pytest_t2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_t2.log
[ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_t2.log; echo "pytest rc=$rc"; exit 1; }
bash tools/gpu_quick.sh || exit 1
if [ -n "$STAMPS" ]; then
  env $STAMP_ENV timeout -k 10 200 python tools/stamps.py run --pop 1 > gpurun_out/stamps.txt 2>&1 || { tail gpurun_out/stamps.txt; exit 1; }
  tail -6 gpurun_out/stamps.txt
fi
echo T2_OK
