#!/bin/bash
# Quick correctness + perf check after a kernel change: ResNet step numerics tests, then the pop 8 / pop 1 benches.
# $TESTS (pytest -k expression, default resnet step), $BENCHES as in tools/gpu_quick.sh.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet_step.py ${XFLAG--x} -q --timeout 120 --timeout-method thread ${TESTS:+-k "$TESTS"} > gpurun_out/check_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/check_pytest.log
[ $rc -ne 0 ] && { tail -40 gpurun_out/check_pytest.log; echo "pytest rc=$rc"; exit 1; }
BENCHES="${BENCHES:---steps 60 --warmup 10;--pop 1 --steps 100 --warmup 20 --exploit_every 0}" bash tools/gpu_quick.sh
