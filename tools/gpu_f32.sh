#!/bin/bash
# fp32 HIP step: oracle tests + pop-8 fp32 bench; then a kernel trace of the bf16 pop-8 / pop-1 benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/f32
timeout -k 10 200 python tools/f32_diag.py 56 32 > gpurun_out/f32/diag.txt 2>&1 || { tail -5 gpurun_out/f32/diag.txt; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_f32.py > gpurun_out/f32/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|rel |worst|passed|failed" gpurun_out/f32/pytest.log | head -40
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 20 --warmup 3 > gpurun_out/f32/bench.log 2>&1 && grep '^{' gpurun_out/f32/bench.log || exit 1
timeout -k 10 300 python -u bench.py --dtype fp32 --resnet_version 1 --steps 20 --warmup 3 > gpurun_out/f32/bench_v1.log 2>&1 && grep '^{' gpurun_out/f32/bench_v1.log || exit 1
bash tools/gpu_prof_cifar.sh
timeout -k 10 120 ./tools/bin/chain_floor > gpurun_out/chain_floor.txt 2>&1; echo "chain_floor rc=$?"; cat gpurun_out/chain_floor.txt
