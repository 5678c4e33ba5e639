#!/bin/bash
# fp32 HIP step: oracle tests + pop-8 fp32 bench (v2, v1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/f32
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_f32.py > gpurun_out/f32/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|rel |worst|passed|failed" gpurun_out/f32/pytest.log | head -40
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 20 --warmup 3 > gpurun_out/f32/bench.log 2>&1 && grep '^{' gpurun_out/f32/bench.log || exit 1
timeout -k 10 300 python -u bench.py --dtype fp32 --resnet_version 1 --steps 20 --warmup 3 > gpurun_out/f32/bench_v1.log 2>&1 && grep '^{' gpurun_out/f32/bench_v1.log || exit 1
bash tools/gpu_prof_f32.sh && python3 tools/kstats.py gpurun_out/pf32/run_kernel_stats.csv 9 | head -30
