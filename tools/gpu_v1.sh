#!/bin/bash
# ResNet v1 CIFAR: oracle step tests (v1 rows), then pop-8 bench v1 vs v2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/v1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resnet_step.py -k "v1" > gpurun_out/v1/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/v1/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/v1/pytest.log | head; exit 1; }
for v in 1 2; do
  timeout -k 10 200 python -u bench.py --resnet_version $v --steps 100 --warmup 10 > gpurun_out/v1/bench_v$v.log 2>&1 || { tail -5 gpurun_out/v1/bench_v$v.log; exit 1; }
  echo "v$v: $(grep '^{' gpurun_out/v1/bench_v$v.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")"
done
