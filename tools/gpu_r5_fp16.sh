#!/bin/bash
# round 5: fp16 (half build) + deterministic poison tests, CIFAR step regression, fp16 / bf16 benches -> gpurun_out/r5a
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_fp16.py \
  tests/test_gpu_det_poison.py tests/test_gpu_resnet_step.py tests/test_gpu_optimizer.py > gpurun_out/r5a/pytest.log 2>&1
rc=$?; grep -E "passed|failed|PASS|FAIL|ARCH|update rel|LOSSES|Error" gpurun_out/r5a/pytest.log | head -40
[ $rc -ne 0 ] && { tail -60 gpurun_out/r5a/pytest.log; exit 1; }
for args in "--steps 100 --warmup 10" "--dtype fp16 --steps 100 --warmup 10" "--pop 1 --steps 200 --warmup 20" \
            "--model imagenet --dtype fp16 --steps 10 --warmup 3"; do
  timeout -k 10 300 python -u bench.py $args > gpurun_out/r5a/one.log 2>&1 || { tail -30 gpurun_out/r5a/one.log; exit 1; }
  echo "$args: $(grep '^{' gpurun_out/r5a/one.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s', d['dtype'])")" | tee -a gpurun_out/r5a/bench.log
done
