#!/bin/bash
# round 5: elastic (ragged) plans with size-proportional work rows: elastic step tests + ragged / uniform benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5r
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resnet_step.py \
  -k "elastic or shrinking or ragged" > gpurun_out/r5r/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|Error" gpurun_out/r5r/pytest.log | head -20
[ $rc -ne 0 ] && { tail -60 gpurun_out/r5r/pytest.log; exit 1; }
for env in "DTF_ELASTIC_PROP=1" "DTF_ELASTIC_PROP=0" "DTF_ELASTIC_PROP=1" "DTF_ELASTIC_PROP=0"; do
  env $env timeout -k 10 300 python -u bench.py --ragged --steps 100 --warmup 10 > gpurun_out/r5r/one.log 2>&1 || { tail -30 gpurun_out/r5r/one.log; exit 1; }
  echo "$env ragged: $(grep '^{' gpurun_out/r5r/one.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s', d['config']['global_batch'])")" | tee -a gpurun_out/r5r/bench.log
done
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > gpurun_out/r5r/one.log 2>&1 || { tail -30 gpurun_out/r5r/one.log; exit 1; }
echo "uniform: $(grep '^{' gpurun_out/r5r/one.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/r5r/bench.log
