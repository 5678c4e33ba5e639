#!/bin/bash
# GPU: ResNet step numerics tests (+ optional extra pytest args), then benches ($BENCHES).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread ${TESTS:-tests/test_gpu_resnet_step.py} > gpurun_out/pytest_t1.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_t1.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit 1; }
: > gpurun_out/bench.log
IFS=';' read -ra B <<< "$BENCHES"
for args in "${B[@]}"; do
  [ -z "$args" ] && continue
  timeout -k 10 300 python bench.py $args > gpurun_out/bench_one.log 2>&1
  rc=$?
  echo "ARGS: $args" >> gpurun_out/bench.log
  grep '"metric"' gpurun_out/bench_one.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d[\"value\"], d[\"ms_per_step\"], d[\"config\"].get(\"exploits_timed\"), d.get(\"exploit_ms_mean\"))" >> gpurun_out/bench.log
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/bench_one.log; echo "bench rc=$rc ($args)"; exit 1; fi
done
cat gpurun_out/bench.log
echo T1_OK
