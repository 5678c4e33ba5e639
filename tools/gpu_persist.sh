#!/bin/bash
# persistent forward segments (hip_resnet PERSIST_FWD): numerics tests per fence variant, then pop 1 / pop 2 bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ps
: > gpurun_out/ps/ab.log
for fence in ${FENCES:-0}; do
DTF_PERSIST_FENCE=$fence timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_resnet_step.py -k "persistent or benchmark_shapes" > gpurun_out/ps/pytest_$fence.log 2>&1
rc=$?; echo "fence $fence tests: $(tail -1 gpurun_out/ps/pytest_$fence.log)" | tee -a gpurun_out/ps/ab.log; [ $rc -ne 0 ] && { grep -E "assert|Error" gpurun_out/ps/pytest_$fence.log | head; exit 1; }
done
for pop in 1 2; do
for v in "0 0" "1 0"; do
  set -- $v
  DTF_PERSIST_FWD=$1 DTF_PERSIST_FENCE=$2 timeout -k 10 200 python -u bench.py --pop $pop --steps 300 --warmup 20 --exploit_every 0 > gpurun_out/ps/b.log 2>&1 || { tail -5 gpurun_out/ps/b.log; exit 1; }
  echo "pop $pop persist $1 fence $2: $(grep '^{' gpurun_out/ps/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s', d['config'].get('step_graph'), 'barrier failures', d['config'].get('persist_barrier_failures'))")" | tee -a gpurun_out/ps/ab.log
done
done
