#!/bin/bash
# GPU: tests, then a bench sweep over tuning env vars (one process per config).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_sweep.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_sweep.log
if [ $rc -ne 0 ]; then tail -40 gpurun_out/pytest_gpu_sweep.log; exit 1; fi
: > gpurun_out/sweep.log
while read -r cfg; do
  [ -z "$cfg" ] && continue
  line=$(env $cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 2>&1 | grep '"metric"')
  rc=$?
  echo "$cfg => $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/sweep.log
  if [ $rc -ne 0 ]; then echo "bench failed for $cfg"; exit 1; fi
done < "${SWEEP_FILE:-tools/sweep_configs.txt}"
