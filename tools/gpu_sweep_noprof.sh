#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/sweep.log
while read -r cfg; do
  [ -z "$cfg" ] && continue
  line=$(env $cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 2>&1 | grep '"metric"')
  rc=$?
  echo "$cfg => $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/sweep.log
  if [ $rc -ne 0 ]; then echo "bench failed for $cfg"; exit 1; fi
done < "${SWEEP_FILE:-tools/sweep_configs.txt}"
if [ -n "$PROF_CFG" ]; then
  cd /tmp && env $PROF_CFG timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_sw -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --exploit_every 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_sw.log 2>&1 || exit 1
  mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof_sw && find /tmp/prof_sw -name "*kernel_stats*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof_sw/ \;
fi
