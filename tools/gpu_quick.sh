#!/bin/bash
# Quick perf check: $BENCHES = ';'-separated "ENV=v ENV2=w|bench args" entries (env part optional), optional
# kernel-stats profile ($PROF_ARGS, env in $PROF_ENV).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/bench.log
IFS=';' read -ra B <<< "$BENCHES"
for entry in "${B[@]}"; do
  [ -z "$entry" ] && continue
  if [[ "$entry" == *"|"* ]]; then envs="${entry%%|*}"; args="${entry#*|}"; else envs=""; args="$entry"; fi
  env $envs timeout -k 10 300 python bench.py $args > gpurun_out/bench_one.log 2>&1
  rc=$?
  line=$(grep '"metric"' gpurun_out/bench_one.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], 'img/s', d['ms_per_step'], 'ms', 'exploits', d['config'].get('exploits_timed'), d.get('exploit_ms_mean'))" 2>/dev/null)
  echo "[$envs] $args => $line" >> gpurun_out/bench.log
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/bench_one.log; echo "bench rc=$rc ($entry)"; cat gpurun_out/bench.log; exit 1; fi
done
cat gpurun_out/bench.log
if [ -n "$PROF_ARGS" ]; then
  cd /tmp && env $PROF_ENV timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_s -o run -- python3 $GRAFT_REPO_ROOT/bench.py $PROF_ARGS > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; echo "rocprof failed"; exit 1; }
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof; mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof
  find /tmp/prof_s \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof/ \;
fi
echo QUICK_OK
