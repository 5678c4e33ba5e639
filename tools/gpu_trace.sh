#!/bin/bash
# Kernel-trace one bench configuration (PROF_ARGS) and keep the per-dispatch trace + stats under gpurun_out/trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/bench.log
IFS=';' read -ra B <<< "$BENCHES"
for args in "${B[@]}"; do
  [ -z "$args" ] && continue
  timeout -k 10 300 python bench.py $args > gpurun_out/bench_one.log 2>&1
  rc=$?
  echo "ARGS: $args" >> gpurun_out/bench.log
  grep '"metric"' gpurun_out/bench_one.log >> gpurun_out/bench.log
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/bench_one.log; echo "bench rc=$rc ($args)"; exit 1; fi
done
cat gpurun_out/bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_t -o run -- python3 $GRAFT_REPO_ROOT/bench.py $PROF_ARGS > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; echo "rocprof failed"; exit 1; }
rm -rf $GRAFT_REPO_ROOT/gpurun_out/trace; mkdir -p $GRAFT_REPO_ROOT/gpurun_out/trace
find /tmp/prof_t -name "*kernel_stats*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/trace/ \;
find /tmp/prof_t -name "*kernel_trace*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/trace/ \;
ls -la $GRAFT_REPO_ROOT/gpurun_out/trace
echo SESSION_OK
