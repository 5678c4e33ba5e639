#!/bin/bash
# One GPU session: targeted tests (TESTS), full GPU suite, bench lines (BENCHES, ';'-separated arg lists),
# optional rocprofv3 kernel-stats run (PROF_ARGS).  Every GPU step has its own time limit; stop at first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_targeted.log 2>&1
  rc=$?; tail -25 gpurun_out/pytest_targeted.log
  [ $rc -ne 0 ] && { echo "targeted tests rc=$rc"; exit 1; }
fi
if [ "$FULL" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; exit 1; }
fi
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
if [ -n "$PROF_ARGS" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_s -o run -- python3 $GRAFT_REPO_ROOT/bench.py $PROF_ARGS > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; echo "rocprof failed"; exit 1; }
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof; mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof && find /tmp/prof_s -name "*kernel_stats*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof/ \;
fi
echo SESSION_OK
