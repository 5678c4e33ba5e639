#!/bin/bash
# Round checkpoint on the GPU: full GPU test suite, smoke(), the headline bench + model-family benches, and a
# kernel-stats profile of the headline config.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; echo "smoke failed"; exit 1; }
tail -1 gpurun_out/smoke.log
: > gpurun_out/bench.log
IFS=';' read -ra B <<< "$BENCHES"
for args in "${B[@]}"; do
  [ -z "$args" ] && continue
  timeout -k 10 400 python bench.py $args > gpurun_out/bench_one.log 2>&1
  rc=$?
  echo "ARGS: $args" >> gpurun_out/bench.log
  grep '"metric"' gpurun_out/bench_one.log >> gpurun_out/bench.log
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/bench_one.log; echo "bench rc=$rc ($args)"; exit 1; fi
done
cat gpurun_out/bench.log
if [ -n "$PROF_ARGS" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_s -o run -- python3 $GRAFT_REPO_ROOT/bench.py $PROF_ARGS > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; echo "rocprof failed"; exit 1; }
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof; mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof
  find /tmp/prof_s \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof/ \;
fi
echo SESSION_OK
