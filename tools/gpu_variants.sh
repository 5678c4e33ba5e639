#!/bin/bash
# Targeted tests, then bench variants: VARIANTS="pop|ENV=1 ENV2=x;pop|..." (env-only A/B of one build), then an
# optional kernel trace of PROF_ARGS.  Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -v -s --timeout 150 --timeout-method thread > gpurun_out/pytest_targeted.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_targeted.log | tail -15
  [ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_targeted.log; echo "targeted tests rc=$rc"; exit 1; }
fi
: > gpurun_out/bench.log
IFS=';' read -ra V <<< "$VARIANTS"
for v in "${V[@]}"; do
  [ -z "$v" ] && continue
  pop="${v%%|*}"; envs="${v#*|}"; [ "$envs" = "$v" ] && envs=""
  timeout -k 10 200 env $envs python bench.py --pop $pop --steps ${STEPS:-40} --warmup 5 ${BARGS} > gpurun_out/bench_one.log 2>&1
  rc=$?
  echo "pop=$pop [$envs] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_one.log) $(grep -o '"value": [0-9.]*' gpurun_out/bench_one.log)" | tee -a gpurun_out/bench.log
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/bench_one.log; echo "bench rc=$rc"; exit 1; fi
done
if [ -n "$PROF_ARGS" ]; then
  [ -n "${PROF_ENV:-}" ] && export $PROF_ENV
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_s -o run -- python3 $GRAFT_REPO_ROOT/bench.py $PROF_ARGS > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; echo "rocprof failed"; exit 1; }
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof; mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof
  find /tmp/prof_s \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof/ \;
fi
echo SESSION_OK
