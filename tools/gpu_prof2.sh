#!/bin/bash
# Kernel-trace two bench configurations ($PROF_A, $PROF_B) into gpurun_out/trace_a|b (stats + trace csv).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in a b; do
  var="PROF_${tag^^}"; args="${!var}"
  evar="PROF_ENV_${tag^^}"; envs="${!evar}"
  [ -z "$args" ] && continue
  rm -rf /tmp/prof_$tag
  cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py $args > $GRAFT_REPO_ROOT/gpurun_out/prof_$tag.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_$tag.log; echo "rocprof failed ($tag)"; exit 1; }
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/trace_$tag; mkdir -p $GRAFT_REPO_ROOT/gpurun_out/trace_$tag
  find /tmp/prof_$tag \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/trace_$tag/ \;
  grep '"metric"' $GRAFT_REPO_ROOT/gpurun_out/prof_$tag.log
done
echo PROF_OK
