#!/bin/bash
# round 6: trajectory (bf16-torch yardstick), world-8 bench rehearsal, placement at world 1/2/4/8 -> gpurun_out/r6t
# usage: gpu_r6_tests.sh [traj] [bench8] [place]   (default: all three)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6t
what="${*:-traj bench8 place}"
run() {  # name timeout pytest-args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u -m pytest -x -v -s --timeout "$((t - 30))" --timeout-method thread -p no:cacheprovider "$@" \
    > gpurun_out/r6t/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|PASSED|FAILED|world|Error|assert|window|eval acc|n_gpus" gpurun_out/r6t/$name.log | tail -40
  [ $rc -ne 0 ] && { tail -40 gpurun_out/r6t/$name.log; exit 1; }
  return 0
}
for w in $what; do
  case $w in
    traj) run traj 1000 tests/test_gpu_trajectory.py ;;
    bench8) run bench8 450 tests/test_gpu_rccl_shared.py -k eight ;;
    place) run place 1180 tests/test_gpu_placement.py ;;
  esac
done
exit 0
