#!/bin/bash
# round 6: dual (dgrad | wgrad roles in one launch) vs deferred weight gradients at pop 1 / 2 on the current
# kernels (DTF_SMALL_DEFER) -> gpurun_out/r6du
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6du
mkdir -p $O
DTF_SMALL_DEFER=0 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_resnet_step.py > $O/pytest.log 2>&1
rc=$?; echo "dual tests: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head; exit 1; }
run() {  # name, bench args, env...
  local n=$1 ba=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py $ba > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for r in 1 2; do
  run p1_defer_$r "--pop 1 --steps 200 --warmup 20"
  run p1_dual_$r "--pop 1 --steps 200 --warmup 20" DTF_SMALL_DEFER=0
  run p2_defer_$r "--pop 2 --steps 200 --warmup 20"
  run p2_dual_$r "--pop 2 --steps 200 --warmup 20" DTF_SMALL_DEFER=0
done
exit 0
