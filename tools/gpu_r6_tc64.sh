#!/bin/bash
# round 6: 64-channel output tiles for the small-image generic conv launches (DTF_CG_TC64_HW) -> gpurun_out/r6t
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6t
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --model imagenet --steps 10 --warmup 3 > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
DTF_CG_TC64_HW=14 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py > $O/pytest.log 2>&1
rc=$?; echo "tc64 tests: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head; exit 1; }
for r in 1 2; do
  run base_$r
  run hw7_$r DTF_CG_TC64_HW=7
  run hw14_$r DTF_CG_TC64_HW=14
done
exit 0
