#!/bin/bash
# round 6: BN folds re-measured with the hoisted MX-1 wide-wgrad coefficients -> gpurun_out/r6fx
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6fx
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --model imagenet --steps 10 --warmup 3 > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for r in 1 2; do
  run base_$r DTF_CG_FOLD1_MAXC=128
  run maxc256_$r DTF_CG_FOLD1_MAXC=256
  run maxc512_$r DTF_CG_FOLD1_MAXC=512
  run fold_all_$r DTF_CG_FOLD=1
done
exit 0
