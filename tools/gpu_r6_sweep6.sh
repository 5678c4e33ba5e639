#!/bin/bash
# round 6 (late): dgrad-role iterations per workgroup (DTF_DG_ITERS) at pop 8 / 4 -> gpurun_out/r6s6
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s6
mkdir -p $O
run() {  # name, bench args, env...
  local n=$1 ba=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py $ba > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for r in 1 2 3; do
  run p8_base_$r "--steps 100 --warmup 10"
  run p8_dg1_$r "--steps 100 --warmup 10" DTF_DG_ITERS=1
  run p8_dg4_$r "--steps 100 --warmup 10" DTF_DG_ITERS=4
done
for r in 1 2; do
  run p4_base_$r "--pop 4 --steps 100 --warmup 10"
  run p4_dg1_$r "--pop 4 --steps 100 --warmup 10" DTF_DG_ITERS=1
done
exit 0
