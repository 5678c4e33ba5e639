#!/bin/bash
# round 6 (late): C = 16 forward iterations per workgroup 8 / 16 -- pop 8, pop 4, ResNet-110 -> gpurun_out/r6s8
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s8
mkdir -p $O
run() {  # name, bench args, env...
  local n=$1 ba=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py $ba > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for r in 1 2; do
  run p8_base_$r "--steps 100 --warmup 10"
  run p8_it8_$r "--steps 100 --warmup 10" DTF_FWD_ITERS16=8
  run p8_it16_$r "--steps 100 --warmup 10" DTF_FWD_ITERS16=16
  run p4_base_$r "--pop 4 --steps 100 --warmup 10"
  run p4_it8_$r "--pop 4 --steps 100 --warmup 10" DTF_FWD_ITERS16=8
  run r110_base_$r "--resnet_size 110 --steps 50 --warmup 5"
  run r110_it8_$r "--resnet_size 110 --steps 50 --warmup 5" DTF_FWD_ITERS16=8
done
exit 0
