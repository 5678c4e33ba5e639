#!/bin/bash
# round 6 (late): forward iterations per workgroup and the C = 16 fused-backward workgroup cap re-swept on the
# register-coefficient kernels -> gpurun_out/r6s2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s2
mkdir -p $O
run() {  # name, bench args, env...
  local n=$1 ba=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py $ba > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
P8="--steps 100 --warmup 10"
P1="--pop 1 --steps 200 --warmup 20"
for r in 1 2; do
  run p8_base_$r "$P8"
  run p8_it3_$r "$P8" DTF_FWD_ITERS=3
  run p8_it6_$r "$P8" DTF_FWD_ITERS=6
  run p8_f16_384_$r "$P8" DTF_FUSED_TOTAL16=384
  run p8_f16_768_$r "$P8" DTF_FUSED_TOTAL16=768
  run p1_base_$r "$P1"
  run p1_it2_$r "$P1" DTF_FWD_ITERS=2
  run p1_it8_$r "$P1" DTF_FWD_ITERS=8
done
exit 0
