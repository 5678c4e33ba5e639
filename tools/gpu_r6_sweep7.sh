#!/bin/bash
# round 6 (late): forward iterations per workgroup for C = 16 / 32 at pop 8 -> gpurun_out/r6s7
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s7
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for r in 1 2 3; do
  run base_$r
  run it16_2_$r DTF_FWD_ITERS16=2
  run it16_8_$r DTF_FWD_ITERS16=8
  run it32_8_$r DTF_FWD_ITERS32=8
done
exit 0
