#!/bin/bash
# round 6 (late): C = 32 fused-backward per-launch workgroup cap re-swept at pop 8 -> gpurun_out/r6s3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s3
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for r in 1 2; do
  run base_$r
  run t32_192_$r DTF_FUSED_TOTAL32=192
  run t32_384_$r DTF_FUSED_TOTAL32=384
  run t32_512_$r DTF_FUSED_TOTAL32=512
  run min128_$r DTF_FUSED_MIN_WG=128
done
exit 0
