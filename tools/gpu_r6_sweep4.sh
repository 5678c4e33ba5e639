#!/bin/bash
# round 6 (late): ResNet-50 work-split knobs re-swept on the final kernels -> gpurun_out/r6s4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6s4
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --model imagenet --steps 8 --warmup 3 > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for r in 1 2; do
  run base_$r
  run minchunk1024_$r DTF_CG_WG_MINCHUNK=1024
  run minchunk4096_$r DTF_CG_WG_MINCHUNK=4096
  run wgt3_384_$r DTF_CG_WGT3_TARGET=384
  run wgt3_768_$r DTF_CG_WGT3_TARGET=768
  run shortk64_$r DTF_CG_SHORTK=64
  run small512_$r DTF_CG_SMALL=512
done
exit 0
