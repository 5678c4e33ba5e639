#!/bin/bash
# round 6 knob sweep: ResNet-56 pop 8 deferred-wgrad split / width set, ResNet-50 fold1 width -> gpurun_out/r6k
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6k
mkdir -p $O
b() {  # tag env... -- bench args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 -u bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "$tag: $(grep '^{' $O/$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for what in ${*:-cifar inet}; do
case $what in
  cifar)
    for r in 1 2; do
      b "p8_base_$r" X=1 -- --steps 100 --warmup 20
      b "p8_d64wg4_$r" DTF_DEFER64_WG=4 -- --steps 100 --warmup 20
      b "p8_d64wg16_$r" DTF_DEFER64_WG=16 -- --steps 100 --warmup 20
      b "p8_mid8_$r" DTF_DEFER_MID_POP=8 -- --steps 100 --warmup 20
      b "p8_f16t768_$r" DTF_FUSED_TOTAL16=768 -- --steps 100 --warmup 20
    done ;;
  inet)
    DTF_CG_FOLD1_MAXC=512 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_imagenet_step.py > $O/inet_fold512.log 2>&1
    rc=$?; tail -1 $O/inet_fold512.log; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/inet_fold512.log | head; exit 1; }
    for r in 1 2; do
      for m in 128 256 512; do
        b "inet_fold1max${m}_$r" DTF_CG_FOLD1_MAXC=$m -- --model imagenet --steps 10 --warmup 3
      done
    done ;;
esac
done
exit 0
