#!/bin/bash
# round 6: CIFAR members interleaved over the workgroup index (one XCD subset per member, ConvArgs.u_xcd) --
# numerics, then A/B: new library with DTF_CIFAR_XCD=1 vs =0 (same library: the interleave is a kernel argument)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6x8
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_resnet_step.py tests/test_gpu_golden_hip.py > $O/pytest.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head; exit 1; }
run() {  # name, bench args, env...
  local n=$1 ba=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py $ba > $O/b_$n.log 2>&1 || { tail -5 $O/b_$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/b_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/ab.log
}
for r in 1 2 3; do
  run p8_off_$r "--steps 100 --warmup 10" DTF_CIFAR_XCD=0
  run p8_on_$r "--steps 100 --warmup 10" DTF_CIFAR_XCD=1
done
for r in 1 2; do
  run p4_off_$r "--pop 4 --steps 100 --warmup 10" DTF_CIFAR_XCD=0
  run p4_on_$r "--pop 4 --steps 100 --warmup 10" DTF_CIFAR_XCD=1
  run p2_off_$r "--pop 2 --steps 200 --warmup 20" DTF_CIFAR_XCD=0
  run p2_on_$r "--pop 2 --steps 200 --warmup 20" DTF_CIFAR_XCD=1
  run r110_off_$r "--resnet_size 110 --steps 50 --warmup 5" DTF_CIFAR_XCD=0
  run r110_on_$r "--resnet_size 110 --steps 50 --warmup 5" DTF_CIFAR_XCD=1
done
exit 0
