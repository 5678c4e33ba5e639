#!/bin/bash
# Per-rank evidence for the BASELINE configs (1 GPU): bench lines of every model family at one member per GPU
# (the per-rank work of pop 8 on 8 GPUs) and at pop 8, then the product PBT loop at config 4 (ResNet-110,
# exploit every 200 steps).  Outputs under gpurun_out/evidence/.  Each GPU step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/evidence
mkdir -p $out
: > $out/bench.log
DEFAULT_BENCHES="--pop 1 --steps 200 --warmup 30;--pop 2 --steps 100 --warmup 20;--pop 4 --steps 100 --warmup 20;--steps 100 --warmup 20;--ragged --steps 100 --warmup 20;--resnet_size 110 --pop 1 --steps 100 --warmup 20;--resnet_size 110 --steps 60 --warmup 10;--resnet_version 1 --steps 60 --warmup 10;--model mnist --pop 1 --steps 400 --warmup 50;--model mnist --steps 400 --warmup 50;--model imagenet --pop 1 --steps 30 --warmup 5;--model imagenet --steps 12 --warmup 3"
IFS=';' read -ra B <<< "${BENCHES:-$DEFAULT_BENCHES}"
for args in "${B[@]}"; do
  [ -z "$args" ] && continue
  timeout -k 10 300 python bench.py $args > $out/bench_one.log 2>&1
  rc=$?
  echo "ARGS: $args" >> $out/bench.log
  grep '"metric"' $out/bench_one.log >> $out/bench.log
  if [ $rc -ne 0 ]; then tail -30 $out/bench_one.log; echo "bench rc=$rc ($args)"; exit 1; fi
done
cat $out/bench.log
[ "${PBT:-1}" = "0" ] && { echo EVIDENCE_OK; exit 0; }
rm -rf /tmp/pbt_cfg4 && mkdir -p /tmp/pbt_cfg4 && cd /tmp/pbt_cfg4
timeout -k 10 600 python -u $GRAFT_REPO_ROOT/main_manager.py 8 --model cifar10 --resnet_size 110 --ready_steps 200 \
  --use_synthetic_data true --rounds ${ROUNDS:-10} --seed 1 --backend hip > $out/main_manager_r110.log 2>&1
rc=$?
cp savedata/metrics.jsonl $out/main_manager_r110_metrics.jsonl 2>/dev/null
cp test_results.txt $out/main_manager_r110_test_results.txt 2>/dev/null
tail -15 $out/main_manager_r110.log
[ $rc -ne 0 ] && { echo "main_manager rc=$rc"; exit 1; }
echo EVIDENCE_OK
