#!/bin/bash
# product PBT loop (main_manager.py, sampled / explored batch sizes, synthetic data) vs bench.py --ragged with the
# SAME per-member batch sizes (metrics.jsonl 'batch_sizes' of each round) on the same box, ResNet-56 / ResNet-110
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/loop
for size in ${SIZES:-56 110}; do
  rm -rf /tmp/loop$size && mkdir -p /tmp/loop$size && cd /tmp/loop$size || exit 1
  timeout -k 10 400 python -u $GRAFT_REPO_ROOT/main_manager.py 8 --model cifar10 --resnet_size $size --use_synthetic_data true \
    --max_train_steps ${STEPS:-300} --rounds ${ROUNDS:-3} --seed 1 --backend hip > $GRAFT_REPO_ROOT/gpurun_out/loop/mm_$size.log 2>&1 \
    || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/loop/mm_$size.log; exit 1; }
  cp savedata/metrics.jsonl $GRAFT_REPO_ROOT/gpurun_out/loop/metrics_$size.jsonl
  cd "$GRAFT_REPO_ROOT" || exit 1
  python3 - > gpurun_out/loop/sizes_$size.txt <<PY
import json
for l in open("gpurun_out/loop/metrics_$size.jsonl"):
    r = json.loads(l)
    print(r["round"], ",".join(str(r["batch_sizes"][k]) for k in sorted(r["batch_sizes"], key=int)))
PY
  while read rnd bs; do
    timeout -k 10 200 python -u bench.py --resnet_size $size --ragged --batch_sizes $bs --steps ${STEPS:-300} --warmup 10 \
      --exploit_every 0 > gpurun_out/loop/bench_${size}_$rnd.log 2>&1 || { tail -5 gpurun_out/loop/bench_${size}_$rnd.log; exit 1; }
  done < gpurun_out/loop/sizes_$size.txt
  python3 - $size <<'PY'
import json, sys
size = sys.argv[1]
for l in open("gpurun_out/loop/metrics_%s.jsonl" % size):
    r = json.loads(l)
    b = [json.loads(x) for x in open("gpurun_out/loop/bench_%s_%d.log" % (size, r["round"])) if x.startswith("{")][-1]
    ph = r["phases_s"]
    ts = ph.get("train_steps", 0)
    tput = r["images"] / ts if ts else 0
    print("R%s round %d sizes %s: loop train_steps %.1f img/s vs bench --ragged (same sizes) %.1f img/s = %.1f%%; "
          "enqueue %.3fs drain %.3fs steps %d; whole round %.1f img/s"
          % (size, r["round"], ",".join(str(r["batch_sizes"][k]) for k in sorted(r["batch_sizes"], key=int)), tput,
             b["value"], 100 * tput / b["value"], ph.get("host_step_enqueue", 0), ph.get("train_drain", 0),
             ph.get("train_step_count", 0), r["images_per_s"] or 0))
PY
done
