#!/bin/bash
# ImageNet kernel changes: numerics (release + det) and an A/B over ARMS ("ENV=.. ENV2=..|lib" entries, lib empty =
# the default build) of bench.py --model imagenet -> gpurun_out/r5ia
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5ia
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py > gpurun_out/r5ia/pytest.log 2>&1
rc=$?; echo "imagenet tests: $(tail -1 gpurun_out/r5ia/pytest.log)"; [ $rc -ne 0 ] && { grep -E "rel|Error|assert" gpurun_out/r5ia/pytest.log | head -30; tail -20 gpurun_out/r5ia/pytest.log; exit 1; }
DTF_DETERMINISTIC=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py > gpurun_out/r5ia/det.log 2>&1
rc=$?; echo "det build: $(tail -1 gpurun_out/r5ia/det.log)"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r5ia/det.log; exit 1; }
fi
: > gpurun_out/r5ia/ab.log
IFS=';' read -ra ARMS_A <<< "${ARMS:-|}"
for pass in 1 2; do
  for arm in "${ARMS_A[@]}"; do
    envs="${arm%%|*}"; lib="${arm#*|}"
    env $envs DTF_LIB=$lib timeout -k 10 300 python -u bench.py --model imagenet --steps 10 --warmup 3 $BENCH_EXTRA > gpurun_out/r5ia/b.log 2>&1 || { tail -5 gpurun_out/r5ia/b.log; exit 1; }
    echo "[$envs|$lib]: $(grep '^{' gpurun_out/r5ia/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/r5ia/ab.log
  done
done
[ -n "$SKIP_PROF" ] && exit 0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/iap -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --model imagenet --steps 3 --warmup 2 --exploit_every 0 > "$GRAFT_REPO_ROOT/gpurun_out/r5ia/prof.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/r5ia/prof.log"; exit 1; }
find /tmp/iap \( -name "*kernel_trace*" \) -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/r5ia/" \;
cd "$GRAFT_REPO_ROOT" && python3 tools/imagenet_roofline.py gpurun_out/r5ia/run_kernel_trace.csv --top 30 > gpurun_out/r5ia/roofline.txt 2>&1; head -12 gpurun_out/r5ia/roofline.txt
exit 0
