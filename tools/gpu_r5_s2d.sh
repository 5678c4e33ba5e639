#!/bin/bash
# space-to-depth ImageNet stem + row-band 3x3 wgrad: numerics (release + det), A/B (DTF_CG_S2D / DTF_CG_WGT3) -> gpurun_out/r5s2d
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5s2d
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py tests/test_gpu_eval.py > gpurun_out/r5s2d/pytest.log 2>&1
rc=$?; echo "imagenet tests: $(tail -1 gpurun_out/r5s2d/pytest.log)"; [ $rc -ne 0 ] && { grep -E "rel|Error|assert" gpurun_out/r5s2d/pytest.log | head -30; tail -20 gpurun_out/r5s2d/pytest.log; exit 1; }
DTF_DETERMINISTIC=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py > gpurun_out/r5s2d/det.log 2>&1
rc=$?; echo "det build: $(tail -1 gpurun_out/r5s2d/det.log)"; [ $rc -ne 0 ] && { tail -20 gpurun_out/r5s2d/det.log; exit 1; }
: > gpurun_out/r5s2d/ab.log
for pass in 1 2; do
  for sw in "1 1" "0 0" "1 0" "0 1"; do
    set -- $sw
    DTF_CG_S2D=$1 DTF_CG_WGT3=$2 timeout -k 10 300 python -u bench.py --model imagenet --steps 10 --warmup 3 > gpurun_out/r5s2d/b.log 2>&1 || { tail -5 gpurun_out/r5s2d/b.log; exit 1; }
    echo "S2D=$1 WGT3=$2: $(grep '^{' gpurun_out/r5s2d/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/r5s2d/ab.log
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/s2dp -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --model imagenet --steps 3 --warmup 2 --exploit_every 0 > "$GRAFT_REPO_ROOT/gpurun_out/r5s2d/prof.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/r5s2d/prof.log"; exit 1; }
find /tmp/s2dp \( -name "*kernel_trace*" \) -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/r5s2d/" \;
cd "$GRAFT_REPO_ROOT" && python3 tools/imagenet_roofline.py gpurun_out/r5s2d/run_kernel_trace.csv > gpurun_out/r5s2d/roofline.txt 2>&1; head -14 gpurun_out/r5s2d/roofline.txt
exit 0
