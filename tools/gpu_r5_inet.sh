#!/bin/bash
# ImageNet ResNet-50 pop 8: bench + kernel trace + full per-launch roofline table -> gpurun_out/r5in
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5in
export TMPDIR=/tmp
if [ "${INET_TEST:-0}" = "1" ]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py > gpurun_out/r5in/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5in/pytest.log; [ $rc -ne 0 ] && { grep -E "assert|Error" gpurun_out/r5in/pytest.log | head; tail -30 gpurun_out/r5in/pytest.log; exit 1; }
fi
timeout -k 10 300 python -u bench.py --model imagenet --steps 10 --warmup 3 > gpurun_out/r5in/bench.log 2>&1 || { tail -5 gpurun_out/r5in/bench.log; exit 1; }
echo "bench: $(grep '^{' gpurun_out/r5in/bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5in -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model imagenet --steps 3 --warmup 2 --exploit_every 0 > $GRAFT_REPO_ROOT/gpurun_out/r5in/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r5in/prof.log; exit 1; }
f=$(find /tmp/r5in -name "*kernel_trace*" | head -1)
cd "$GRAFT_REPO_ROOT" && python3 tools/imagenet_roofline.py --top 400 $f > gpurun_out/r5in/roofline.txt 2>&1; head -12 gpurun_out/r5in/roofline.txt
