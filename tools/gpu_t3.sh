#!/bin/bash
# ImageNet ResNet-50: step tests, bench, kernel trace + roofline table -> gpurun_out/t3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/t3
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_imagenet_step.py tests/test_gpu_eval.py -k "imagenet" > gpurun_out/t3/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/t3/pytest.log; [ $rc -ne 0 ] && { grep -E "assert|Error" gpurun_out/t3/pytest.log | head; exit 1; }
timeout -k 10 300 python -u bench.py --model imagenet --steps 10 --warmup 3 > gpurun_out/t3/bench.log 2>&1 || { tail -5 gpurun_out/t3/bench.log; exit 1; }
echo "bench: $(grep '^{' gpurun_out/t3/bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/t3p -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model imagenet --steps 3 --warmup 2 --exploit_every 0 > $GRAFT_REPO_ROOT/gpurun_out/t3/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/t3/prof.log; exit 1; }
f=$(find /tmp/t3p -name "*kernel_trace*" | head -1)
cd "$GRAFT_REPO_ROOT" && python3 tools/imagenet_roofline.py $f > gpurun_out/t3/roofline.txt 2>&1; head -12 gpurun_out/t3/roofline.txt
