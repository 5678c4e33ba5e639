#!/bin/bash
# CIFAR step tests at the bench shapes, pop 1 / pop 8 bench, pop-1 kernel stats -> gpurun_out/p1x
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/p1x
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_resnet_step.py -k "benchmark_shapes or pop1 or pop2" > gpurun_out/p1x/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/p1x/pytest.log; [ $rc -ne 0 ] && { grep -E "assert|Error" gpurun_out/p1x/pytest.log | head; exit 1; }
for pop in 1 8; do
  timeout -k 10 200 python -u bench.py --pop $pop --steps 200 --warmup 20 > gpurun_out/p1x/b$pop.log 2>&1 || { tail -5 gpurun_out/p1x/b$pop.log; exit 1; }
  echo "pop $pop: $(grep '^{' gpurun_out/p1x/b$pop.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")"
done
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p1x -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --pop 1 --steps 30 --warmup 5 --exploit_every 0 > "$GRAFT_REPO_ROOT/gpurun_out/p1x/prof.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/p1x/prof.log"; exit 1; }
find /tmp/p1x \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/p1x/" \;
cd "$GRAFT_REPO_ROOT" && python3 tools/kstats.py gpurun_out/p1x/run_kernel_stats.csv 40 | grep -E "total|slab|head|weight_prep|trans|wgrad_all"
