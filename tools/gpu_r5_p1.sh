#!/bin/bash
# round 5: pop-1 / pop-8 step tests + benches + pop-1 kernel trace (-> gpurun_out/r5p1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5p1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resnet_step.py tests/test_gpu_pbt_loop.py > gpurun_out/r5p1/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r5p1/pytest.log; [ $rc -ne 0 ] && { grep -E "assert|Error" gpurun_out/r5p1/pytest.log | head; tail -40 gpurun_out/r5p1/pytest.log; exit 1; }
for args in "--pop 1 --steps 200 --warmup 20" "--pop 2 --steps 200 --warmup 20" "--steps 100 --warmup 10" "${EXTRA_BENCH:---pop 1 --steps 200 --warmup 20}"; do
  timeout -k 10 200 python -u bench.py $args > gpurun_out/r5p1/b.log 2>&1 || { tail -5 gpurun_out/r5p1/b.log; exit 1; }
  echo "$args: $(grep '^{' gpurun_out/r5p1/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/r5p1/bench.log
done
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p1x -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --pop 1 --steps 30 --warmup 5 --exploit_every 0 > "$GRAFT_REPO_ROOT/gpurun_out/r5p1/prof.log" 2>&1 || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/r5p1/prof.log"; exit 1; }
find /tmp/p1x \( -name "*kernel_stats*" -o -name "*kernel_trace*" \) -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/r5p1/" \;
cd "$GRAFT_REPO_ROOT" && python3 tools/kstats.py gpurun_out/r5p1/run_kernel_stats.csv 40 > gpurun_out/r5p1/kstats.txt && head -25 gpurun_out/r5p1/kstats.txt
python3 tools/trace_gaps.py gpurun_out/r5p1/run_kernel_trace.csv > gpurun_out/r5p1/gaps.txt 2>&1; head -8 gpurun_out/r5p1/gaps.txt
