#!/bin/bash
# side-stream deferred-wgrad overlap (hip_resnet WG_OVERLAP): step tests at pop 1/2, then pop-1 / pop-2 bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ov
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_state_import.py tests/test_gpu_resnet_step.py -k "benchmark_shapes or pop1 or pop2 or side_stream" > gpurun_out/ov/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ov/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/ov/pytest.log | head; exit 1; }
for pop in 1 2; do
for v in "0 0" "1 0" "1 4" "1 3"; do
  set -- $v
  DTF_WG_OVERLAP=$1 DTF_WG_OVERLAP_CHUNK=$2 timeout -k 10 200 python -u bench.py --pop $pop --steps 200 --warmup 20 --exploit_every 0 > gpurun_out/ov/b.log 2>&1 || { tail -5 gpurun_out/ov/b.log; exit 1; }
  echo "pop $pop overlap $1 chunk $2: $(grep '^{' gpurun_out/ov/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s', d['config'].get('step_graph'))")" | tee -a gpurun_out/ov/ab.log
done
done
