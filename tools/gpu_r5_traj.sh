#!/bin/bash
# strict trajectory test (recomputed BN statistics, per-member eval gap <= 0.05), three passes; det bench -> gpurun_out/r5tr
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5tr
for i in 1 2 3; do
  timeout -k 10 560 python -u -m pytest -x -v -s --timeout 540 --timeout-method thread tests/test_gpu_trajectory.py > gpurun_out/r5tr/pass$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; grep -E "passed|failed|eval acc|Error" gpurun_out/r5tr/pass$i.log | head -8
  [ $rc -ne 0 ] && { tail -40 gpurun_out/r5tr/pass$i.log; exit 1; }
done
DTF_DETERMINISTIC=1 timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 > gpurun_out/r5tr/det.log 2>&1 || { tail -5 gpurun_out/r5tr/det.log; exit 1; }
echo "det bench: $(grep '^{' gpurun_out/r5tr/det.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")"
