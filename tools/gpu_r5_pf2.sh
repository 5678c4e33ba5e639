#!/bin/bash
# forward two-band prefetch (DTF_FWD_PF2, default build) vs one-band (tools/abl/libdtf_pf1.so): numerics + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5pf
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resnet_step.py > gpurun_out/r5pf/pytest.log 2>&1
rc=$?; echo "resnet step tests: $(tail -1 gpurun_out/r5pf/pytest.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r5pf/pytest.log; exit 1; }
: > gpurun_out/r5pf/ab.log
for pass in 1 2; do
  for lib in "" tools/abl/libdtf_pf1.so; do
    for args in "--steps 100 --warmup 10" "--pop 1 --steps 200 --warmup 20" "--pop 2 --steps 200 --warmup 20"; do
      DTF_LIB=$lib timeout -k 10 200 python -u bench.py $args > gpurun_out/r5pf/b.log 2>&1 || { tail -5 gpurun_out/r5pf/b.log; exit 1; }
      echo "[$lib] $args: $(grep '^{' gpurun_out/r5pf/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/r5pf/ab.log
    done
  done
done
exit 0
