#!/bin/bash
# LDS pitch A/B (conv.hip DTF_WP64 / DTF_CPF16 builds in tools/abl): pop 8 and pop 1 benches, two interleaved
# passes -> gpurun_out/r5pa/ab.log
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5pa
for pass in 1 2; do
  for lib in "" tools/abl/libdtf_wp16.so tools/abl/libdtf_wp16c16.so tools/abl/libdtf_c16.so; do
    for args in "--steps 100 --warmup 10" "--pop 1 --steps 200 --warmup 20"; do
      DTF_LIB=$lib timeout -k 10 200 python -u bench.py $args > gpurun_out/r5pa/b.log 2>&1 || { tail -5 gpurun_out/r5pa/b.log; exit 1; }
      echo "[$lib] $args: $(grep '^{' gpurun_out/r5pa/b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a gpurun_out/r5pa/ab.log
    done
  done
done
