#!/bin/bash
# t3 microbench over the variant libraries in tools/var (and the product library) -> gpurun_out/t3b/bench.log
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/t3b
out=gpurun_out/t3b/bench.log
: > $out
for lib in "" tools/var/*.so; do
  for cfg in "--hw 28" "--hw 28 --ci 256" "--hw 28 --dgrad" "--hw 14" "--hw 14 --ci 512" "--hw 14 --dgrad" "--hw 56" "--hw 56 --dgrad" ${T3_EXTRA}; do
    echo "LIB ${lib:-product} $cfg" >> $out
    timeout -k 10 120 python -u tools/t3_bench.py ${lib:+--lib $lib} $cfg >> $out 2>&1 || { tail -20 $out; exit 1; }
  done
done
grep -E "^LIB|^t3" $out
