#!/bin/bash
# A/B of alternative kernel-library builds (DTF_LIB): LIBS="path1;path2" (empty entry = the release library),
# bench args in $BARGS, $REPS rounds of alternation.  One line per run in gpurun_out/ablib.log.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ablib.log
IFS=';' read -ra V <<< "$LIBS"
IFS='|' read -ra A <<< "$BARGS"
for r in $(seq 1 ${REPS:-2}); do
  for args in "${A[@]}"; do
    for lib in "${V[@]}"; do
      DTF_LIB=$lib timeout -k 10 300 python bench.py $args > gpurun_out/ablib_one.log 2>&1
      rc=$?
      line=$(grep '"metric"' gpurun_out/ablib_one.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')" 2>/dev/null)
      echo "[${lib:-release}] $args => $line" >> gpurun_out/ablib.log
      if [ $rc -ne 0 ]; then tail -30 gpurun_out/ablib_one.log; cat gpurun_out/ablib.log; exit 1; fi
    done
  done
done
cat gpurun_out/ablib.log
