#!/bin/bash
# A/B of work-split constants (tools/ab_bench.py): AB="--set A=1 --set B=2;;--set C=3" (';'-separated variants,
# empty = defaults), bench args in $BARGS.  One line per variant in gpurun_out/ab.log.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.log
IFS=';' read -ra V <<< "$AB"
for sets in "${V[@]}"; do
  timeout -k 10 300 python tools/ab_bench.py $sets -- $BARGS > gpurun_out/ab_one.log 2>&1
  rc=$?
  line=$(grep '"metric"' gpurun_out/ab_one.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')" 2>/dev/null)
  echo "[$sets] => $line" >> gpurun_out/ab.log
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/ab_one.log; cat gpurun_out/ab.log; exit 1; fi
done
cat gpurun_out/ab.log
