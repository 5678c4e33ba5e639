#!/bin/bash
# A/B of the in-tree library against distributedtf_amd/ops/libdtf_kernels_old.so (DTF_LIB), runs interleaved:
#   bash tools/gpu_ab_lib.sh <out subdir> "<pytest files>" "<bench args>" ["<bench args 2>"]
# -> gpurun_out/<out>/ab.log (numerics first: the pytest files on the new library)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider $2 > $O/pytest.log 2>&1
  rc=$?; echo "tests: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/pytest.log | head; exit 1; }
fi
OLD=$GRAFT_REPO_ROOT/distributedtf_amd/ops/libdtf_kernels_old.so
shift 2
for BA in "$@"; do
  tag=$(echo "$BA" | tr -c 'a-z0-9' '_')
  for r in 1 2 3; do
    for f in old new; do
      if [ $f = old ]; then L=$OLD; else L=""; fi
      DTF_LIB=$L timeout -k 10 300 python3 -u bench.py $BA > $O/b_${tag}_${f}_$r.log 2>&1 || { tail -5 $O/b_${tag}_${f}_$r.log; exit 1; }
      echo "[$BA] lib=$f run $r: $(grep '^{' $O/b_${tag}_${f}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], d['unit'])")" | tee -a $O/ab.log
    done
  done
done
exit 0
