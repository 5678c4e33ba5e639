#!/bin/bash
# A/B of alternative kernel-library builds (DTF_LIB) on the bench: step tests at the bench shapes with each
# variant, then interleaved bench runs.  Usage: AB_LIBS="default x1 DTF_FOO=0" AB_POPS="8 1" tools/gpu_ab.sh
# (a variant is a library suffix -- ops/libdtf_kernels_<v>.so -- or one VAR=value environment assignment)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
LIBS=${AB_LIBS:-"default x1"}
POPS=${AB_POPS:-"8"}
REPS=${AB_REPS:-2}
EXTRA=${AB_EXTRA:-""}
# (lib:VAR=value: both)
libpath() { local l=${1%%:*}; case "$l" in default|*=*) echo "";; *) echo "$GRAFT_REPO_ROOT/distributedtf_amd/ops/libdtf_kernels_$l.so";; esac; }
venv() { local e=${1#*:}; case "$e" in *=*) echo "${e//,/ }";; *) echo "DTF_AB_NONE=1";; esac; }  # A=1,B=2
for v in $LIBS; do
  [ "$v" = default ] && continue
  env $(venv $v) DTF_LIB=$(libpath $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
    tests/test_gpu_resnet_step.py -k "${AB_TESTS:-benchmark_shapes}" > gpurun_out/ab/pytest_$v.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/ab/pytest_$v.log)"
  [ $rc -ne 0 ] && { grep -E "assert|Error" gpurun_out/ab/pytest_$v.log | head; exit 1; }
done
for r in $(seq 1 $REPS); do
  for pop in $POPS; do
    for v in $LIBS; do
      env $(venv $v) DTF_LIB=$(libpath $v) timeout -k 10 200 python -u bench.py --pop $pop --steps 200 --warmup 20 $EXTRA \
        > gpurun_out/ab/b_${v}_p${pop}_r$r.log 2>&1 || { tail -5 gpurun_out/ab/b_${v}_p${pop}_r$r.log; exit 1; }
      echo "rep $r pop $pop $v: $(grep '^{' gpurun_out/ab/b_${v}_p${pop}_r$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")"
    done
  done
done
echo AB_OK
