#!/bin/bash
# PMC counters (one pass per group; kernel-trace-free --pmc runs only) for the kernels matching KRE of
# `bench.py $BARGS`.  Output: gpurun_out/pmc/counters_<i>.csv
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_ANY" \
           "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-conv_}" --output-format csv -d /tmp/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py $BARGS > $GRAFT_REPO_ROOT/gpurun_out/pmc/run$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc"
  find /tmp/pmc$i -name "*counter_collection*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/pmc/counters_$i.csv \;
  rm -rf /tmp/pmc$i
  if [ $rc -ne 0 ]; then tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc/run$i.log; echo "stopping after rc=$rc"; exit 1; fi
done
echo SESSION_OK
