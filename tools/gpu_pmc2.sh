#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "MfmaUtil OccupancyPercent" \
           "MemUnitStalled SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 150 rocprofv3 --pmc $grp --kernel-include-regex "conv_|bn_bwd" --output-format csv -d /tmp/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --exploit_every 0 > $GRAFT_REPO_ROOT/gpurun_out/pmc2/run$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc"
  find /tmp/pmc$i -name "*counter_collection*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/pmc2/counters_$i.csv \;
  rm -rf /tmp/pmc$i
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; break; fi
done
