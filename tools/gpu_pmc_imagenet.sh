#!/bin/bash
# PMC counters of the ImageNet convg kernels (one pass per group; kernel-trace style collection only).
# Group sizes respect the per-pass limits (<= 8 SQ, <= 4 TCC with FETCH_SIZE = 3 and WRITE_SIZE = 2, <= 2 GRBM).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_in
ARGS=${ARGS:---model imagenet --steps 1 --warmup 1 --exploit_every 0}
REGEX=${REGEX:-convg_}
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex "$REGEX" --output-format csv -d /tmp/pmcin$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $GRAFT_REPO_ROOT/gpurun_out/pmc_in/run$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc"
  find /tmp/pmcin$i -name "*counter_collection*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/pmc_in/counters_$i.csv \;
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc_in/run$i.log; exit 1; fi
done
ls -la $GRAFT_REPO_ROOT/gpurun_out/pmc_in
echo PMC_OK
