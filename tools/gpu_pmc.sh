#!/bin/bash
# PMC counter collection for the conv kernels (separate runs, kernel-trace only; no sys/runtime trace).
# Per pass at most 8 SQ_, 4 TCC_ (FETCH_SIZE = 3, WRITE_SIZE = 2), 2 GRBM_ counters.  $PMC_REGEX / $PMC_BENCH
# override the kernel filter and the bench arguments.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
grep -o -E "^[[:space:]]*(SQ_|TCC_|TCP_|TA_|GRBM_|FETCH|WRITE|Mfma|VALU|LDS|Occ)[A-Za-z0-9_]*" gpurun_out/pmc/avail.txt | sort -u > gpurun_out/pmc/names.txt || true
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "${PMC_REGEX:-conv_|bn_bwd}" --output-format csv -d /tmp/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py ${PMC_BENCH:---steps 2 --warmup 1 --exploit_every 0} > $GRAFT_REPO_ROOT/gpurun_out/pmc/run$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc"
  find /tmp/pmc$i -name "*counter_collection*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/pmc/counters_$i.csv \;
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; break; fi
done
ls -la $GRAFT_REPO_ROOT/gpurun_out/pmc
