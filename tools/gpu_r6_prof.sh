#!/bin/bash
# round 6 evidence pass: pop-8 kernel stats (release + deterministic build), pop-1 stats, pop-8 PMC of the fused
# backward / forward stage kernels, fp16 deterministic replay -> gpurun_out/r6p
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6p
mkdir -p $O
prof() {  # tag env... -- bench args
  local tag=$1; shift
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$tag -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  find /tmp/prof_$tag -name "*kernel_stats*" -exec cp {} $O/${tag}_kernel_stats.csv \;
  find /tmp/prof_$tag -name "*kernel_trace*" -exec cp {} $O/${tag}_kernel_trace.csv \;
  rm -rf /tmp/prof_$tag
  cd "$GRAFT_REPO_ROOT" && python3 tools/kstats.py $O/${tag}_kernel_stats.csv 30 > $O/${tag}_kstats.txt && head -12 $O/${tag}_kstats.txt
}
for what in ${*:-p8 det p1 pmc f16det}; do
case $what in
  p8) prof p8 --pop 8 --steps 30 --warmup 5 --exploit_every 0 ;;
  det) DTF_DETERMINISTIC=1 prof det --pop 8 --steps 30 --warmup 5 --exploit_every 0 ;;
  p1) prof p1 --pop 1 --steps 30 --warmup 5 --exploit_every 0 ;;
  pmc)
    i=0
    for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA" \
               "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_ANY" \
               "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
      i=$((i+1))
      cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "conv_" --output-format csv -d /tmp/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --pop 8 --steps 10 --warmup 3 --exploit_every 0 > $O/pmc_run$i.log 2>&1
      rc=$?
      find /tmp/pmc$i -name "*counter_collection*" -exec cp {} $O/pmc_counters_$i.csv \;
      rm -rf /tmp/pmc$i
      [ $rc -ne 0 ] && { tail -5 $O/pmc_run$i.log; exit 1; }
    done
    cd "$GRAFT_REPO_ROOT" && python3 tools/pmc_summary.py $O/pmc_counters_*.csv > $O/pmc_pop8.txt && head -14 $O/pmc_pop8.txt ;;
  f16det)
    cd "$GRAFT_REPO_ROOT" && DTF_HALF=1 DTF_DETERMINISTIC=1 timeout -k 10 200 python3 -u tools/det_check.py > $O/f16det.log 2>&1; rc=$?
    cat $O/f16det.log | tail -8; [ $rc -ne 0 ] && exit 1 ;;
esac
done
exit 0
