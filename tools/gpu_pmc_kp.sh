#!/bin/bash
# LDS bank conflicts of the k-major transposed-read kernels: product library vs LIBB (e.g. tools/var/libdtf_nokp.so)
# -> gpurun_out/pmckp/{a,b}.csv ; summary: python tools/pmc_summary.py gpurun_out/pmckp/a.csv
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmckp
grp="SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES"
for arm in a b; do
  lib=""; [ $arm = b ] && lib="$GRAFT_REPO_ROOT/$LIBB"
  cd /tmp && DTF_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-convg_}" --output-format csv -d /tmp/pk$arm -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model imagenet --steps 1 --warmup 1 --exploit_every 0 > $GRAFT_REPO_ROOT/gpurun_out/pmckp/run_$arm.log 2>&1
  rc=$?
  echo "arm $arm rc=$rc"
  find /tmp/pk$arm -name "*counter_collection*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/pmckp/$arm.csv \;
  rm -rf /tmp/pk$arm
  [ $rc -ne 0 ] && { tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmckp/run_$arm.log; exit 1; }
  cd "$GRAFT_REPO_ROOT" || exit 1
done
echo "== product (k-permuted tiles)"; python3 tools/pmc_summary.py gpurun_out/pmckp/a.csv | head -16
echo "== $LIBB"; python3 tools/pmc_summary.py gpurun_out/pmckp/b.csv | head -16
