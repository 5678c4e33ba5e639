#!/bin/bash
# round 6: ResNet-50 pop-8 kernel trace + per-kernel stats with the current defaults, the HBM-floor roofline over it
# and the per-family memory traffic (FETCH_SIZE / WRITE_SIZE passes) -> gpurun_out/r6i
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6i
mkdir -p $O
BA="--model imagenet --steps 3 --warmup 1 --exploit_every 0"
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r6i_tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py $BA > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
find /tmp/r6i_tr -name "*kernel_stats*" -exec cp {} $O/kernel_stats.csv \;
find /tmp/r6i_tr -name "*kernel_trace*" -exec cp {} $O/kernel_trace.csv \;
rm -rf /tmp/r6i_tr
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d /tmp/r6i_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py $BA > $O/$c.log 2>&1
  rc=$?
  find /tmp/r6i_$c -name "*counter_collection*" -exec cp {} $O/$c.csv \;
  rm -rf /tmp/r6i_$c
  [ $rc -ne 0 ] && { tail -5 $O/$c.log; exit 1; }
done
cd "$GRAFT_REPO_ROOT" || exit 1
python3 tools/imagenet_roofline.py $O/kernel_trace.csv > $O/roofline.txt 2>&1 && head -30 $O/roofline.txt
python3 tools/bw_summary.py $O/FETCH_SIZE.csv $O/WRITE_SIZE.csv $O/kernel_stats.csv > $O/bw.txt && head -30 $O/bw.txt
exit 0
