#!/bin/bash
# round 6: memory traffic per kernel family (FETCH_SIZE / WRITE_SIZE passes + a counter-free kernel trace) for the
# pop-8 ResNet-56 step and the pop-8 ResNet-50 step -> gpurun_out/r6b
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6b
mkdir -p $O
for m in resnet imagenet; do
  if [ $m = resnet ]; then BA="--pop 8 --steps 10 --warmup 3 --exploit_every 0"; else BA="--model imagenet --steps 3 --warmup 1 --exploit_every 0"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d /tmp/bw_$m$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py $BA > $O/${m}_$c.log 2>&1
    rc=$?
    find /tmp/bw_$m$c -name "*counter_collection*" -exec cp {} $O/${m}_$c.csv \;
    rm -rf /tmp/bw_$m$c
    [ $rc -ne 0 ] && { tail -5 $O/${m}_$c.log; exit 1; }
  done
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bw_${m}_tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py $BA > $O/${m}_trace.log 2>&1 || { tail -5 $O/${m}_trace.log; exit 1; }
  find /tmp/bw_${m}_tr -name "*kernel_stats*" -exec cp {} $O/${m}_kernel_stats.csv \;
  rm -rf /tmp/bw_${m}_tr
  cd "$GRAFT_REPO_ROOT" && python3 tools/bw_summary.py $O/${m}_FETCH_SIZE.csv $O/${m}_WRITE_SIZE.csv $O/${m}_kernel_stats.csv > $O/${m}_bw.txt && head -16 $O/${m}_bw.txt
done
exit 0
