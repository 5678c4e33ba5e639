#!/bin/bash
# round 6: deterministic build after the head / deferred-wgrad / coefficient fixes: replay check, pop-8 bench
# (release and det), det kernel stats, placement invariance at world 1/2/4/8 -> gpurun_out/r6d
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6d
mkdir -p $O
for what in ${*:-check bench prof place}; do
case $what in
  check)
    DTF_DETERMINISTIC=1 timeout -k 10 300 python3 -u tools/det_check.py > $O/det_check.log 2>&1; rc=$?
    grep -E "identical|DET_" $O/det_check.log; [ $rc -ne 0 ] && { tail -20 $O/det_check.log; exit 1; } ;;
  bench)
    for r in 1 2; do
      for d in 0 1; do
        DTF_DETERMINISTIC=$d timeout -k 10 200 python3 -u bench.py --steps 50 > $O/bench_det${d}_$r.log 2>&1 || { tail -5 $O/bench_det${d}_$r.log; exit 1; }
        echo "det=$d run $r: $(grep '^{' $O/bench_det${d}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")" | tee -a $O/bench_ab.log
      done
    done ;;
  prof)
    cd /tmp && DTF_DETERMINISTIC=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_det -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --pop 8 --steps 30 --warmup 5 --exploit_every 0 > $O/prof_det.log 2>&1 || { tail -5 $O/prof_det.log; exit 1; }
    find /tmp/prof_det -name "*kernel_stats*" -exec cp {} $O/det_kernel_stats.csv \;
    rm -rf /tmp/prof_det
    cd "$GRAFT_REPO_ROOT" && python3 tools/kstats.py $O/det_kernel_stats.csv 30 > $O/det_kstats.txt && head -12 $O/det_kstats.txt ;;
  place)
    cd "$GRAFT_REPO_ROOT" && timeout -k 10 1180 python3 -u -m pytest -x -v -s --timeout 1150 --timeout-method thread -p no:cacheprovider tests/test_gpu_placement.py > $O/placement.log 2>&1; rc=$?
    grep -E "passed|failed|world|Error|assert" $O/placement.log | head -30; [ $rc -ne 0 ] && { tail -30 $O/placement.log; exit 1; } ;;
esac
done
exit 0
