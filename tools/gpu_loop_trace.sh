#!/bin/bash
# kernel traces of the product loop (main_manager.py R56, 1 round) and of bench.py --ragged with the same sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lt
export TMPDIR=/tmp
rm -rf /tmp/ltm && mkdir -p /tmp/ltm && cd /tmp/ltm || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/ltm/prof -o run -- python3 $GRAFT_REPO_ROOT/main_manager.py 8 --model cifar10 --resnet_size 56 --use_synthetic_data true --max_train_steps 300 --rounds 1 --seed 1 --backend hip > $GRAFT_REPO_ROOT/gpurun_out/lt/mm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/lt/mm.log; exit 1; }
f=$(find /tmp/ltm/prof -name "*kernel_trace*" | head -1)
python3 $GRAFT_REPO_ROOT/tools/step_spans.py $f | tee $GRAFT_REPO_ROOT/gpurun_out/lt/loop_spans.txt
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/ltb -o run -- python3 $GRAFT_REPO_ROOT/bench.py --ragged --batch_sizes 231,220,72,173,153,112,142,127 --steps 300 --warmup 10 --exploit_every 0 > $GRAFT_REPO_ROOT/gpurun_out/lt/bench.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/lt/bench.log; exit 1; }
f=$(find /tmp/ltb -name "*kernel_trace*" | head -1)
python3 $GRAFT_REPO_ROOT/tools/step_spans.py $f | tee $GRAFT_REPO_ROOT/gpurun_out/lt/bench_spans.txt
