#!/bin/bash
# GPU: new eval / PBT-loop tests, then the product PBT loop (main_manager.py) at the headline config on one GPU,
# then a bench line for comparison.  Outputs under gpurun_out/pbt_run/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pbt_run
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_eval.py tests/test_gpu_pbt_loop.py} > gpurun_out/pbt_run/pytest.log 2>&1
rc=$?; tail -25 gpurun_out/pbt_run/pytest.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit 1; }
[ "${PBT:-1}" = "0" ] && { echo PBT_OK; exit 0; }
rm -rf /tmp/pbt_run && mkdir -p /tmp/pbt_run && cd /tmp/pbt_run
timeout -k 10 600 python -u $GRAFT_REPO_ROOT/main_manager.py 8 --model cifar10 --resnet_size 56 --use_synthetic_data ${SYN:-true} \
  --max_train_steps ${STEPS:-200} --rounds ${ROUNDS:-4} --seed 1 --backend hip $PBT_ARGS > $GRAFT_REPO_ROOT/gpurun_out/pbt_run/main_manager.log 2>&1
rc=$?
cp savedata/metrics.jsonl savedata/best_model.json test_results.txt $GRAFT_REPO_ROOT/gpurun_out/pbt_run/ 2>/dev/null
tail -15 $GRAFT_REPO_ROOT/gpurun_out/pbt_run/main_manager.log
cat $GRAFT_REPO_ROOT/gpurun_out/pbt_run/metrics.jsonl
[ $rc -ne 0 ] && { echo "main_manager rc=$rc"; exit 1; }
echo PBT_OK
