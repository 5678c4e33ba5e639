#!/bin/bash
# Sweep runner (reference test_runner.sh:1-24, which looped MPI world sizes x population sizes):
# world size (GPUs, one process each) x population size; every run appends
# "n = <world>, pop_size = <P>, time = <s>s" to test_results.txt (main_manager.py).
#
#   tools/test_runner.sh                       # CIFAR-10 ResNet-56, synthetic data, GPUs 1 2 4 8, pop 8 16
#   MODEL=toy GPUS="2 3 5" POPS="10 20" tools/test_runner.sh   # CPU plumbing sweep over gloo
set -u
MODEL=${MODEL:-cifar10}
GPUS=${GPUS:-"1 2 4 8"}
POPS=${POPS:-"8 16"}
ROUNDS=${ROUNDS:-4}
EXTRA=${EXTRA:-"--use_synthetic_data true --max_train_steps 200"}
cd "$(dirname "$0")/.." || exit 1
for n in $GPUS; do
  for pop in $POPS; do
    echo "=== n=$n pop=$pop model=$MODEL"
    if [ "$MODEL" = "toy" ]; then
      python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29533 \
        main_manager.py "$pop" --model toy --rounds "$ROUNDS" || exit 1
    else
      python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29533 \
        main_manager.py "$pop" --model "$MODEL" --rounds "$ROUNDS" $EXTRA || exit 1
    fi
  done
done
tail -n 20 test_results.txt
