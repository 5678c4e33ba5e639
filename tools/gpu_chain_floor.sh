#!/bin/bash
# Launch-chain floor on the GPU box (tools/chain_floor.hip).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/bin/chain_floor > gpurun_out/chain_floor.txt 2>&1 || { cat gpurun_out/chain_floor.txt; exit 1; }
cat gpurun_out/chain_floor.txt
