#!/bin/bash
# round checkpoint: smoke(), every model family's bench (bf16 / fp32 / fp16 HIP, deterministic builds) -> gpurun_out/fam
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fam
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fam/smoke.log 2>&1 || { tail -20 gpurun_out/fam/smoke.log; echo "smoke failed"; exit 1; }
echo "smoke: $(tail -1 gpurun_out/fam/smoke.log)"
: > gpurun_out/fam/bench.log
run() {  # env-prefix ; args
  local envs="$1"; shift
  env $envs timeout -k 10 400 python -u bench.py "$@" > gpurun_out/fam/one.log 2>&1
  local rc=$?
  echo "ARGS: [$envs] $*" >> gpurun_out/fam/bench.log
  grep '"metric"' gpurun_out/fam/one.log >> gpurun_out/fam/bench.log
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/fam/one.log; echo "bench rc=$rc ($*)"; exit 1; fi
  echo "[$envs] $*: $(grep '^{' gpurun_out/fam/one.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms', d['value'], 'img/s')")"
}
run "" --steps 100 --warmup 10
run "" --pop 1 --steps 200 --warmup 20
run "" --pop 2 --steps 200 --warmup 20
run "" --pop 4 --steps 100 --warmup 10
run "" --ragged --steps 100 --warmup 10
run "" --resnet_size 110 --steps 50 --warmup 5
run "" --resnet_size 110 --pop 1 --steps 100 --warmup 10
run "" --resnet_version 1 --steps 100 --warmup 10
run "" --model mnist --steps 100 --warmup 10
run "" --model mnist --pop 1 --steps 200 --warmup 20
run "" --model imagenet --steps 10 --warmup 3
run "" --model imagenet --pop 1 --steps 10 --warmup 3
run "" --model imagenet --resnet_version 1 --steps 10 --warmup 3
run "" --dtype fp32 --steps 20 --warmup 3
run "" --dtype fp32 --resnet_version 1 --steps 20 --warmup 3
run "" --model mnist --dtype fp32 --steps 100 --warmup 10
run "" --dtype fp16 --steps 100 --warmup 10
run "" --model imagenet --dtype fp16 --steps 10 --warmup 3
run "DTF_DETERMINISTIC=1" --steps 50 --warmup 5
run "DTF_DETERMINISTIC=1" --dtype fp32 --steps 20 --warmup 3
run "DTF_DETERMINISTIC=1" --model imagenet --steps 10 --warmup 3
run "" --model imagenet --dtype fp32 --steps 4 --warmup 1
echo FAMILIES_OK
