#!/bin/bash
# Functional rehearsal of the multi-rank bench paths on ONE GPU (ranks share the card, gloo group,
# host-staged shard exchange). Numbers are not meaningful; the 8-GPU runs belong to the driver.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export KB_BENCH_SAME_GPU=1
run() {  # run <name> <args...>
  local name=$1; shift
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 2 "$@" > gpurun_out/$name.log 2>&1
  local rc=$?; echo "=== $name rc=$rc"; grep '^{' gpurun_out/$name.log | head -c 1500; echo
  return $rc
}
run rehearse_auto --steps 2 --warmup 1 --no-cpu-baseline --jobs 300 --shard-jobs 50 &&
run rehearse_shard --steps 2 --warmup 1 --no-cpu-baseline --mode shard --config C5 --nodes 40000 --jobs 100
