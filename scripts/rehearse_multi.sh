#!/bin/bash
# Functional rehearsal of the multi-rank bench paths on ONE GPU (ranks share the card, gloo group for the
# handle exchange, the engines' inboxes IPC-mapped between the processes). Numbers are not meaningful; the 8-GPU runs belong to the driver.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# --same-gpu: every rank on GPU 0, plain engine launches (cooperative launches from several processes take turns on
# the card)
run() {  # run <name> <args...>: `bench.py --gpus 2` spawns its two ranks itself (as the driver's N=2 line)
  local name=$1; shift
  timeout -k 10 500 python bench.py --gpus 2 --same-gpu "$@" > gpurun_out/$name.log 2>&1
  local rc=$?; echo "=== $name rc=$rc"; grep '^{' gpurun_out/$name.log | head -c 1500; echo
  return $rc
}
run rehearse_auto --steps 1 --warmup 1 --no-cpu-baseline --jobs 400 --side-steps 2 &&
run rehearse_replicas --steps 2 --warmup 1 --no-cpu-baseline --mode replicas
