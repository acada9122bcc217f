#!/bin/bash
# eval_plain A/B: the production kernel, the store-only variant (one node per lane) and the store-only variant
# with two nodes per lane (64-bit stores), each through scripts/eval_probe.py at the bench's eval workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05e}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in "" evalso evalso2; do
  lib=scheduler_amd/libkbgpu${v:+_$v}.so
  KBGPU_LIB=$lib timeout -k 10 120 python scripts/eval_probe.py 0 > "gpurun_out/${TAG}_eval${v}.log" 2>&1 || { tail -3 "gpurun_out/${TAG}_eval${v}.log"; exit 1; }
  echo "${v:-prod}: $(tail -1 "gpurun_out/${TAG}_eval${v}.log")"
done
