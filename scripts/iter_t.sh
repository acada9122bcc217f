#!/bin/bash
# Round-4 iteration T: the C2 bench line with the eval side measurement after a long warm-up.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/r04t_bench_C2.log 2>&1
echo "rc=$?"; grep -o '"eval_roofline": {[^}]*}' gpurun_out/r04t_bench_C2.log; grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r04t_bench_C2.log | head -1
