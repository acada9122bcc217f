#!/bin/bash
# Round-4 iteration N: class-loop stamps per round part (C4 diag line only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04n}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so timeout -k 10 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval > gpurun_out/${TAG}_diag_C4.log 2>&1
echo "rc=$?"; grep -o '"diag_place_phases": {[^}]*}[^}]*}' gpurun_out/${TAG}_diag_C4.log
