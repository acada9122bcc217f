#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so timeout -k 10 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval > gpurun_out/r04g_diag_C4.log 2>&1
rc=$?; grep -o '"diag_place_phases": {[^}]*}[^}]*}' gpurun_out/r04g_diag_C4.log; exit $rc
