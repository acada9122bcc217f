#!/bin/bash
# Round-4 iteration E: class-phase diag counters on C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so timeout -k 10 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval > gpurun_out/r04e_diag_C4.log 2>&1
rc=$?; grep -o '"diag_place_phases": {[^}]*}[^}]*}' gpurun_out/r04e_diag_C4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/eval_probe.py 0 8 12 16 20 26 32 > gpurun_out/r04e_eval.log 2>&1 || exit $?
cat gpurun_out/r04e_eval.log
