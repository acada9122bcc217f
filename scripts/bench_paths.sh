#!/bin/bash
# bench every device path once (C2), each under its own time limit; stops at the first crash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for p in ${PATHS:-engine select}; do
  timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --path $p > gpurun_out/bench_$p.log 2>&1
  rc=$?; echo "=== $p rc=$rc"; tail -n 2 gpurun_out/bench_$p.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  if [ -n "${DIAG:-}" ]; then
    KBGPU_LIB=scheduler_amd/libkbgpu_diag.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --path $p > gpurun_out/bench_diag_$p.log 2>&1 || exit $?
  fi
done
