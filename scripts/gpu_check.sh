#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace. Each GPU step has its own time
# limit; a crash / fault / timeout ends the script (test failures, exit 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export PYTHONUNBUFFERED=1
step() {  # step <name> <timeout-seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step gpu_tests ${TEST_TIMEOUT:-1000} python -u -m pytest -m gpu -v -p no:cacheprovider --maxfail=${MAXFAIL:-25} --timeout 300 --timeout-method thread ${TESTS:-tests}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps ${STEPS:-5} --warmup 1
fi
if [ "$MODE" = diag ]; then  # phase cycle counts of the place loop (KB_DIAG build)
  KBGPU_LIB=scheduler_amd/libkbgpu_diag.so step bench_diag 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline
fi
if [ "$MODE" = diagsel ]; then  # node-selection sub-phases of the selection kernel (KB_DIAG_SEL build)
  KBGPU_LIB=scheduler_amd/libkbgpu_diagsel.so step bench_diagsel 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --path select
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- \
       python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
  # HBM bytes per launch: one counter per pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
  # Counter collection serialises dispatches, which the resident fed engine cannot run under (it waits for
  # sweep kernels on another stream): these passes take the per-job launch path (KB_NO_FED=1).
  export KB_NO_FED=1
  export TMPDIR=/tmp
  step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- \
       python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
  step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- \
       python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
  unset KB_NO_FED
  python3 scripts/prof_summary.py "$OUT/prof" "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/prof_summary.json" \
       > "$OUT/prof_summary.log" 2>&1; echo "=== prof_summary rc=$?"
fi
if [ "$MODE" = cpubase ]; then  # the oracle's CPU baselines for every config on the box's host cores
  step cpubase 1100 python3 scripts/cpu_baselines.py "$OUT/cpu_baselines.json"
fi
echo "=== done"
