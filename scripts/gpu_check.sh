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
  step gpu_tests 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps ${STEPS:-5} --warmup 1
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- \
       python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
fi
echo "=== done"
