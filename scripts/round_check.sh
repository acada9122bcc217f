#!/bin/bash
# Round check on the GPU box: the whole -m gpu suite, smoke(), and the bench lines of every configuration
# (C2 headline with eval + cpu baseline; C1, C3, C4, C5), into gpurun_out/<TAG>_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-check}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: a crash / timeout ends the script (test failures, exit 1, do not)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  # -v -s: every test's name as it starts, and the long tests' heartbeats (a silent call is taken to be hung)
  step tests 1000 python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 900 --timeout-method thread tests
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_C2 400 python bench.py --steps 20 --warmup 2
for C in C1 C3 C4 C5; do
  step bench_$C 400 python bench.py --config $C --steps 5 --warmup 1 --no-eval
done
