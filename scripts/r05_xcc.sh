#!/bin/bash
# Round 5: the mixed-cycle tests (stop on ANY failure: a fault there must not be repeated by the benches), the C2M
# line, and the C2 line with the split engine's workgroups placed on each XCC in turn (option fed_xcc=k+1; 0: where
# the dispatcher puts them). TAG names the outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05c}
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: any non-zero exit ends the script
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/${TAG}_$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "${K:-mixed or pipeline_parity or takes_long or fed_split or overlap}"
step b2m 300 python bench.py --config C2M --steps 10 --warmup 2 --no-eval --no-cpu-baseline
for X in ${XCCS:-0 1 2 3 4 5 6 7 8}; do
  step b2_xcc$X 200 python bench.py --steps 10 --warmup 2 --no-eval --no-cpu-baseline --opt fed_xcc=$X
  grep -o '"us_per_job": [0-9.]*, "clock_mhz": [0-9.]*, "placement": {[^}]*}, "selector": {[^}]*}' "gpurun_out/${TAG}_b2_xcc$X.log"
done
echo "=== done"
