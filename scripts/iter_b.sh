#!/bin/bash
# Round-4 iteration B: the class loop's phases (affinity variants, C4 digest, C4 bench) and the C2 host trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04b}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: a crash / timeout ends the script (test failures, exit 1, do not)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/${TAG}_$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_affinity_errors.py tests/test_e2e_ref.py tests/test_gpu_digest.py -k "variants or affinity or e2e or C4"
step bench_C4 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --no-eval
KB_HOST_TRACE=1 step trace_C2 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-eval
