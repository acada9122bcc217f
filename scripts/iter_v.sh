#!/bin/bash
# Round-4 iteration V: reused result buffers (C2 step), bulk merge without the flush in its loop (C4).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04v}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_digest.py -k "reused or variants or affinity or C4 or C2 or pipeline or e2e"
step bench_C2 300 python bench.py --steps 20 --warmup 2 --no-eval --no-cpu-baseline
step bench_C4 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --no-eval
