#!/bin/bash
# Round-4 iteration J: class phases without the per-round preamble (affinity tests, C4 digest, diag, bench) and
# the 100k-node bench line on the re-key path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04j}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/${TAG}_$name.log" | cut -c1-900
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_affinity_errors.py tests/test_e2e_ref.py tests/test_gpu_digest.py tests/test_gpu_big.py -k "variants or affinity or e2e or C4 or 100k"
grep "cycle ms" gpurun_out/${TAG}_tests.log | head -2
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so step diag_C4 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval
grep -o '"diag_place_phases": {[^}]*}[^}]*}' gpurun_out/${TAG}_diag_C4.log
step bench_C4 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --no-eval
step bench_100k 300 python bench.py --nodes 100000 --jobs 100 --steps 2 --warmup 1 --no-cpu-baseline --no-eval
step eval 200 python scripts/eval_probe.py 0
step eval2 200 python scripts/eval_probe.py 0
step eval3 200 python scripts/eval_probe.py 0
