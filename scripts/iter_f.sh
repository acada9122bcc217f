#!/bin/bash
# Round-4 iteration F: the class phases' hot-node rounds (affinity tests, C4 digest, diag, bench) and the eval A/B
# (non-temporal vs plain stores; specs per block).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04f}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/${TAG}_$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_affinity_errors.py tests/test_e2e_ref.py tests/test_gpu_digest.py -k "variants or affinity or e2e or C4"
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so step diag_C4 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval
grep -o '"diag_place_phases": {[^}]*}[^}]*}' gpurun_out/${TAG}_diag_C4.log
step bench_C4 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --no-eval
step eval_nt 200 python scripts/eval_probe.py 0 26 32
KBGPU_LIB=scheduler_amd/libkbgpu_evalt.so step eval_t 200 python scripts/eval_probe.py 0 26 32
step eval_nt2 200 python scripts/eval_probe.py 0 26 32
cat gpurun_out/${TAG}_eval_*.log
