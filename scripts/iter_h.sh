#!/bin/bash
# Round-4 iteration H: class-phase stretches with the deep keys between passes (affinity tests, C4 digest, diag,
# bench), the C2 engine's phase stamps, and the C2 bench with the cached session struct.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04h}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/${TAG}_$name.log" | cut -c1-1200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_affinity_errors.py tests/test_e2e_ref.py tests/test_gpu_digest.py tests/test_gpu_big.py -k "variants or affinity or e2e or C4 or C2 or 100k"
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so step diag_C4 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval
grep -o '"diag_place_phases": {[^}]*}[^}]*}' gpurun_out/${TAG}_diag_C4.log
step bench_C4 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --no-eval
KBGPU_LIB=scheduler_amd/libkbgpu_diag.so step diag_C2 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-eval --opt fed_diag
grep -h "kb_fed" gpurun_out/${TAG}_diag_C2.log | tail -2; grep -o '"diag_place_phases": {[^}]*}' gpurun_out/${TAG}_diag_C2.log
step bench_C2 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-eval
step bench_C2_plain 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-eval --opt fed_plain_launch
TAG=r04h_evalmodes bash scripts/eval_modes.sh > gpurun_out/r04h_evalmodes.log 2>&1; tail -5 gpurun_out/r04h_evalmodes.log
