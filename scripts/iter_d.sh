#!/bin/bash
# Round-4 iteration D: the class loop's 32-bit phases (affinity tests, C4 digest, C4 diag + bench), and the C2
# profile (kernel trace with the plain engine launch + PMC passes with dispatch counts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04d}
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: a crash / timeout ends the script (test failures, exit 1, do not)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/${TAG}_$name.log" | cut -c1-1800
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_affinity_errors.py tests/test_e2e_ref.py tests/test_gpu_digest.py -k "variants or affinity or e2e or C4"
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so step diag_C4 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval
step bench_C4 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --no-eval
step prof_C2 600 bash scripts/profile_round.sh r04d C2
