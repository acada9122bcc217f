#!/bin/bash
# Quick diag round: the split-engine parity tests, then the KB_DIAG C2 line with the per-job timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05d}
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "${K:-fed_split}" > "gpurun_out/${TAG}_tests.log" 2>&1 || { tail -5 "gpurun_out/${TAG}_tests.log"; exit 1; }
tail -1 "gpurun_out/${TAG}_tests.log"
KBGPU_LIB=scheduler_amd/libkbgpu_diag.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-eval \
  --opt fed_diag > "gpurun_out/${TAG}_diag2.log" 2>&1 || { tail -5 "gpurun_out/${TAG}_diag2.log"; exit 1; }
grep -h "kb_fed_" "gpurun_out/${TAG}_diag2.log" | tail -5
KBGPU_LIB=scheduler_amd/libkbgpu_tl.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-eval \
  --opt fed_diag > "gpurun_out/${TAG}_tl2.log" 2>&1 || { tail -5 "gpurun_out/${TAG}_tl2.log"; exit 1; }
grep -h "kb_fed_timeline\|kb_fed_host" "gpurun_out/${TAG}_tl2.log" | tail -2
grep -o '"us_per_job": [0-9.]*' "gpurun_out/${TAG}_tl2.log"
timeout -k 10 200 python bench.py --steps 20 --warmup 2 --no-eval --no-cpu-baseline > "gpurun_out/${TAG}_b2.log" 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"us_per_job": [0-9.]*' "gpurun_out/${TAG}_b2.log" | tr '\n' ' '; echo
