#!/bin/bash
# Round-4 iteration Y: host cycle setup (CSR pending lists): driver parity tests, C2 trace and bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_digest.py -k "pipeline or C2 or C1 or reused or partial or gang" > gpurun_out/r04y_tests.log 2>&1
echo "tests rc=$?"; tail -1 gpurun_out/r04y_tests.log
KB_HOST_TRACE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-eval --no-cpu-baseline > gpurun_out/r04y_trace_C2.log 2>&1
grep "pre_ms\|init_ms" gpurun_out/r04y_trace_C2.log | sed -n 3,6p
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-eval --no-cpu-baseline > gpurun_out/r04y_bench_C2.log 2>&1
echo "bench rc=$?"; grep -o '"value": [0-9.]*' gpurun_out/r04y_bench_C2.log | head -1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04y_bench_C2.log | head -1; grep -o '"host_ms_per_step": {[^}]*}' gpurun_out/r04y_bench_C2.log
