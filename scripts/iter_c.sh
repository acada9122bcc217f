#!/bin/bash
# Round-4 iteration C: the new bench lines (C2, C4, C1, C3), the 2-rank shared-GPU rehearsal of the sharded C2 line,
# and one rocprofv3 kernel trace of C2 with the engine's cooperative launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04c}
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: a crash / timeout ends the script (test failures, exit 1, do not)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/${TAG}_$name.log" | cut -c1-3000
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step bench_C2 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline
step bench_C4 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --no-eval
KBGPU_LIB=scheduler_amd/libkbgpu_diagaff.so step diag_C4 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-eval
step bench_C1 300 python bench.py --config C1 --steps 5 --warmup 1 --no-cpu-baseline --no-eval
step bench_C3 300 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-eval
step rehearse2 400 python bench.py --gpus 2 --same-gpu --steps 3 --warmup 1 --no-cpu-baseline --side-steps 2
step trace_coop 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/${TAG}_trace" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-timing --no-cpu-baseline --no-eval
find gpurun_out/${TAG}_trace -name "*kernel_trace.csv" -delete
