#!/bin/bash
# Round-5 iteration on the GPU box: the tests touched this round, the C2 line on the production (plain) engine
# launch and on the old cooperative one (A/B), and a rocprofv3 kernel trace of the unmodified production C2 bench.
# TAG names the outputs under gpurun_out/. Any crash / timeout ends the script (test failures, exit 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05a}
K=${K:-overlap or pipeline_parity or fed_split or loop_variants or survives or peer or progress or hazard or mixed}
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests 700 python -u -m pytest -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_shard_peer.py tests/test_gpu_fed_queues.py -k "$K"
fi
step b2 200 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-eval
step b2m 300 python bench.py --config C2M --steps 10 --warmup 2 --no-cpu-baseline --no-eval
step b2coop 200 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-eval --opt fed_coop_launch
step trace 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/${TAG}_trace" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-eval
find "gpurun_out/${TAG}_trace" -name "*kernel_trace.csv" -delete
echo "=== done"
