#!/bin/bash
# Round-4 iteration A: the tests touched by the kb_opts switches and the inbox epoch wrap, the cross-process C2
# spread probe, and the C2 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04a}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: a crash / timeout ends the script (test failures, exit 1, do not)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_shard_peer.py tests/test_gpu_fed_queues.py tests/test_gpu_parity.py -k "peer or queues or hazard or pipeline or variants or stall or split or eval_plain"
step digest 600 python -u -m pytest -m gpu -v -rf -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_digest.py -k "C4 or C2"
step bench_C4 300 python bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --no-eval
step spread 400 python scripts/spread_probe.py --runs 5 --steps 8 --pin none,local,remote
step bench_C2 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline
