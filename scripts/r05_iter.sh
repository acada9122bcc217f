#!/bin/bash
# Round-5 iteration: the fed-engine / split / mixed / digest parity tests (any failure ends the script), the C2 line
# (20 steps) twice, the KB_DIAG placer stamps, and the C5 / C2M lines. TAG names the outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05f}
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: any non-zero exit ends the script
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 1 "gpurun_out/${TAG}_$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
pick() { grep -o '"value": [0-9.]*\|"us_per_job": [0-9.]*\|"ms_per_step": [0-9.]*' "gpurun_out/${TAG}_$1.log" | tr '\n' ' '; echo; }
step tests 900 python -u -m pytest -m gpu -v -x -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_digest.py tests/test_gpu_shard_peer.py tests/test_gpu_fed_queues.py \
  -k "${K:-mixed or pipeline_parity or takes_long or fed_split or survives or full_size or peer_engine or progress}"
for i in 1 2 3; do step b2_$i 200 python bench.py --steps 20 --warmup 2 --no-eval --no-cpu-baseline; pick b2_$i; done
KBGPU_LIB=scheduler_amd/libkbgpu_diag.so step diag2 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-eval --opt fed_diag
grep -h "kb_fed_timeline\|kb_fed_placer_fine\|kb_fed_late\|kb_fed_host\|kb_fed_placer_merge" "gpurun_out/${TAG}_diag2.log" | tail -5; grep -o '"diag_place_phases": {[^}]*}' "gpurun_out/${TAG}_diag2.log"
step b5 300 python bench.py --config C5 --steps 3 --warmup 1 --no-eval --no-cpu-baseline; pick b5
step b2m 300 python bench.py --config C2M --steps 10 --warmup 2 --no-eval --no-cpu-baseline; pick b2m
step b3 300 python bench.py --config C3 --steps 5 --warmup 1 --no-eval --no-cpu-baseline; pick b3
if [ -n "${EVALP:-}" ]; then
  step evalp 200 python scripts/eval_probe.py 0; cat "gpurun_out/${TAG}_evalp.log"
  for v in evalso evalt; do
    KBGPU_LIB=scheduler_amd/libkbgpu_$v.so step evalp_$v 200 python scripts/eval_probe.py 0; cat "gpurun_out/${TAG}_evalp_$v.log"
  done
fi
echo "=== done"
