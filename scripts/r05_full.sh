#!/bin/bash
# Round-5 full check on the GPU box: the whole -m gpu suite, smoke(), and the bench lines C2, C2M (mixed cycle),
# C4, C3, C5 (TAG names the outputs under gpurun_out/). A crash / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05b}
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/${TAG}_$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests 1000 python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 900 --timeout-method thread ${TESTS:-tests}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
for C in ${CONFIGS:-C2 C2M C4 C3 C5}; do
  step bench_$C 400 python bench.py --config $C --steps 10 --warmup 2 --no-eval --no-cpu-baseline
done
KB_HOST_TRACE=1 step trace_C2M 300 python bench.py --config C2M --steps 2 --warmup 1 --no-eval --no-cpu-baseline --no-timing

if [ "${AB:-1}" = 1 ]; then  # the engine's launch, A/B on one box: plain (production) / cooperative, alternating
  for i in 1 2; do
    step ab_plain_$i 200 python bench.py --steps 20 --warmup 2 --no-eval --no-cpu-baseline
    step ab_coop_$i 200 python bench.py --steps 20 --warmup 2 --no-eval --no-cpu-baseline --opt fed_coop_launch
  done
fi
echo "=== done"
