#!/bin/bash
# one bench line per BASELINE configuration on one GPU (each under its own time limit)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-C1 C3 C4}; do
  timeout -k 10 500 python bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${EXTRA:-} > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "=== $c rc=$rc"; grep '^{' gpurun_out/bench_$c.log | head -c 1200; echo
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
