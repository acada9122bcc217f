#!/bin/bash
# Final-build bench lines of every configuration (default bench.py run: timed steps, the eval side measurement on
# C2, the CPU baseline), one log per configuration under gpurun_out/<TAG>_<config>.log; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-final}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for C in ${CONFIGS:-C1 C2 C3 C4 C5 C2M}; do
  timeout -k 10 400 python bench.py --config "$C" > "gpurun_out/${TAG}_$C.log" 2>&1
  rc=$?
  echo "=== $C rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "gpurun_out/${TAG}_$C.log"; exit $rc; fi
  grep "^{" "gpurun_out/${TAG}_$C.log" | tail -1 | cut -c1-220
done
echo "=== done"
