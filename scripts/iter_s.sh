#!/bin/bash
# Small-block sharded engine diagnosis: 3 ranks, the sharded parity test's sequence of contexts, repeated, traced.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
PROBE_REPEAT=${PROBE_REPEAT:-4} timeout -k 10 300 python scripts/shard_small_probe.py ssp4 3 all > gpurun_out/ssp4.log 2>&1
echo "rc=$?"; grep -c ": ok" gpurun_out/ssp4.log; grep "rank" gpurun_out/ssp4.log | grep -v ": ok\|Gloo" | head
