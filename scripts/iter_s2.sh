#!/bin/bash
# Small-block sharded engine diagnosis: every context in fresh processes (3 ranks, 7 cases x 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
PROBE_REPEAT=2 timeout -k 10 500 python scripts/shard_small_probe.py ssp5 3 fresh > gpurun_out/ssp5.log 2>&1
echo "rc=$?"; grep -c ": ok" gpurun_out/ssp5.log; grep "rank" gpurun_out/ssp5.log | grep -v ": ok\|Gloo" | head
