#!/bin/bash
# The node-sharded engine on small blocks: 3 ranks on one GPU, the sharded parity test's sequence of contexts
# repeated in the same processes (scripts/shard_small_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
PROBE_REPEAT=${PROBE_REPEAT:-4} timeout -k 10 400 python scripts/shard_small_probe.py ssps 3 all > gpurun_out/ssps.log 2>&1
echo "rc=$?"; grep -o "[A-Za-z0-9.-]*: ok" gpurun_out/ssps.log | wc -l; grep "rank" gpurun_out/ssps.log | grep -v ": ok\|Gloo" | head -5
