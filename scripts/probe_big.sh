#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
PROBE_REPEAT=10 timeout -k 10 400 python scripts/shard_small_probe.py sspbig 3 big > gpurun_out/sspbig.log 2>&1
echo "rc=$?"; grep -o "c2big[0-9]*: ok[^r]*" gpurun_out/sspbig.log | wc -l; grep "rank" gpurun_out/sspbig.log | grep -v ": ok\|Gloo" | head -5
