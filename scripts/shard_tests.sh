#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 bash scripts/probe_small.sh && \
timeout -k 10 900 python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 400 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_shard_peer.py > gpurun_out/r04fix_tests.log 2>&1
echo "tests rc=$?"; grep -E "^E |passed|failed" gpurun_out/r04fix_tests.log | cut -c1-300 | tail -5
