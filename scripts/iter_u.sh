#!/bin/bash
# Round-4 iteration U: C2 host split (KB_HOST_TRACE) and the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
KB_HOST_TRACE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-eval --no-cpu-baseline > gpurun_out/r04u_trace_C2.log 2>&1
echo "rc=$?"; grep "kb_host_trace" gpurun_out/r04u_trace_C2.log | tail -4; grep -i "spec\|fin\|apply\|iter" gpurun_out/r04u_trace_C2.log | grep -v "^{" | tail -6 | cut -c1-300
