#!/bin/bash
# One profiling session per configuration: the rocprofv3 kernel trace (+ stats) of the bench line, then the PMC
# HBM-byte passes (FETCH_SIZE, WRITE_SIZE: one counter per pass), summarised per kernel into
# gpurun_out/<tag>/<tag>_<config>_prof_summary.json (copy into profiles/ to commit).
# Fed-engine configurations take their PMC passes on the per-job launch path (--opt no_fed): counter collection
# serialises dispatches and the resident engine waits on the sweeps; the sweep kernel (sel_sweep_kernel) and its
# launch size are the same on both paths. The C2 pass also carries the kb_eval side measurement (eval_kernel).
# Usage: scripts/profile_round.sh <tag> [configs...]   (default: C1 C2 C3 C4 C5)
# The PMC passes run `--steps 1 --warmup 0 --no-timing`: two allocate cycles (the step and bench.py's host-split
# cycle), which prof_summary.py takes as pmc_cycles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-prof}
shift || true
CONFIGS=${*:-C1 C2 C3 C4 C5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
# ABI 14: the engine is a plain launch in production too (rocprofv3 7.2 segfaulted at exit after the cooperative
# launch rounds 1-4 used), so the profiled cycle is the production cycle. PLAIN=fed_coop_launch: the old launch.
PLAIN=${PLAIN:-none}
run() {  # run <name> <timeout> <cmd...>: stop the script on a crash / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$name.log"; exit $rc; fi
}
for C in $CONFIGS; do
  EVAL="--no-eval"
  [ "$C" = C2 ] && EVAL=""
  run ${C}_trace 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/${C}_trace" -o run --output-format csv -- python3 bench.py --config $C --steps 3 --warmup 1 --no-timing --no-cpu-baseline --no-eval --opt $PLAIN
  NOFED=""
  # FEDPMC=1: the PMC passes on the fed engine itself (its resident sweepers take the commands from a pinned ring:
  # no other-stream dispatch for the profiler's serialisation to stall; the pass counts the engine's one dispatch).
  # Split-engine configurations only (C2, C3, C5): C1's 1k-node table runs the one-workgroup engine, fed by sweep
  # kernels, which the serialisation stalls into its idle exit (r05m)
  [ "$C" != C4 ] && [ "${FEDPMC:-0}" != 1 ] && NOFED=,no_fed
  # (the PMC passes keep the sweep stream in the shared queue pool: with a dedicated CU-masked queue the profiler's
  # serialisation leaves the launch path's place kernel waiting for its overlapped sweep)
  run ${C}_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/${C}_fetch" -o run --output-format csv -- python3 bench.py --config $C --steps 1 --warmup 0 --no-timing --no-cpu-baseline $EVAL --opt $PLAIN,fed_shared_queues$NOFED
  run ${C}_write 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/${C}_write" -o run --output-format csv -- python3 bench.py --config $C --steps 1 --warmup 0 --no-timing --no-cpu-baseline $EVAL --opt $PLAIN,fed_shared_queues$NOFED
  python3 scripts/prof_summary.py "$OUT/${C}_trace" "$OUT/${C}_fetch" "$OUT/${C}_write" "$OUT/${TAG}_${C}_prof_summary.json" 2 > "$OUT/sum_${C}.log" 2>&1
  rm -rf "$OUT/${C}_fetch" "$OUT/${C}_write"  # raw per-dispatch CSVs: large, summarised above
done
find "$OUT" -name "*kernel_trace.csv" -delete
echo "=== done"
