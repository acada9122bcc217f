#!/bin/bash
# One profiling session: rocprofv3 kernel trace (+ stats) of the C2 headline bench and of the C4 bench, and
# the PMC HBM-byte passes (FETCH_SIZE, WRITE_SIZE: one counter per pass) of each, summarised per kernel.
# C2's PMC passes take the per-job launch path (KB_NO_FED=1): counter collection serialises dispatches,
# which the resident engine cannot run under. Usage: scripts/profile_round.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() {  # run <name> <timeout> <cmd...>: stop the script on a crash / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$name.log"; exit $rc; fi
}
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-eval"
run c2_trace 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/c2_trace" -o run --output-format csv -- python3 $B
run c4_trace 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/c4_trace" -o run --output-format csv -- python3 $B --config C4
run c4_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/c4_fetch" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-eval --config C4
run c4_write 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/c4_write" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-eval --config C4
export KB_NO_FED=1
run c2_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/c2_fetch" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
run c2_write 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/c2_write" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
unset KB_NO_FED
python3 scripts/prof_summary.py "$OUT/c2_trace" "$OUT/c2_fetch" "$OUT/c2_write" "$OUT/${TAG}_prof_summary.json" > "$OUT/sum_c2.log" 2>&1
python3 scripts/prof_summary.py "$OUT/c4_trace" "$OUT/c4_fetch" "$OUT/c4_write" "$OUT/${TAG}_C4_prof_summary.json" > "$OUT/sum_c4.log" 2>&1
rm -rf "$OUT"/c2_fetch "$OUT"/c2_write "$OUT"/c4_fetch "$OUT"/c4_write  # raw per-dispatch CSVs: large, summarised above
find "$OUT" -name "*kernel_trace.csv" -delete
echo "=== done"
