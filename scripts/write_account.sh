#!/bin/bash
# The fed engine's write accounting, on the GPU box:
#   1. the store-form calibration (scripts/build/wcal: known byte counts per kernel) under rocprofv3 --pmc WRITE_SIZE;
#   2. the production C2 cycle's engine dispatch under WRITE_SIZE, and A/B passes that each drop one writer: the level
#      records (option fed_no_levels) and the committed rows (libkbgpu_wanorows.so, -DKB_WA_NO_ROWS);
#   3. scripts/write_account.py: the per-writer table (store counts per job x calibrated bytes per store) against the
#      measured WRITE_SIZE per job, into gpurun_out/<TAG>/write_account.json.
# Build first (here): make -C scheduler_amd/csrc all wanorows; hipcc --offload-arch=gfx950 -O3 -o scripts/build/wcal
# scripts/wcal.hip.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-wa}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() {  # run <name> <timeout> <cmd...>: stop on a crash / timeout
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/$name.log"; exit $rc; fi
}
run wcal 120 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/wcal" -o run --output-format csv -- scripts/build/wcal
BENCH="bench.py --config C2 --steps 1 --warmup 0 --no-timing --no-cpu-baseline --no-eval"
run prod 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/prod" -o run --output-format csv -- python3 $BENCH --opt fed_shared_queues
run nolvl 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/nolvl" -o run --output-format csv -- python3 $BENCH --opt fed_shared_queues,fed_no_levels
KBGPU_LIB=scheduler_amd/libkbgpu_wanorows.so run norows 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/norows" -o run --output-format csv -- python3 $BENCH --opt fed_shared_queues
for v in noacq noswrows noswst; do  # (A/B builds: make -C scheduler_amd/csrc wasw)
  [ -f scheduler_amd/libkbgpu_wa$v.so ] && KBGPU_LIB=scheduler_amd/libkbgpu_wa$v.so run $v 300 rocprofv3 --pmc WRITE_SIZE \
    -d "$PWD/$OUT/$v" -o run --output-format csv -- python3 $BENCH --opt fed_shared_queues
done
run fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/fetch" -o run --output-format csv -- python3 $BENCH --opt fed_shared_queues
python3 scripts/write_account.py "$OUT" > "$OUT/write_account.log" 2>&1
cat "$OUT/write_account.log"
find "$OUT" -name "*.csv" -size +2M -delete
echo "=== done"
