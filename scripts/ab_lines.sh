#!/bin/bash
# A/B bench lines on one GPU box: LINES is a space-separated list of name:config:options[:steps] (options as bench.py
# --opt takes them, "-" for the production path; KBGPU_LIB=<lib> prefixes are not supported here -- use LIBLINES,
# name:lib:config:options[:steps], for variant builds). Optional TESTS (pytest -k expression) runs the named GPU tests
# first; a failed test ends the script. Each line's summary (pods/s, ms per step, engine us per job, depth, sweepers,
# mispredicts) is printed; the JSON lines stay in gpurun_out/<TAG>_<name>.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-ab}
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: any non-zero exit ends the script
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "=== $name rc=$rc"; tail -n 5 "gpurun_out/${TAG}_$name.log" | cut -c1-400; exit $rc; fi
}
summ() {
  python3 - "gpurun_out/${TAG}_$1.log" "$1" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
e = d.get("engine") or {}
print(f"{sys.argv[2]:>14} {d['config']['workload'][:18]:>18} {d['value']/1e6:7.3f} M/s {d['ms_per_step']:8.3f} ms "
      f"p50 {d['p50_cycle_ms']:8.3f}  us/job {e.get('us_per_job')} depth {e.get('depth')} sw {e.get('sweepers')} "
      f"mis/step {e.get('mispredicts_per_step')} skip/step {e.get('skipped_per_step')} "
      f"roof {d['roofline']['kernel']} {d['roofline']['avg_launch_us']}")
EOF
}
if [ -n "${TESTS:-}" ]; then
  step tests 900 python -u -m pytest -m gpu -v -s -x -p no:cacheprovider --timeout 600 --timeout-method thread tests -k "$TESTS"
  grep -E "passed|failed" "gpurun_out/${TAG}_tests.log" | tail -1
fi
for spec in ${LINES:-}; do
  IFS=: read -r name cfg opt steps <<< "$spec"
  [ "$opt" = "-" ] && opt=""
  step "$name" 300 python bench.py --config "$cfg" --steps "${steps:-10}" --warmup 2 --no-eval --no-cpu-baseline --opt "$opt"
  summ "$name"
done
for spec in ${LIBLINES:-}; do
  IFS=: read -r name lib cfg opt steps <<< "$spec"
  [ "$opt" = "-" ] && opt=""
  KBGPU_LIB="$lib" step "$name" 300 python bench.py --config "$cfg" --steps "${steps:-10}" --warmup 2 --no-eval \
    --no-cpu-baseline --opt "$opt"
  summ "$name"
  grep -h "kb_fed_timeline\|kb_fed_late\|kb_fed_host" "gpurun_out/${TAG}_$name.log" | cut -c1-600 | tail -3
done
echo "=== done"
