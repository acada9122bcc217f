#!/bin/bash
# kb_eval's two per-process timing modes: several processes of the eval probe, each under rocprofv3
# with the UTCL1 (address translation) counters and the kernel trace, so every process's eval_plain_kernel
# durations sit beside its translation misses per request. The profiled process is the measuring one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-evalmodes}
mkdir -p $OUT
for i in 1 2 3 4; do
  timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --kernel-trace -d $PWD/$OUT/p$i -o run --output-format csv -- python3 scripts/eval_probe.py --batches 2 --per 5 > $OUT/p$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
res = []
for i in (1, 2, 3, 4):
    d = os.path.join(out, f"p{i}")
    dur = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "eval_plain_kernel" in r.get("Kernel_Name", ""):
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "eval_plain_kernel" in r.get("Kernel_Name", ""):
                ctr.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    dur.sort()
    e = {"process": i, "launches": len(dur), "median_us": dur[len(dur) // 2] if dur else None,
         **{k: sum(v) / len(v) for k, v in ctr.items()}}
    if e.get("TCP_UTCL1_REQUEST_sum"):
        e["miss_per_request"] = e.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0) / e["TCP_UTCL1_REQUEST_sum"]
    res.append(e)
    print(json.dumps(e))
json.dump(res, open(os.path.join(out, "eval_modes.json"), "w"), indent=1)
PY
find $OUT -name "*.csv" -size +2M -delete
