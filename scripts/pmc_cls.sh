#!/bin/bash
# SQ / SQC counters of the class loop (cls_place_kernel) on C4: instruction-cache hits and misses beside the wave's
# busy, waiting and instruction counts, per launch (one pass; two allocate cycles: the step + the host split).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_cls}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $PWD/$OUT/p1 -o run --output-format csv -- python3 bench.py --config C4 --steps 1 --warmup 0 --no-timing --no-cpu-baseline --no-eval > $OUT/p1.log 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
agg = {}
for f in glob.glob(os.path.join(out, "p1", "**", "*counter_collection.csv"), recursive=True):
    per = {}
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        name = "cls_place_kernel" if "cls_place_kernel" in k else ("sel_place_kernel" if "sel_place_kernel" in k else None)
        if name is None:
            continue
        per.setdefault((name, r["Counter_Name"]), {}).setdefault(r["Dispatch_Id"], 0.0)
        per[(name, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for (name, c), d in per.items():
        agg.setdefault(name, {})[c] = sum(d.values()) / len(d)
        agg[name]["dispatches"] = len(d)
print(json.dumps(agg, indent=1))
json.dump(agg, open(os.path.join(out, "cls_counters.json"), "w"), indent=1)
PY
find $OUT -name "*.csv" -delete
