#!/bin/bash
# SQ counters of kb_eval's eval_kernel (scripts/eval_probe.py: 256 specs x 50k nodes), one pass per group
# (rocprofv3 takes at most 8 SQ counters per pass): instructions per wave by kind and where the waves wait.
# The profiled process is the measuring one (eval_probe.py starts no other program) at the launcher's own grid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_eval}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/trace -o run --output-format csv -- python3 scripts/eval_probe.py --batches 5 > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH -d $PWD/$OUT/p1 -o run --output-format csv -- python3 scripts/eval_probe.py --batches 1 --per 2 > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_TRANS_F32 -d $PWD/$OUT/p2 -o run --output-format csv -- python3 scripts/eval_probe.py --batches 1 --per 2 > $OUT/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $PWD/$OUT/p3 -o run --output-format csv -- python3 scripts/eval_probe.py --batches 1 --per 2 > $OUT/p3.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $PWD/$OUT/p4 -o run --output-format csv -- python3 scripts/eval_probe.py --batches 1 --per 2 > $OUT/p4.log 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
res = {}
for d in ("p1", "p2", "p3", "p4"):
    for f in glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True):
        per = {}
        for row in csv.DictReader(open(f)):
            if not any(k in row.get("Kernel_Name", "") for k in ("eval_kernel", "eval_plain_kernel")):
                continue
            k = (row["Counter_Name"], row["Dispatch_Id"])
            per[k] = per.get(k, 0.0) + float(row["Counter_Value"])
        agg = {}
        for (name, _), v in per.items():
            agg.setdefault(name, []).append(v)
        for name, vs in agg.items():
            res[name] = sum(vs) / len(vs)
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "eval_kernel" in row["Name"] or "eval_plain_kernel" in row["Name"]:
            res["avg_ns"] = float(row["AverageNs"])
pairs = 256 * 50000
res["pairs"] = pairs
if "SQ_INSTS_VALU" in res:
    res["valu_lane_ops_per_pair"] = res["SQ_INSTS_VALU"] * 64 / pairs
if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
    res["hbm_bytes_per_launch"] = (2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024
json.dump(res, open(os.path.join(out, "eval_counters.json"), "w"), indent=1)
print(json.dumps(res))
PY
