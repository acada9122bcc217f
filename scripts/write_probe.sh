#!/bin/bash
# Write-request breakdown of the C2 engine dispatch: TCC counters in passes of at most four, on the
# production cycle (A) and without level records (B), plus the calibration kernels. Output: gpurun_out/<TAG>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-wp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
BENCH="bench.py --config C2 --steps 1 --warmup 0 --no-timing --no-cpu-baseline --no-eval"
P1="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WR_UNCACHED_32B_sum TCC_EA0_WRREQ_WRITE_IO_32B_sum"
P2="TCC_ALL_TC_OP_WB_WRITEBACK_sum TCC_NORMAL_WRITEBACK_sum TCC_NORMAL_EVICT_sum TCC_EA0_WRREQ_WRITE_DRAM_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  for v in prod nolvl; do
    opt=fed_shared_queues
    [ $v = nolvl ] && opt=$opt,fed_no_levels
    timeout -s KILL 300 rocprofv3 --pmc $P -d "$PWD/$OUT/${v}_p$i" -o run --output-format csv -- python3 $BENCH --opt $opt > "$OUT/${v}_p$i.log" 2>&1 || exit $?
    echo "=== ${v}_p$i ok"
  done
  timeout -s KILL 120 rocprofv3 --pmc $P -d "$PWD/$OUT/wcal_p$i" -o run --output-format csv -- scripts/build/wcal > "$OUT/wcal_p$i.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, os, re, sys, json
out = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(out, "*_p[12]"))):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            m = re.search(r"kbgpu::(\w+)", name) or re.search(r"(\w+)\(", name)
            k = m.group(1) if m else name
            if k not in ("fed_engine_kernel", "w_plain16", "w_at8_scatter", "w_plain4"):
                continue
            per.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    res[os.path.basename(d)] = {k: {c: sorted(v)[len(v) // 2] for c, v in cs.items()} for k, cs in per.items()}
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out, "write_probe.json"), "w"), indent=1)
PY
find "$OUT" -name "*.csv" -size +2M -delete
