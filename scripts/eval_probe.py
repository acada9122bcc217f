"""Probe: bench.py's kb_eval side measurement (256 plain specs x 50k nodes through kb_eval32, HIP events around the
kernel) repeated in batches, per eval_plain_kernel specs-per-block value (kb_opts.eval_spb; 0 = the launcher's own
choice from the device's CU count). One process, one context per value; prints one JSON line per value: the median
and minimum of the batches' average launch time. The measuring process is the profiled one (scripts/pmc_eval.sh).
Usage: python3 scripts/eval_probe.py [--batches B] [--per P] [SPB ...]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(spb, batches, per):
    import bench
    from scheduler_amd import runtime, synth
    snap = synth.c2_snapshot(n_nodes=bench.EVAL_NODES, n_jobs=bench.EVAL_SPECS, tasks_per_job=1, seed=synth.SEED)
    ctx = runtime.Context(0, timing=True, options={"eval_spb": spb})
    ctx.upload(snap)
    ids = (np.arange(bench.EVAL_SPECS) % len(snap.spec_arr)).astype(np.int32)
    for _ in range(3):
        ctx.eval32(ids)
    k = runtime.KERNELS.index("eval_kernel")
    us = []
    for _ in range(batches):
        ctx.stats(reset=True)
        for _ in range(per):
            ctx.eval32(ids)
        st = ctx.stats()
        us.append(st["kernel_ms"][k] * 1e3 / max(1, st["launches"][k]))
    ctx.close()
    alg = len(ids) * bench.EVAL_NODES * bench.EVAL_OUT_BYTES + bench.EVAL_NODES * 76
    med = float(np.median(us))
    print(json.dumps({"eval_spb": spb or "auto", "median_us": round(med, 3), "min_us": round(min(us), 3),
                      "frac_median": round(alg / (med * 1e-6) / 1e9 / bench.HBM_PEAK_GBS, 4),
                      "plain": bench.snap_plain(snap, ids)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=12)
    ap.add_argument("--per", type=int, default=10)
    ap.add_argument("spb", nargs="*", type=int)
    a = ap.parse_args()
    for v in a.spb or [0]:
        one(v, a.batches, a.per)
    return 0


if __name__ == "__main__":
    sys.exit(main())
