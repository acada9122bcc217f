"""Probe: bench.py's kb_eval side measurement (256 plain specs x 50k nodes through kb_eval32, HIP events around the
kernel) repeated in batches, for eval_plain_kernel's specs per block (KB_EVAL_SPB, read once per process: one
process per value). Prints one JSON line per value: the median and minimum of the batches' average launch time.
Usage: python3 scripts/eval_probe.py [SPB ...]   (no arguments: the launcher's own choice)"""
import json
import os
import subprocess
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(batches=12, per=10):
    import bench
    from scheduler_amd import runtime, synth
    snap = synth.c2_snapshot(n_nodes=bench.EVAL_NODES, n_jobs=bench.EVAL_SPECS, tasks_per_job=1, seed=synth.SEED)
    ctx = runtime.Context(0, timing=True)
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
    print(json.dumps({"KB_EVAL_SPB": os.environ.get("KB_EVAL_SPB", "auto"), "median_us": round(med, 3),
                      "min_us": round(min(us), 3), "frac_median": round(alg / (med * 1e-6) / 1e9 / bench.HBM_PEAK_GBS, 4),
                      "plain": bench.snap_plain(snap, ids)}), flush=True)


def main():
    if os.environ.get("KB_EVAL_PROBE_CHILD"):
        one()
        return 0
    for v in sys.argv[1:] or ["auto"]:
        env = dict(os.environ, KB_EVAL_PROBE_CHILD="1")
        env.pop("KB_EVAL_SPB", None)
        if v != "auto":
            env["KB_EVAL_SPB"] = v
        rc = subprocess.call([sys.executable, os.path.abspath(__file__)], env=env, timeout=120)
        if rc:
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
