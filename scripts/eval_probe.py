"""GPU probe: kb_eval32 (eval_plain_kernel) at bench.py's eval side measurement (256 specs x 50k nodes), for several
specs-per-block settings (kb_opts.eval_spb; 0 = the default resident-round sizing). Prints avg launch us each."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from scheduler_amd import runtime, synth  # noqa: E402

NODES, SPECS = 50000, 256
snap = synth.c2_snapshot(n_nodes=NODES, n_jobs=SPECS, tasks_per_job=1, seed=synth.SEED)
ids = (np.arange(SPECS) % len(snap.spec_arr)).astype(np.int32)
k = runtime.KERNELS.index("eval_kernel")
alg = SPECS * NODES * 8 + NODES * 76
for spb in [int(a) for a in sys.argv[1:]] or [0, 16, 32, 43, 64]:
    ctx = runtime.Context(0, timing=True, options={"eval_spb": spb})
    try:
        ctx.upload(snap)
        for _ in range(200):
            ctx.eval32(ids)
        ctx.stats(reset=True)
        for _ in range(20):
            ctx.eval32(ids)
        st = ctx.stats()
    finally:
        ctx.close()
    us = st["kernel_ms"][k] * 1e3 / max(1, st["launches"][k])
    print(f"eval_spb={spb} avg_us={us:.2f} alg_frac={alg / (us * 1e-6) / 8e12:.3f}", flush=True)
