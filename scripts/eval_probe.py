"""kb_eval on its own (bench.py's eval side measurement: 256 specs x 50k C2-shaped nodes), for rocprofv3 counter
passes: python3 scripts/eval_probe.py [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scheduler_amd import runtime, synth  # noqa: E402

SPECS, NODES = 256, 50000


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    snap = synth.c2_snapshot(n_nodes=NODES, n_jobs=SPECS, tasks_per_job=1, seed=synth.SEED)
    ctx = runtime.Context(0, timing=True)
    ctx.upload(snap)
    ids = (np.arange(SPECS) % len(snap.spec_arr)).astype(np.int32)
    ctx.eval32(ids)
    ctx.stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.eval32(ids)
    el = time.perf_counter() - t0
    st = ctx.stats()
    k = runtime.KERNELS.index("eval_kernel")
    print(f"eval_kernel {st['kernel_ms'][k] * 1e3 / max(1, st['launches'][k]):.2f} us per launch, "
          f"{el / reps * 1e3:.2f} ms per kb_eval call, pairs {SPECS * NODES}")
    ctx.close()


if __name__ == "__main__":
    main()
