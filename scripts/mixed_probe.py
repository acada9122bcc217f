"""Mixed-cycle cost probe (GPU box): the C2M shape with its two-template and affinity job fractions switched on
and off, cycle time per configuration and the driver's counters (units off the engine, engine pauses)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scheduler_amd import columns, runtime, synth  # noqa: E402


def main():
    opts = runtime.parse_options(sys.argv[1] if len(sys.argv) > 1 else "")
    for fm, fa in ((0.0, 0.0), (0.02, 0.0), (0.0, 0.02), (0.02, 0.02)):
        snap = columns.build(synth.c2m_columns(n_nodes=10000, n_jobs=1000, tasks_per_job=100, frac_multi=fm,
                                               frac_aff=fa))
        ctx = runtime.Context(0, options=opts)
        ctx.upload(snap)
        out = None
        for _ in range(2):
            ctx.restore()
            out = ctx.allocate(snap, out=out)
        ctx.stats(reset=True)
        t = []
        for _ in range(5):
            ctx.restore()
            t0 = time.perf_counter()
            out = ctx.allocate(snap, out=out)
            t.append((time.perf_counter() - t0) * 1e3)
        st = ctx.stats()
        ctx.close()
        print(f"multi={fm} aff={fa}: {min(t):.3f} ms/cycle (median {sorted(t)[2]:.3f}), placed {int(out['n_events'])}, "
              f"job_calls/cycle {st['job_calls'] / 5:.0f}, off_engine {st['off_engine_units'] / 5:.0f}, "
              f"pauses {st['fed_pauses'] / 5:.0f}, engine launches {st['fed_cycles'] / 5:.1f}", flush=True)


if __name__ == "__main__":
    main()
