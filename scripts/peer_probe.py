"""GPU probe: the peer-engine cases of tests/test_gpu_shard_peer.py on the split fed engine, the one-workgroup fed
engine and the one-rank sharded engine, three cycles each; prints where they differ (first tasks, per cycle)."""
import sys

sys.path.insert(0, "tests")
import numpy as np  # noqa: E402

from scheduler_amd import runtime  # noqa: E402
from test_gpu_shard import _summary  # noqa: E402
from test_gpu_shard_peer import _cases, _sharded  # noqa: E402


def plain(snap, cycles, options=None):
    ctx = runtime.Context(0, options=options)
    try:
        ctx.upload(snap)
        out = []
        for _ in range(cycles):
            ctx.restore()
            out.append(_summary(ctx.allocate(snap)))
        return out, ctx.stats()
    finally:
        ctx.close()


def diff(a, b, tag):
    for c, (x, y) in enumerate(zip(a, b)):
        for k in x:
            if x[k] != y[k]:
                xa, ya = np.asarray(x[k]), np.asarray(y[k])
                if xa.shape != ya.shape:
                    print(f"  {tag} cycle {c} {k}: shapes {xa.shape} {ya.shape}")
                    continue
                idx = np.nonzero(xa != ya)[0]
                print(f"  {tag} cycle {c} {k}: {len(idx)} differ, first {idx[:8].tolist()} "
                      f"a={xa[idx[:8]].tolist()} b={ya[idx[:8]].tolist()}")


for name, snap in _cases(1).items():
    split, st_s = plain(snap, 3)
    onewg, st_o = plain(snap, 3, {"no_fed_split": True})
    shard, st_h = _sharded(snap, 0, 1, lambda b: b, 3)
    print(name, "split", st_s["fed_split"], "shard", st_h["fed_sharded"], flush=True)
    diff(split, onewg, "split-vs-onewg")
    diff(shard, onewg, "shard-vs-onewg")
