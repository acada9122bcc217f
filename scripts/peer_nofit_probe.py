"""Probe: the node-sharded engine on one rank over several cycles of a NO_FIT-heavy C2 cycle, each against the
unsharded engine (the tests' c2-nofit case). Usage: python3 scripts/peer_nofit_probe.py [cycles]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from scheduler_amd import runtime, synth  # noqa: E402
from test_gpu_shard import _summary  # noqa: E402


def main():
    cycles = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    snap = synth.c2_snapshot(n_nodes=2400, n_jobs=60, tasks_per_job=100, seed=22, fill=2.5)
    ctx = runtime.Context(0)
    ctx.upload(snap)
    ref = _summary(ctx.allocate(snap))
    ctx.close()
    ctx = runtime.Context(0)
    if os.environ.get("KB_PROBE_UNSHARDED") != "1":
        ctx.set_shard(0, 1, snap.n_nodes, allgather=lambda b: b, peer=True)
    ctx.upload(snap)
    bad = 0
    for c in range(cycles):
        ctx.restore()
        try:
            got = _summary(ctx.allocate(snap))
            ok = got == ref
            if not ok:
                for k in ref:
                    if got[k] != ref[k]:
                        a, b = got[k], ref[k]
                        i = next((i for i in range(min(len(a), len(b))) if a[i] != b[i]), min(len(a), len(b)))
                        print(f"cycle {c}: {k} differs at {i} (len {len(a)} vs {len(b)}): got {a[i:i + 3]} want "
                              f"{b[i:i + 3]}", flush=True)
        except runtime.KbError as e:
            ok = False
            print(f"cycle {c}: {e}", flush=True)
        bad += not ok
        print(f"cycle {c}: {'ok' if ok else 'DIFFERS'}", flush=True)
    print(f"self_inbox={os.environ.get('KB_SHARD_SELF_INBOX', '0')} unsharded="
          f"{os.environ.get('KB_PROBE_UNSHARDED', '0')} bad cycles {bad} of {cycles}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
