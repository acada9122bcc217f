"""Practical HBM write ceiling on this card for a kb_eval-sized output (256 specs x 50k nodes x 8 B = 102.4 MB):
torch's fill kernel (a pure store stream) and hipMemsetAsync-backed zero_, timed with HIP events over 200 launches
after 200 warm-up launches, as bench.py's eval_side times eval_plain_kernel. Prints one JSON line."""
import json

import torch


def timed(fn, n=200, warm=200):
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n  # us per launch


def main():
    nbytes = 256 * 50000 * 8
    buf = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda:0")
    src = torch.ones_like(buf)
    out = {"bytes": nbytes}
    for name, fn in (("fill", lambda: buf.fill_(7)), ("zero", lambda: buf.zero_()),
                     ("copy_rw", lambda: buf.copy_(src))):
        us = timed(fn)
        moved = nbytes * (2 if name == "copy_rw" else 1)
        out[name] = {"us": round(us, 2), "GBps": round(moved / us / 1e3, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
