"""Probe: the C2 cycle time across processes (the unsharded engine ran 18.5-29.0 ms per cycle in
consecutive processes of one binary). Each child process reports where its host thread runs relative to the GPU
(the CPU it is on, that CPU's NUMA node, the GPU's NUMA node from sysfs), the engine's shader clock over its
launches (kb_stats fed_clock_ticks / fed_real_ticks: s_memtime against the 100 MHz s_memrealtime) and the cycle
times, so a slow mode can be told apart as clock, host placement or neither.
Usage: python3 scripts/spread_probe.py [--runs N] [--steps K] [--pin none,local,remote,...]
The parent starts the children before it touches the GPU (no exec from a GPU process)."""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpulist(text):
    out = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def cpu_node(cpu):
    base = f"/sys/devices/system/cpu/cpu{cpu}"
    try:
        for e in os.listdir(base):
            if e.startswith("node") and e[4:].isdigit():
                return int(e[4:])
    except OSError:
        pass
    return -1


def current_cpu():
    with open("/proc/self/stat") as f:
        return int(f.read().rsplit(")", 1)[1].split()[36])


def gpu_pci():
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, 0) != 0:
        return None
    return buf.value.decode().lower()


def child(pin, steps):
    bus = gpu_pci()  # (initialises HIP: this process is the measuring one from here on)
    dev = f"/sys/bus/pci/devices/{bus}" if bus else None
    gnode, local = -1, set()
    try:
        gnode = int(open(f"{dev}/numa_node").read())
        local = cpulist(open(f"{dev}/local_cpulist").read())
    except (OSError, TypeError, ValueError):
        pass
    allowed = os.sched_getaffinity(0)
    if pin == "local" and local & allowed:
        os.sched_setaffinity(0, local & allowed)
    elif pin == "remote" and allowed - local:
        os.sched_setaffinity(0, allowed - local)
    from scheduler_amd import runtime, synth
    snap = synth.c2_snapshot(seed=synth.SEED)
    ctx = runtime.Context(0)
    ctx.upload(snap)
    ctx.allocate(snap)
    ctx.stats(reset=True)
    ts = []
    for _ in range(steps):
        ctx.restore()
        t0 = time.perf_counter()
        ctx.allocate(snap)
        ts.append((time.perf_counter() - t0) * 1e3)
    st = ctx.stats()
    ctx.close()
    cpu = current_cpu()
    clk = 100.0 * st["fed_clock_ticks"] / st["fed_real_ticks"] if st["fed_real_ticks"] else None
    ts.sort()
    print(json.dumps({"pin": pin, "gpu_bus": bus, "gpu_numa": gnode, "cpu": cpu, "cpu_numa": cpu_node(cpu),
                      "cpu_local_to_gpu": cpu in local, "allowed_cpus": len(os.sched_getaffinity(0)),
                      "engine_clock_mhz": round(clk, 1) if clk else None,
                      "engine_ms_per_cycle": round(st["fed_real_ticks"] / 1e5 / max(1, st["fed_cycles"]), 3),
                      "cycle_ms_min": round(ts[0], 3), "cycle_ms_p50": round(ts[len(ts) // 2], 3)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--pin", default="none")
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child is not None:
        child(a.child, a.steps)
        return 0
    for pin in a.pin.split(","):
        for _ in range(a.runs):
            rc = subprocess.call([sys.executable, os.path.abspath(__file__), "--child", pin, "--steps", str(a.steps)],
                                 timeout=180)
            if rc:
                return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
