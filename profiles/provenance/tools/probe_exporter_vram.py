#!/usr/bin/env python3
"""How much VRAM does the exporter itself take on a GPU?  Reads the GPU's used VRAM
(mem_info_vram_used, device-wide, once it has settled) before the engine starts and while it
runs with each GPU source on (amdsmi raw path only / + KFD events / + PMC counters / +
sentinel), each in a fresh process, plus the KFD proc entries that appeared or grew (the
exporter's own, by host PID).  Run on an otherwise idle GPU.  profiles/r04/exporter_vram.txt.
Usage: python tools/probe_exporter_vram.py
"""
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def our_gpu() -> tuple:
    """(KFD gpu_id, PCI BDF) of the GPU this process sees first (the box shows the host's
    whole KFD topology; other GPUs belong to other tenants)."""
    from kubernetes_gpu_exporter_amd.utils.kfdself import hip_order_bdfs
    bdf = hip_order_bdfs()[0].lower()
    dom, bus, rest = bdf.split(":")
    dev, fn = rest.split(".")
    want = (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn)
    for node in glob.glob("/sys/class/kfd/kfd/topology/nodes/*"):
        try:
            gid = int(open(node + "/gpu_id").read().strip() or 0)
            kv = dict(line.split() for line in open(node + "/properties") if len(line.split()) == 2)
            if gid and int(kv.get("location_id", -1)) == want and int(kv.get("domain", 0)) == int(dom, 16):
                return gid, bdf
        except (OSError, ValueError):
            continue
    return 0, bdf


GPU_ID, BDF = our_gpu()


def vram_used() -> int:
    """Used VRAM of OUR GPU (device-wide: every process on it)."""
    try:
        return int(open(f"/sys/bus/pci/devices/{BDF}/mem_info_vram_used").read())
    except (OSError, ValueError):
        return -1


def kfd_vram() -> dict:
    """pid -> vram_<our gpu_id> of every process in the KFD proc directory (host PIDs)."""
    out = {}
    for f in glob.glob(f"/sys/class/kfd/kfd/proc/*/vram_{GPU_ID}"):
        try:
            out[f.split("/")[-2]] = int(open(f).read())
        except (OSError, ValueError):
            pass
    return out


def settle(timeout: float = 15.0) -> int:
    """Device-wide used VRAM once it stops moving (a previous process's memory is released
    asynchronously after it exits)."""
    last, t_end = vram_used(), time.time() + timeout
    while time.time() < t_end:
        time.sleep(0.5)
        v = vram_used()
        if abs(v - last) < (1 << 20):
            return v
        last = v
    return last


def run(n, counters: bool, sentinel: bool, kfd_events: bool) -> dict:
    from kubernetes_gpu_exporter_amd._native import rocprof_plugin_path
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0.1
    c.serve_http = False
    c.series_profile = "full"
    c.enable_counters = counters
    c.enable_sentinel = sentinel
    c.enable_kfd_events = kfd_events
    c.counters_plugin = rocprof_plugin_path("aqlpmc")
    c.device_filter = [0]
    before = settle()
    k0 = kfd_vram()
    e = n.Engine(c)
    e.start()
    time.sleep(2.0)
    during = vram_used()
    k1 = kfd_vram()
    status = e.source_status()
    rss = [int(l.split()[1]) for l in open("/proc/self/status") if l.startswith("VmRSS:")][0]
    e.stop()
    new = {p: v for p, v in k1.items() if p not in k0}
    grown = {p: v - k0[p] for p, v in k1.items() if p in k0 and v != k0[p]}
    return {"counters": counters, "sentinel": sentinel, "kfd_events": kfd_events,
            "device_used_before_mib": round(before / 2**20, 1),
            "device_delta_mib": round((during - before) / 2**20, 1),
            "new_kfd_processes_mib": {p: round(v / 2**20, 1) for p, v in new.items()},
            "grown_kfd_processes_mib": {p: round(v / 2**20, 1) for p, v in grown.items()},
            "rss_mib": round(rss / 1024, 1),
            "env": {k: v for k, v in os.environ.items() if k.startswith("HSA_") and k != "HSA_ENABLE_IPC_MODE_LEGACY"},
            "gpu_id": GPU_ID, "bdf": BDF, "status": status[:120]}


def main() -> int:
    if len(sys.argv) == 5 and sys.argv[1] == "--one":  # child: one configuration, fresh process
        from kubernetes_gpu_exporter_amd._native import load
        print(json.dumps(run(load(), sys.argv[2] == "1", sys.argv[3] == "1", sys.argv[4] == "1")), flush=True)
        return 0
    import subprocess
    rows = []
    configs = (("0", "0", "0"), ("0", "0", "1"), ("1", "0", "1"), ("1", "1", "1"))
    if "--queue-only" in sys.argv:  # the HSA-queue configuration only (runtime setting A/B)
        configs = (("1", "1", "1"),)
    for counters, sentinel, kfd_events in configs:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", counters, sentinel, kfd_events],
                           capture_output=True, text=True, timeout=120)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        row = json.loads(line[-1]) if line else {"error": r.stderr[-500:]}
        rows.append(row)
        print(json.dumps(row), flush=True)
    print("RESULT " + json.dumps(rows), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
