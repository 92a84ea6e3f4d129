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


def vram_used() -> int:
    for f in sorted(glob.glob("/sys/class/drm/card*/device/mem_info_vram_used")):
        try:
            return int(open(f).read())
        except (OSError, ValueError):
            continue
    return -1


def kfd_vram() -> dict:
    """pid -> summed vram_<id> of every process in the KFD proc directory (host PIDs)."""
    out = {}
    for d in glob.glob("/sys/class/kfd/kfd/proc/*"):
        tot = 0
        for f in glob.glob(d + "/vram_*"):
            try:
                tot += int(open(f).read())
            except (OSError, ValueError):
                pass
        out[os.path.basename(d)] = tot
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
    e.stop()
    new = {p: v for p, v in k1.items() if p not in k0}
    grown = {p: v - k0[p] for p, v in k1.items() if p in k0 and v != k0[p]}
    return {"counters": counters, "sentinel": sentinel, "kfd_events": kfd_events,
            "device_used_before_mib": round(before / 2**20, 1),
            "device_delta_mib": round((during - before) / 2**20, 1),
            "new_kfd_processes_mib": {p: round(v / 2**20, 1) for p, v in new.items()},
            "grown_kfd_processes_mib": {p: round(v / 2**20, 1) for p, v in grown.items()},
            "status": status[:120]}


def main() -> int:
    if len(sys.argv) == 5 and sys.argv[1] == "--one":  # child: one configuration, fresh process
        from kubernetes_gpu_exporter_amd._native import load
        print(json.dumps(run(load(), sys.argv[2] == "1", sys.argv[3] == "1", sys.argv[4] == "1")), flush=True)
        return 0
    import subprocess
    rows = []
    for counters, sentinel, kfd_events in (("0", "0", "0"), ("0", "0", "1"), ("1", "0", "1"), ("1", "1", "1")):
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
