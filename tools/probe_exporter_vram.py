#!/usr/bin/env python3
"""How much VRAM does the exporter itself take on a GPU?  Reads the GPU's used VRAM
(mem_info_vram_used, device-wide) before the engine starts, while it runs with each GPU
source on (amdsmi raw path only / + PMC counters / + sentinel), and after it stops.  Run on an
otherwise idle GPU (the deltas are device-wide).  profiles/r04/exporter_vram.txt.
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


def run(n, counters: bool, sentinel: bool) -> dict:
    from kubernetes_gpu_exporter_amd._native import rocprof_plugin_path
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0.1
    c.serve_http = False
    c.series_profile = "full"
    c.enable_counters = counters
    c.enable_sentinel = sentinel
    c.counters_plugin = rocprof_plugin_path("aqlpmc")
    c.device_filter = [0]
    before = vram_used()
    e = n.Engine(c)
    e.start()
    time.sleep(2.0)
    during = vram_used()
    status = e.source_status()
    e.stop()
    time.sleep(1.0)
    after = vram_used()
    return {"counters": counters, "sentinel": sentinel, "before_mib": round(before / 2**20, 1),
            "during_delta_mib": round((during - before) / 2**20, 1), "after_delta_mib": round((after - before) / 2**20, 1),
            "status": status[:160]}


def main() -> int:
    if len(sys.argv) == 4 and sys.argv[1] == "--one":  # child: one configuration, fresh process
        from kubernetes_gpu_exporter_amd._native import load
        print(json.dumps(run(load(), sys.argv[2] == "1", sys.argv[3] == "1")), flush=True)
        return 0
    import subprocess
    rows = []
    for counters, sentinel in (("0", "0"), ("1", "0"), ("1", "1")):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", counters, sentinel],
                           capture_output=True, text=True, timeout=120)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        row = json.loads(line[-1]) if line else {"error": r.stderr[-500:]}
        rows.append(row)
        print(json.dumps(row), flush=True)
    print("RESULT " + json.dumps(rows), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
