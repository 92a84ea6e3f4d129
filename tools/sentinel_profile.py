#!/usr/bin/env python3
"""Runs the amdsmi engine with the HIP sentinel at `hz` for `seconds`, stops it and exits
normally (no os._exit) so a profiler wrapping this process can flush — e.g.
  rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sent -o sent -- \\
      python3 tools/sentinel_profile.py 100 3
Torch-free: the only HIP runtime in the process is the sentinel's.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    hz = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    from kubernetes_gpu_exporter_amd._native import load
    from kubernetes_gpu_exporter_amd.utils import promtext
    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 1.0 / hz
    c.serve_http = False
    c.enable_sentinel = True
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    time.sleep(secs)
    fams = promtext.parse(e.snapshot_text())
    out = {"status": e.source_status(), "ticks": e.stats()["ticks"]}
    for name in ("amd_gpu_sentinel_runs_total", "amd_gpu_sentinel_sclk_hz", "amd_gpu_sentinel_dispatch_latency_seconds"):
        v = promtext.samples(fams, name)
        out[name] = v[0][2] if v else None
    e.stop()
    print("RESULT " + json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
