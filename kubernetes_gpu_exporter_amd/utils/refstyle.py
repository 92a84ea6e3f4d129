"""Reference-ARCHITECTURE exporter, for same-hardware comparison in bench.py only.

The reference (/root/reference/main.go) cannot run here (Go + NVML + in-cluster).  Its
design is: a custom registry of GaugeVecs (main.go:21-42), a promhttp handler that
gathers and renders on every scrape (main.go:68-70), and a polling loop that calls the
vendor management library per device and sets gauges (main.go:116-150).  This module
rebuilds exactly that architecture on MI355X — prometheus_client registry + its threaded
HTTP server (render-on-scrape), amdsmi Python binding as the NVML analog — exposing the
same two legacy families plus 62 device series per GPU so the payload matches the
native exporter's standard profile (64 series/GPU).  It is a measuring stick, not a
product path; run:  python -m kubernetes_gpu_exporter_amd.utils.refstyle --port P --devices 0,1
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import threading
import time

DEVICE_FIELDS = 62  # + 2 legacy families = 64 series per GPU


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--interval", type=float, default=0.1)
    ap.add_argument("--devices", default="0")
    ap.add_argument("--mock", action="store_true", help="no amdsmi: synthetic values (CPU-only runs)")
    a = ap.parse_args()
    from prometheus_client import CollectorRegistry, Gauge, start_http_server
    reg = CollectorRegistry()
    mem = Gauge("pod_gpu_memory_usage", "GPU memory used by Kubernetes Pod", ["pid", "pod"], registry=reg)
    perc = Gauge("docker_gpu_memory_perc_usage", "GPU memory in percentage used by pod", ["pid", "pod"], registry=reg)
    dev = Gauge("amd_gpu_metric", "device metric", ["gpu", "field"], registry=reg)
    start_http_server(a.port, addr="127.0.0.1", registry=reg)
    idx = [int(x) for x in a.devices.split(",") if x != ""]
    handles = []
    smi = None
    if not a.mock:
        import amdsmi as smi
        smi.amdsmi_init()
        hs = smi.amdsmi_get_processor_handles()
        handles = [hs[i] for i in idx]
    pod_map_path = os.environ.get("GPUEXP_POD_MAP_FILE", "")
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *x: stop.set())
    while not stop.is_set():
        t0 = time.monotonic()
        pods = {}
        if pod_map_path and os.path.exists(pod_map_path):
            with open(pod_map_path) as fh:
                m = json.load(fh)
            uid2name = {p["uid"]: p["name"] for p in m.get("pods", [])}
            for pid, cg in m.get("pid_cgroups", {}).items():
                for uid, name in uid2name.items():
                    if uid in cg or uid.replace("-", "_") in cg:
                        pods[int(pid)] = name
        for gi, g in enumerate(idx):
            if smi is not None:
                mtr = smi.amdsmi_get_gpu_metrics_info(handles[gi])
                vram = smi.amdsmi_get_gpu_vram_usage(handles[gi])
                total = vram["vram_total"] * (1 << 20)
                vals = [v for v in mtr.values() if isinstance(v, (int, float))]
                procs = smi.amdsmi_get_gpu_process_list(handles[gi])
            else:
                total, vals, procs = 309220868096, list(range(DEVICE_FIELDS)), []
            for k in range(DEVICE_FIELDS):
                dev.labels(str(g), f"f{k}").set(float(vals[k % len(vals)]) if vals else 0.0)
            for p in procs:
                pid = int(p.get("pid", 0)) if isinstance(p, dict) else 0
                used = float(p.get("mem", 0)) if isinstance(p, dict) else 0.0
                if pid in pods:
                    mem.labels(str(pid), pods[pid]).set(used)
                    perc.labels(str(pid), pods[pid]).set(used / total * 100)
        stop.wait(max(0.0, a.interval - (time.monotonic() - t0)))
    if smi is not None:
        smi.amdsmi_shut_down()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
