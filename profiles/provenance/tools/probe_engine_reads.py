#!/usr/bin/env python3
"""GPU-box probe: run the amdsmi engine at a given rate for a few seconds and report the
device-read path (raw gpu_metrics vs amdsmi), fresh/coalesced read counts, learnt PMFW
period and the sampler's stage timings.  Usage: python tools/probe_engine_reads.py [hz] [s]
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
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    time.sleep(secs)
    fams = promtext.parse(e.snapshot_text())
    out = {"status": e.source_status(), "stats": e.stats(),
           "reads": {s[1]["kind"]: s[2] for s in promtext.samples(fams, "gpuexp_gpu_metrics_reads_total")},
           "period_s": [s[2] for s in promtext.samples(fams, "gpuexp_gpu_metrics_refresh_period_seconds")]}
    e.stop()
    print("RESULT " + json.dumps(out, default=str))
    # raw sequence, as the engine would see it at this rate
    import glob
    fd = os.open(sorted(glob.glob("/sys/class/drm/renderD*/device/gpu_metrics"))[0], os.O_RDONLY)
    t0 = time.monotonic_ns()
    seq = []
    for k in range(30):
        d = n.decode_gpu_metrics(os.pread(fd, 8192, 0))
        seq.append(((time.monotonic_ns() - t0) / 1e6, d["fw_ts_10ns"]))
        time.sleep(1.0 / hz)
    base = seq[0][1]
    print("SEQ " + json.dumps([(round(t, 2), (f - base) / 1e5) for t, f in seq]))  # ms, ms
    sys.stdout.flush()
    os._exit(0)


if __name__ == "__main__":
    sys.exit(main())
