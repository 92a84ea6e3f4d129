#!/usr/bin/env python3
"""GPU-box probe: how often does the PMFW refresh the gpu_metrics table, and what does one
read cost?  Reads <render node>/device/gpu_metrics at several rates for a few seconds
each (single pread per read, like the exporter) and reports, per rate:
  - wall and thread-CPU time per read (p50/p90),
  - the fraction of reads whose firmware_timestamp / accumulation_counter / energy changed,
  - the median firmware_timestamp step between distinct tables.
Drives the sampler's read-coalescing decision (EngineConfig::metrics_min_interval_ms).
Usage: python tools/probe_pmfw_rate.py [seconds_per_rate]
"""
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
    from kubernetes_gpu_exporter_amd._native import load
    n = load()
    paths = sorted(glob.glob("/sys/class/drm/renderD*/device/gpu_metrics"))
    if not paths:
        print("no gpu_metrics file")
        return 1
    fd = os.open(paths[0], os.O_RDONLY)
    out = {"path": paths[0], "rates": {}}
    for hz in (1000, 200, 100, 50, 10):
        period = 1.0 / hz
        rows = []
        t_end = time.perf_counter() + secs
        nxt = time.perf_counter()
        while time.perf_counter() < t_end:
            c0 = time.thread_time_ns()
            w0 = time.perf_counter_ns()
            blob = os.pread(fd, 8192, 0)
            w1 = time.perf_counter_ns()
            c1 = time.thread_time_ns()
            d = n.decode_gpu_metrics(blob)
            if d:
                rows.append((w1 - w0, c1 - c0, d["fw_ts_10ns"], d["accumulation_counter"], d["energy_acc"]))
            nxt += period
            delay = nxt - time.perf_counter()
            if delay > 0:
                time.sleep(delay)
        walls = sorted(r[0] / 1e3 for r in rows)
        cpus = sorted(r[1] / 1e3 for r in rows)
        ch_ts = sum(1 for a, b in zip(rows, rows[1:]) if a[2] != b[2])
        ch_acc = sum(1 for a, b in zip(rows, rows[1:]) if a[3] != b[3])
        ch_en = sum(1 for a, b in zip(rows, rows[1:]) if a[4] != b[4])
        steps = [(b[2] - a[2]) * 10 / 1e3 for a, b in zip(rows, rows[1:]) if b[2] != a[2]]  # us
        out["rates"][hz] = {
            "reads": len(rows),
            "wall_us_p50": round(walls[len(walls) // 2], 1), "wall_us_p90": round(walls[int(len(walls) * 0.9)], 1),
            "cpu_us_p50": round(cpus[len(cpus) // 2], 1), "cpu_us_p90": round(cpus[int(len(cpus) * 0.9)], 1),
            "changed_fw_ts": round(ch_ts / max(1, len(rows) - 1), 3),
            "changed_accumulation": round(ch_acc / max(1, len(rows) - 1), 3),
            "changed_energy": round(ch_en / max(1, len(rows) - 1), 3),
            "fw_ts_step_us_median": round(statistics.median(steps), 1) if steps else None,
        }
        print(hz, json.dumps(out["rates"][hz]), flush=True)
    os.close(fd)
    print("RESULT " + json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
