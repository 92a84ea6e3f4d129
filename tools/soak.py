#!/usr/bin/env python3
"""Soak run of the exporter's default GPU path on one MI355X: the engine (amdsmi raw path,
aqlprofile counters with inline read rounds, sentinel, HTTP with gzip, full profile) at
10 Hz under a bf16 GEMM pod, scraped at 10 Hz, for `--minutes`.  Every `--every` seconds it
prints one line: RSS, open file descriptors, threads, ticks, overruns, late counter reads,
scrape p50/p99 over the interval and scrape errors -- so leaks (memory, fds, threads) and
drift show as growth across the lines.  profiles/r04/soak.txt.

Usage: python tools/soak.py [--minutes 8] [--every 30]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GEMM = ("import sys, time; sys.path.insert(0, {root!r});"
        "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
        "t = time.time()\n"
        "while time.time() - t < {secs}: gemm_burn(0, 8192, 20.0, 4)")


def proc_status(pid: int) -> dict:
    out = {}
    for line in open(f"/proc/{pid}/status"):
        k, _, v = line.partition(":")
        if k in ("VmRSS", "Threads"):
            out[k] = int(v.split()[0])
    out["fds"] = len(os.listdir(f"/proc/{pid}/fd"))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=8.0)
    ap.add_argument("--every", type=float, default=30.0)
    args = ap.parse_args()
    secs = args.minutes * 60
    gemm = subprocess.Popen([sys.executable, "-c", GEMM.format(root=ROOT, secs=secs + 30)])
    from kubernetes_gpu_exporter_amd._native import load, rocprof_plugin_path
    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0.1
    c.series_profile = "full"
    c.enable_counters = True
    c.enable_sentinel = True
    c.counters_plugin = rocprof_plugin_path("aqlpmc")
    c.http.host = "127.0.0.1"
    c.http.port = 0
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    print("status:", e.source_status(), flush=True)
    cl = n.ScrapeClient("127.0.0.1", e.http_port, "/metrics", True)
    lat: list = []
    errors = [0]
    stop = threading.Event()

    def scrape():
        nxt = time.monotonic()
        while not stop.is_set():
            nxt += 0.1
            time.sleep(max(0.0, nxt - time.monotonic()))
            t0 = time.perf_counter()
            try:
                if cl.scrape() <= 0:
                    errors[0] += 1
            except Exception:
                errors[0] += 1
            lat.append(time.perf_counter() - t0)

    th = threading.Thread(target=scrape, daemon=True)
    th.start()
    rows = []
    t_end = time.monotonic() + secs
    time.sleep(5.0)  # past start-up
    me = os.getpid()
    while True:
        lat.clear()
        time.sleep(args.every)
        st = e.stats()
        ps = proc_status(me)
        from kubernetes_gpu_exporter_amd.utils import promtext
        fams = promtext.parse(e.snapshot_text())
        late = promtext.samples(fams, "gpuexp_counters_late_ticks_total")
        stalls = [v for _, lab, v in promtext.samples(fams, "gpuexp_counters_events_total")
                  if lab.get("event") == "read_stall"]
        mfma = promtext.samples(fams, "amd_gpu_mfma_busy_percent")
        window = sorted(lat)
        row = {"t_s": round(secs - (t_end - time.monotonic()), 1), "rss_mb": round(ps["VmRSS"] / 1024, 1),
               "fds": ps["fds"], "threads": ps["Threads"], "ticks": st["ticks"], "overruns": st["overruns"],
               "counters_late": late[0][2] if late else None, "read_stalls": stalls[0] if stalls else None,
               "mfma_busy": round(mfma[0][2], 1) if mfma else None, "scrapes": len(window),
               "p50_us": round(statistics.median(window) * 1e6, 1) if window else None,
               "p99_us": round(window[int(0.99 * (len(window) - 1))] * 1e6, 1) if window else None,
               "scrape_errors": errors[0], "gemm_alive": gemm.poll() is None}
        rows.append(row)
        print(json.dumps(row), flush=True)
        if time.monotonic() >= t_end:
            break
    stop.set()
    th.join(timeout=5)
    e.stop()
    gemm.terminate()
    gemm.wait(timeout=60)
    first, last = rows[0], rows[-1]
    summary = {"minutes": args.minutes, "rss_growth_mb": round(last["rss_mb"] - first["rss_mb"], 1),
               "fd_growth": last["fds"] - first["fds"], "thread_growth": last["threads"] - first["threads"],
               "overruns": last["overruns"], "scrape_errors": last["scrape_errors"],
               "p50_us_first_last": [first["p50_us"], last["p50_us"]]}
    print("RESULT " + json.dumps(summary), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
