#!/usr/bin/env python3
"""Soak test on a GPU box: the exporter (amdsmi backend, full profile, sentinel, PMC
counters) samples at `hz` while a GEMM child keeps the GPU busy and a keep-alive client
scrapes at the same rate with gzip, for `seconds`.  Every 10 s it records the exporter's
RSS, CPU%, series count, tick overruns and scrape errors, and reports the drift.
Usage: python tools/soak.py [seconds] [hz] [backend]  -> prints progress lines and a RESULT json"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rss_kb(pid: int) -> int:
    for line in open(f"/proc/{pid}/status"):
        if line.startswith("VmRSS:"):
            return int(line.split()[1])
    return 0


def main() -> int:
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    hz = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
    backend = sys.argv[3] if len(sys.argv) > 3 else "amdsmi"
    from kubernetes_gpu_exporter_amd._native import load
    from kubernetes_gpu_exporter_amd.utils import promtext
    from kubernetes_gpu_exporter_amd.utils.procstat import cpu_seconds_precise
    n = load()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    exp = subprocess.Popen([sys.executable, "-m", "kubernetes_gpu_exporter_amd", "--listen", f"127.0.0.1:{port}",
                            "--interval", str(1.0 / hz), "--backend", backend, "--devices", "0",
                            "--series-profile", "full", "--enable-sentinel", "true", "--enable-counters", "true",
                            "--log-level", "warn"], cwd=ROOT)
    gemm = None if backend == "mock" else subprocess.Popen([sys.executable, "-c",
                             f"import sys; sys.path.insert(0, {ROOT!r});"
                             "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                             f"print(gemm_burn(0, 8192, {seconds + 20}, 4), flush=True)"], cwd=ROOT)
    try:
        cl = None
        for _ in range(600):
            try:
                cl = n.ScrapeClient("127.0.0.1", port, "/metrics", True, 2000)
                if cl.scrape() > 0 and cl.last_status == 200:
                    break
            except Exception:
                pass
            time.sleep(0.1)
        time.sleep(3.0)  # first ticks, counters warm-up
        samples = []
        lat = []
        t0 = time.monotonic()
        next_report = t0
        cpu0 = cpu_seconds_precise(exp.pid)
        period = 1.0 / hz
        t_next = t0
        while time.monotonic() - t0 < seconds:
            ns = cl.scrape()
            if ns > 0:
                lat.append(ns / 1e3)
            now = time.monotonic()
            if now >= next_report:
                import gzip
                fams = promtext.parse(gzip.decompress(cl.last_body()).decode())
                row = {"t": round(now - t0, 1), "rss_kb": rss_kb(exp.pid),
                       "cpu_pct": round(100 * (cpu_seconds_precise(exp.pid) - cpu0) / max(1e-9, now - t0), 3),
                       "series": promtext.value(fams, "gpuexp_series"),
                       "overruns": promtext.value(fams, "gpuexp_tick_overruns_total"),
                       "ticks": promtext.value(fams, "gpuexp_ticks_total"),
                       "scrape_errors": cl.errors}
                samples.append(row)
                print("PROGRESS " + json.dumps(row), flush=True)
                next_report += 10.0
            t_next += period
            time.sleep(max(0.0, t_next - time.monotonic()))
        lat.sort()
        first, last = samples[0], samples[-1]
        res = {"seconds": seconds, "hz": hz, "scrapes": len(lat), "p50_us": lat[len(lat) // 2] if lat else None,
               "p99_us": lat[int(len(lat) * 0.99)] if lat else None,
               "rss_kb_first": first["rss_kb"], "rss_kb_last": last["rss_kb"],
               "rss_growth_kb": last["rss_kb"] - first["rss_kb"], "cpu_pct": last["cpu_pct"],
               "series_first": first["series"], "series_last": last["series"],
               "overruns": last["overruns"] - first["overruns"], "ticks": last["ticks"] - first["ticks"],
               "scrape_errors": last["scrape_errors"]}
        print("RESULT " + json.dumps(res), flush=True)
    finally:
        exp.terminate()
        try:
            exp.wait(timeout=10)
        except subprocess.TimeoutExpired:
            exp.kill()
        if gemm is not None:
            gemm.terminate()
            try:
                gemm.wait(timeout=30)
            except subprocess.TimeoutExpired:
                gemm.kill()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
