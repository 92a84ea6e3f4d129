#!/usr/bin/env python3
"""Soak run of the default exporter configuration on one MI355X: does anything grow?

The exporter (amdsmi raw path + queue sentinel + aqlprofile PMC, full profile) samples at
`--hz` while short-lived GEMM pods come and go (a new child process every `--pod-life`
seconds, so PIDs, KFD entries, per-process series and their GC churn the whole time) and a
keep-alive gzip scraper polls /metrics at 10 Hz.  Every 10 s it records the exporter's RSS,
open fds, threads, CPU and series count; the result is the first-to-last deltas and the
least-squares RSS slope over the second half (after warm-up), plus scrape errors.

Usage: python tools/soak.py [--seconds 300] [--hz 100] [--pod-life 6]  -> prints RESULT json
This parent never touches the GPU; every GPU user is a child process.
"""
import argparse
import gzip
import http.client
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def proc_stats(pid: int) -> dict:
    st = {}
    with open(f"/proc/{pid}/status") as fh:
        for line in fh:
            k, _, v = line.partition(":")
            if k in ("VmRSS", "Threads"):
                st[k] = int(v.split()[0])
    with open(f"/proc/{pid}/stat") as fh:
        f = fh.read().rsplit(")", 1)[1].split()
    tck = os.sysconf("SC_CLK_TCK")
    return {"rss_mb": st["VmRSS"] / 1024, "threads": st["Threads"], "fds": len(os.listdir(f"/proc/{pid}/fd")),
            "cpu_s": (int(f[11]) + int(f[12])) / tck}


def slope(xs, ys):
    n = len(xs)
    if n < 2:
        return 0.0
    mx, my = sum(xs) / n, sum(ys) / n
    den = sum((x - mx) ** 2 for x in xs)
    return sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / den if den else 0.0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300)
    ap.add_argument("--hz", type=float, default=100)
    ap.add_argument("--pod-life", type=float, default=6)
    args = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "kubernetes_gpu_exporter_amd", "--listen", f"127.0.0.1:{port}", "--interval",
           str(1.0 / args.hz), "--backend", "amdsmi", "--devices", "0", "--enable-sentinel", "true",
           "--enable-counters", "true", "--series-profile", "full", "--log-level", "warn"]
    exp = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    pods = []
    try:
        for _ in range(600):
            try:
                c = http.client.HTTPConnection("127.0.0.1", port, timeout=0.5)
                c.request("GET", "/readyz")
                if c.getresponse().status == 200:
                    break
            except OSError:
                pass
            time.sleep(0.05)
        conn = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
        burn = ("import sys; sys.path.insert(0, {root!r});"
                "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                "gemm_burn(0, 4096, {life}, 4)").format(root=ROOT, life=args.pod_life)
        samples, scrapes, errors, pids_seen = [], 0, 0, set()
        t0 = time.monotonic()
        next_sample = t0
        next_pod = t0
        next_scrape = t0
        series = 0
        while time.monotonic() - t0 < args.seconds:
            now = time.monotonic()
            if now >= next_pod:
                pods = [p for p in pods if p.poll() is None]
                p = subprocess.Popen([sys.executable, "-c", burn], cwd=ROOT, stdout=subprocess.DEVNULL,
                                     stderr=subprocess.DEVNULL)
                pods.append(p)
                pids_seen.add(p.pid)
                next_pod += args.pod_life / 2  # two pods overlap at any time
            if now >= next_scrape:
                try:
                    conn.request("GET", "/metrics", headers={"Accept-Encoding": "gzip"})
                    r = conn.getresponse()
                    body = r.read()
                    if r.status != 200:
                        errors += 1
                    elif now >= next_sample:
                        text = gzip.decompress(body) if r.getheader("Content-Encoding") == "gzip" else body
                        series = sum(1 for line in text.split(b"\n") if line and not line.startswith(b"#"))
                    scrapes += 1
                except (OSError, http.client.HTTPException):
                    errors += 1
                    conn = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
                next_scrape += 0.1
            if now >= next_sample:
                st = proc_stats(exp.pid)
                st.update({"t": round(now - t0, 1), "series": series})
                samples.append(st)
                print(json.dumps(st), flush=True)
                next_sample += 10
            time.sleep(0.005)
        half = [x for x in samples if x["t"] >= args.seconds / 2]
        first, last = samples[0], samples[-1]
        out = {"seconds": args.seconds, "hz": args.hz, "pods_started": len(pids_seen), "scrapes": scrapes,
               "scrape_errors": errors, "exporter_alive": exp.poll() is None,
               "rss_mb": [round(first["rss_mb"], 1), round(last["rss_mb"], 1)],
               "rss_slope_mb_per_hour_second_half": round(slope([x["t"] for x in half],
                                                                [x["rss_mb"] for x in half]) * 3600, 2),
               "fds": [first["fds"], last["fds"]], "threads": [first["threads"], last["threads"]],
               "cpu_percent": round(100 * (last["cpu_s"] - first["cpu_s"]) / max(1e-9, last["t"] - first["t"]), 3),
               "series": [first["series"], last["series"]]}
        print("RESULT " + json.dumps(out), flush=True)
        return 0
    finally:
        for p in pods:
            if p.poll() is None:
                p.terminate()
        for p in pods:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
        exp.terminate()
        try:
            exp.wait(timeout=20)
        except subprocess.TimeoutExpired:
            exp.kill()


if __name__ == "__main__":
    sys.exit(main())
