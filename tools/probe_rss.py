#!/usr/bin/env python3
"""GPU-box probe: exporter resident memory by optional source.  Starts the exporter with
each combination of sentinel / PMC counters, waits for a few ticks, and reports VmRSS plus
the largest mappings from /proc/<pid>/smaps (by Rss).  Usage: python tools/probe_rss.py"""
import json
import os
import socket
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def smaps_individual(pid: int, k: int = 8) -> list:
    rows, cur = [], None
    for line in open(f"/proc/{pid}/smaps"):
        parts = line.split()
        if len(parts) >= 5 and "-" in parts[0] and ":" not in parts[0]:
            a, b = (int(x, 16) for x in parts[0].split("-"))
            cur = {"map": " ".join(parts[5:]) or "[anon]", "perm": parts[1], "size_kb": (b - a) >> 10, "rss_kb": 0}
            rows.append(cur)
        elif parts and parts[0] == "Rss:" and cur is not None:
            cur["rss_kb"] = int(parts[1])
    return sorted(rows, key=lambda x: -x["rss_kb"])[:k]


def smaps_top(pid: int, k: int = 8) -> list:
    rows, cur = [], None
    for line in open(f"/proc/{pid}/smaps"):
        parts = line.split()
        if len(parts) >= 5 and "-" in parts[0] and ":" not in parts[0]:
            cur = {"map": " ".join(parts[5:]) or "[anon]", "perm": parts[1], "rss_kb": 0}
            rows.append(cur)
        elif parts and parts[0] == "Rss:" and cur is not None:
            cur["rss_kb"] = int(parts[1])
    agg: dict = {}
    for r in rows:
        key = r["map"]
        agg[key] = agg.get(key, 0) + r["rss_kb"]
    return sorted(({"map": m, "rss_kb": v} for m, v in agg.items()), key=lambda x: -x["rss_kb"])[:k]


def run(sentinel: bool, counters: bool, env_extra: dict) -> dict:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, **env_extra)
    p = subprocess.Popen([sys.executable, "-m", "kubernetes_gpu_exporter_amd", "--listen", f"127.0.0.1:{port}",
                          "--interval", "0.1", "--backend", "amdsmi", "--devices", "0", "--series-profile", "full",
                          "--enable-sentinel", str(sentinel).lower(), "--enable-counters", str(counters).lower(),
                          "--log-level", "warn"], cwd=ROOT, env=env)
    try:
        for _ in range(300):
            try:
                if urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=1).status == 200:
                    break
            except Exception:
                time.sleep(0.1)
        time.sleep(2.0)
        rss = int([l for l in open(f"/proc/{p.pid}/status") if l.startswith("VmRSS:")][0].split()[1])
        threads = len(os.listdir(f"/proc/{p.pid}/task"))
        return {"sentinel": sentinel, "counters": counters, "env": env_extra, "rss_kb": rss, "threads": threads,
                "top": smaps_top(p.pid), "top_maps": smaps_individual(p.pid)}
    finally:
        p.terminate()
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()


def main() -> int:
    cases = [(False, False, {}), (True, False, {}), (False, True, {}), (True, True, {})]
    if len(sys.argv) > 1 and sys.argv[1] == "knobs":
        cases = [(True, False, {"MALLOC_ARENA_MAX": "2"}), (True, False, {"GPU_MAX_HW_QUEUES": "1"}),
                 (True, False, {"HIP_FORCE_DEV_KERNARG": "1"}), (False, True, {"MALLOC_ARENA_MAX": "2"})]
    for sen, cnt, env in cases:
        print("RESULT " + json.dumps(run(sen, cnt, env)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
