#!/usr/bin/env python3
"""What does continuous PMC counting cost against duty-cycled counting (and none)?

For each mode the exporter runs as its own process (amdsmi raw path + sentinel on the PMC
queue, full profile, `--interval` 0.1 s) on an otherwise idle GPU, interleaved over
`rounds` so drift cancels:
  off         --enable-counters false
  duty        --counters-mode duty   (20 ms window every 100 ms: the round-2 default was
                                      20 ms every 1000 ms, also measured as duty1000)
  continuous  --counters-mode continuous (one read per tick, counting never paused)
and reports, per mode: the exporter's CPU (utime + stime of its process over `seconds`),
and the GPU's board power averaged over the same window from a second observer that
needs no PMC (amdsmi, read by a separate exporter-free Python process would take the
GPU too, so the exporter's own amd_gpu_power_watts (PMFW, not PMC-derived) is sampled
every 0.5 s).  This parent never touches the GPU.
Usage: python tools/pmc_cost.py [seconds] [rounds] -> RESULT json
"""
import http.client
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kubernetes_gpu_exporter_amd.utils import promtext  # noqa: E402

MODES = {
    "off": ["--enable-counters", "false"],
    "duty1000": ["--enable-counters", "true", "--counters-mode", "duty", "--counters-window-ms", "20",
                 "--counters-interval-ms", "1000"],
    "duty": ["--enable-counters", "true", "--counters-mode", "duty", "--counters-window-ms", "20",
             "--counters-interval-ms", "100"],
    "continuous": ["--enable-counters", "true", "--counters-mode", "continuous"],
}


def start(mode: str):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "kubernetes_gpu_exporter_amd", "--listen", f"127.0.0.1:{port}", "--interval", "0.1",
           "--backend", "amdsmi", "--devices", "0", "--enable-sentinel", "true", "--series-profile", "full",
           "--log-level", "warn"] + MODES[mode]
    p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    for _ in range(1200):
        try:
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=0.5)
            c.request("GET", "/readyz")
            if c.getresponse().status == 200:
                return p, port
        except OSError:
            pass
        time.sleep(0.05)
    p.kill()
    raise RuntimeError("exporter not ready")


def cpu_s(pid: int) -> float:
    f = open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()
    return (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK")


def scrape(port: int) -> dict:
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=2)
    c.request("GET", "/metrics")
    return promtext.parse(c.getresponse().read().decode())


def measure(mode: str, seconds: float) -> dict:
    p, port = start(mode)
    try:
        time.sleep(3.0)  # past start-up (HSA queue, amdsmi validation)
        c0, t0 = cpu_s(p.pid), time.monotonic()
        power = []
        while time.monotonic() - t0 < seconds:
            time.sleep(0.5)
            try:
                power.append(promtext.value(scrape(port), "amd_gpu_power_watts", gpu=0))
            except (OSError, KeyError):
                pass
        c1, t1 = cpu_s(p.pid), time.monotonic()
        fams = scrape(port)
        status = {lab.get("source"): v for _, lab, v in promtext.samples(fams, "gpuexp_source_up")}
    finally:
        p.terminate()
        p.wait(timeout=30)
    return {"cpu_pct": 100.0 * (c1 - c0) / (t1 - t0), "power_w": statistics.mean(power) if power else None,
            "power_samples": len(power), "sources": status}


def main() -> int:
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    res = {m: [] for m in MODES}
    for r in range(rounds):
        for m in MODES:
            res[m].append(measure(m, seconds))
            print(m, {k: (round(v, 3) if isinstance(v, float) else v) for k, v in res[m][-1].items()}, flush=True)
    summary = {m: {"cpu_pct_median": round(statistics.median(x["cpu_pct"] for x in v), 3),
                   "power_w_median": round(statistics.median(x["power_w"] for x in v if x["power_w"]), 1)}
               for m, v in res.items()}
    print("RESULT " + json.dumps({"seconds": seconds, "rounds": rounds, "summary": summary, "runs": res}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
