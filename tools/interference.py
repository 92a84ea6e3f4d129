#!/usr/bin/env python3
"""Exporter interference on a saturated MFMA workload (BASELINE config 5's question: what
does monitoring cost the pods?).  Runs a torch-free bf16 GEMM burn (8192^3, our gfx950
kernel) for `seconds` per trial, alternating trials with no exporter and with the
exporter sampling at 10 Hz and 100 Hz (amdsmi raw path + HIP sentinel + aqlprofile PMC
counters, full profile) — interleaved so clock/thermal drift cancels out.  This parent
never touches the GPU; every GPU user is a child process.
Usage: python tools/interference.py [seconds_per_trial] [rounds] [gemm|copy] [modes]  -> prints RESULT json
  modes: comma list of none | 10hz | 100hz | <counters mode><hz> (cont10, duty10, cont100, ...),
         default none,10hz,100hz (the default counters mode)
  gemm  MFMA-bound pod (TFLOP/s);  copy  HBM-bound pod: the calibration stream copy of
        1 GiB per launch (probe_device.h), read+write TB/s
"""
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


COPY_BURN = """
import json, sys, time
sys.path.insert(0, {root!r})
import torch
from kubernetes_gpu_exporter_amd.ops.gemm import stream_copy
src = torch.empty(1 << 30, dtype=torch.uint8, device="cuda").fill_(1)
dst = torch.empty_like(src)
for _ in range(10):
    stream_copy(src, dst)
torch.cuda.synchronize()
n, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < {seconds}:
    for _ in range(50):
        stream_copy(src, dst)
    torch.cuda.synchronize()
    n += 50
dt = time.perf_counter() - t0
print(json.dumps({{"tflops": 2.0 * (1 << 30) * n / dt / 1e12}}), flush=True)  # TB/s, read+write
"""


def burn(seconds: float, workload: str = "gemm") -> float:
    if workload == "copy":
        code = COPY_BURN.format(root=ROOT, seconds=seconds)
    else:
        code = (f"import sys, json; sys.path.insert(0, {ROOT!r});"
                "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                f"print(json.dumps(gemm_burn(0, 8192, {seconds}, 4)), flush=True)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=seconds + 120)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not line:
        raise RuntimeError(f"gemm_burn failed: {r.stderr[-800:]}")
    return float(json.loads(line[-1])["tflops"])


def start_exporter(hz: float, counters_mode: str = ""):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "kubernetes_gpu_exporter_amd", "--listen", f"127.0.0.1:{port}", "--interval",
           str(1.0 / hz), "--backend", "amdsmi", "--devices", "0", "--enable-sentinel", "true", "--enable-counters",
           "true", "--series-profile", "full", "--log-level", "warn"]
    if counters_mode:
        cmd += ["--counters-mode", counters_mode, "--counters-interval-ms", str(int(1000 / hz))]
    p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    import http.client
    for _ in range(600):
        try:
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=0.5)
            c.request("GET", "/readyz")
            if c.getresponse().status == 200:
                return p
        except OSError:
            pass
        time.sleep(0.05)
    p.kill()
    raise RuntimeError("exporter not ready")


def main() -> int:
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    workload = sys.argv[3] if len(sys.argv) > 3 else "gemm"
    modes = (sys.argv[4] if len(sys.argv) > 4 else "none,10hz,100hz").split(",")
    res = {m: [] for m in modes}
    burn(2.0, workload)  # warm clocks / code objects

    def exporter_for(mode):
        if mode == "none":
            return None
        import re
        m = re.fullmatch(r"(cont|duty)?(\d+)(?:hz)?", mode)
        cmode = {"cont": "continuous", "duty": "duty", None: ""}[m.group(1)]
        return start_exporter(float(m.group(2)), cmode)

    for r in range(rounds):
        for mode in modes:
            p = exporter_for(mode)
            try:
                time.sleep(1.0 if p else 0.0)
                res[mode].append(burn(secs, workload))
            finally:
                if p is not None:
                    p.terminate()
                    p.wait(timeout=20)
            print(mode, round(res[mode][-1], 1), flush=True)
    med = {k: statistics.median(v) for k, v in res.items()}
    out = {"tflops": res, "median_tflops": {k: round(v, 1) for k, v in med.items()},
           "slowdown_pct": {k: round(100.0 * (med["none"] - med[k]) / med["none"], 3) for k in modes if k != "none"},
           "seconds_per_trial": secs, "rounds": rounds, "workload": workload,
           "unit": "TB/s read+write" if workload == "copy" else "TFLOP/s"}
    print("RESULT " + json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
