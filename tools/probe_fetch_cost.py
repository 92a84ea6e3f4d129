#!/usr/bin/env python3
"""CPU cost of a fresh gpu_metrics fetch on MI355X, the per-read figure the 8-GPU projection
uses (tests/test_fakehost.py SMU_FETCH_CPU_US; profiles/r04/fetch_cost.txt).

N threads (N = 1, 2, 4, 8) each pread() the real gpu_metrics file once per tick at 10 Hz, the
way an N-GPU exporter's reads would land, on this box's one GPU; every read's thread CPU
(user + system: the kernel busy-waits for the SMU's reply) and wall time is recorded.  This
is a per-read cost projection, not a scaling curve: on an 8-GPU node each GPU has its own
SMU, here N threads share one (a read that waits for another's SMU message sleeps on the
driver's lock, so its wall grows while its CPU should not).  Run idle, then again while a
child process keeps the GPU busy with the bf16 GEMM pod kernel.
Usage: python tools/probe_fetch_cost.py [--seconds 3] -> RESULT json
"""
import argparse
import glob
import json
import os
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def metrics_path() -> str:
    for p in sorted(glob.glob("/sys/class/drm/renderD*/device/gpu_metrics")):
        return p
    raise SystemExit("no gpu_metrics file")


def run(path: str, nthreads: int, seconds: float, hz: float) -> dict:
    cpu, wall = [], []
    lock = threading.Lock()
    stop = time.monotonic() + seconds

    def worker(k):
        fd = os.open(path, os.O_RDONLY)
        nxt = time.monotonic() + k * 0.001  # readers 1 ms apart, like a serial tick loop
        mine_c, mine_w = [], []
        while True:
            now = time.monotonic()
            if now >= stop:
                break
            if nxt > now:
                time.sleep(nxt - now)
            nxt += 1.0 / hz
            c0, w0 = time.thread_time_ns(), time.monotonic_ns()
            os.pread(fd, 8192, 0)
            mine_c.append((time.thread_time_ns() - c0) / 1e3)
            mine_w.append((time.monotonic_ns() - w0) / 1e3)
        os.close(fd)
        with lock:
            cpu.extend(mine_c)
            wall.extend(mine_w)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()

    def q(v, p):
        v = sorted(v)
        return round(v[min(len(v) - 1, int(p * len(v)))], 1) if v else None
    return {"threads": nthreads, "reads": len(cpu), "cpu_us_p50": q(cpu, 0.5), "cpu_us_p90": q(cpu, 0.9),
            "cpu_us_mean": round(statistics.mean(cpu), 1) if cpu else None,
            "wall_us_p50": q(wall, 0.5), "wall_us_p90": q(wall, 0.9)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--hz", type=float, default=10.0)
    args = ap.parse_args()
    path = metrics_path()
    res = {"path": path, "idle": [], "loaded": []}
    for n in (1, 2, 4, 8):
        r = run(path, n, args.seconds, args.hz)
        res["idle"].append(r)
        print("idle", r, flush=True)
    # the GEMM pod in a child process (torch-free: the kernels extension's own burn loop)
    burn = subprocess.Popen([sys.executable, "-c",
                             "import sys; sys.path.insert(0, %r)\n"
                             "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn\n"
                             "print(gemm_burn(0, 8192, %f), flush=True)" % (ROOT, 4 * args.seconds + 6)],
                            stdout=subprocess.PIPE, text=True)
    time.sleep(3.0)  # clocks and power settle under the load
    for n in (1, 2, 4, 8):
        r = run(path, n, args.seconds, args.hz)
        res["loaded"].append(r)
        print("loaded", r, flush=True)
    out, _ = burn.communicate(timeout=120)
    res["gemm_burn"] = out.strip()
    print("RESULT " + json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
