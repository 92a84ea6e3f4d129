#!/usr/bin/env python3
"""What unit is KFD's per-process sdma_<gpu_id> file in, on MI355X?

amd_gpu_process_sdma_seconds_total reads /sys/class/kfd/kfd/proc/<pid>/sdma_<gpu_id> as
microseconds of SDMA time.  A bench exposition (profiles/r04/session5) showed 1.26e6 "s" for
a 30 s process, so the unit is checked here: a child runs copy phases of known wall time
(pageable H2D / D2H, pinned H2D / D2H, D2D, idle) and this process reads the child's raw
sdma_<id> value around each phase.
Usage: python tools/probe_sdma_units.py [--seconds 1.5] -> RESULT json
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import time

CHILD = r"""
import sys, time, torch
sys.path.insert(0, {root!r})
from kubernetes_gpu_exporter_amd.utils.kfdself import find_own_kfd_pid
torch.zeros(1, device="cuda:0"); torch.cuda.synchronize()
hostpid = find_own_kfd_pid(0)  # KFD names processes by host PID (the box may be a container)
dev = torch.empty(256 << 20, dtype=torch.uint8, device="cuda:0")
dev2 = torch.empty_like(dev)
page = torch.empty(256 << 20, dtype=torch.uint8)
pin = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
phases = {
    "idle": lambda: time.sleep(0.01),
    "h2d_pageable": lambda: dev.copy_(page),
    "d2h_pageable": lambda: page.copy_(dev),
    "h2d_pinned": lambda: dev.copy_(pin, non_blocking=True),
    "d2h_pinned": lambda: pin.copy_(dev, non_blocking=True),
    "d2d": lambda: dev2.copy_(dev),
}
print("ready", hostpid, flush=True)
for line in sys.stdin:
    name, secs = line.split()
    t0 = time.perf_counter(); n = 0
    while time.perf_counter() - t0 < float(secs):
        phases[name](); n += 1
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    bytes_ = 0 if name == "idle" else n * (256 << 20)
    print(f"done {dt:.4f} {bytes_}", flush=True)
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=1.5)
    args = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.Popen([sys.executable, "-c", CHILD.replace("{root!r}", repr(root))], stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, text=True)
    ready = p.stdout.readline().split()
    assert ready and ready[0] == "ready", ready
    hostpid = int(ready[1]) if len(ready) > 1 and ready[1] != "None" else p.pid
    print("child pid", p.pid, "KFD pid", hostpid, flush=True)
    files = sorted(glob.glob(f"/sys/class/kfd/kfd/proc/{hostpid}/sdma_*"))
    print("files:", files, flush=True)

    def raw():
        out = {}
        for f in files:
            try:
                out[os.path.basename(f)] = int(open(f).read().strip() or 0)
            except (OSError, ValueError):
                out[os.path.basename(f)] = None
        return out

    rows = []
    for name in ("idle", "h2d_pageable", "d2h_pageable", "h2d_pinned", "d2h_pinned", "d2d", "idle"):
        a, t0 = raw(), time.monotonic()
        p.stdin.write(f"{name} {args.seconds}\n")
        p.stdin.flush()
        _, dt, nbytes = p.stdout.readline().split()
        b, t1 = raw(), time.monotonic()
        delta = {k: (b[k] - a[k]) if a.get(k) is not None and b.get(k) is not None else None for k in b}
        row = {"phase": name, "child_wall_s": float(dt), "read_wall_s": round(t1 - t0, 4),
               "GBps": round(int(nbytes) / float(dt) / 1e9, 2), "raw_before": a, "delta": delta}
        for k, v in delta.items():
            if v is not None:
                row[f"{k}_delta_per_wall_s"] = round(v / (t1 - t0), 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
    p.stdin.close()
    p.wait(timeout=60)
    print("RESULT " + json.dumps(rows), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
