#!/usr/bin/env python3
"""GPU-box probe: CPU time (this thread's user+sys, CLOCK_THREAD_CPUTIME_ID) and wall time
of each per-tick sysfs read the sampler does, at 10 Hz spacing (cold caches, as in the
engine): gpu_metrics (PMFW table via the SMU), mem_info_vram_used, and the KFD per-process
directory listing.  Usage: python tools/probe_read_costs.py [n=40] [hz=10]"""
import glob
import os
import statistics
import sys
import time


def cost(fn, n, hz):
    cpu, wall = [], []
    for _ in range(n):
        time.sleep(1.0 / hz)
        c0, w0 = time.thread_time_ns(), time.perf_counter_ns()
        fn()
        cpu.append((time.thread_time_ns() - c0) / 1e3)
        wall.append((time.perf_counter_ns() - w0) / 1e3)
    return round(statistics.median(cpu), 1), round(statistics.median(wall), 1), round(max(wall), 1)


def main() -> int:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    hz = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    dev = sorted(glob.glob("/sys/class/drm/renderD*/device/gpu_metrics"))[0].rsplit("/", 1)[0]
    fd_gm = os.open(dev + "/gpu_metrics", os.O_RDONLY)
    fd_vr = os.open(dev + "/mem_info_vram_used", os.O_RDONLY)
    probes = {
        "gpu_metrics pread": lambda: os.pread(fd_gm, 8192, 0),
        "mem_info_vram_used pread": lambda: os.pread(fd_vr, 64, 0),
        "kfd proc listdir": lambda: os.listdir("/sys/class/kfd/kfd/proc"),
        "getpid (floor)": lambda: os.getpid(),
    }
    print(f"{'read':28s} {'cpu_us_p50':>10s} {'wall_us_p50':>11s} {'wall_us_max':>11s}   ({n} reads at {hz} Hz)")
    for name, fn in probes.items():
        c, w, m = cost(fn, n, hz)
        print(f"{name:28s} {c:10.1f} {w:11.1f} {m:11.1f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
