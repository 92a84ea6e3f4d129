"""CPU accounting of a process from /proc/<pid>/stat (utime + stime), the BASELINE
"exporter CPU%" metric: 100 * d(cpu seconds) / d(wall seconds) (percent of one core)."""
from __future__ import annotations

import os
import time


def cpu_seconds(pid: int) -> float:
    with open(f"/proc/{pid}/stat") as fh:
        s = fh.read()
    rest = s[s.rindex(")") + 2:].split()
    # fields after comm: state(3) ... utime(14) stime(15) -> indices 11, 12 in `rest`
    utime, stime = int(rest[11]), int(rest[12])
    return (utime + stime) / os.sysconf("SC_CLK_TCK")


def cpu_seconds_precise(pid: int) -> float:
    """Sum of per-thread run time (ns resolution, /proc/<pid>/task/*/schedstat); falls back
    to the 10 ms-granular utime+stime of /proc/<pid>/stat."""
    total = 0
    try:
        for tid in os.listdir(f"/proc/{pid}/task"):
            try:
                with open(f"/proc/{pid}/task/{tid}/schedstat") as fh:
                    total += int(fh.read().split()[0])
            except OSError:
                continue
    except OSError:
        return cpu_seconds(pid)
    return total * 1e-9 if total else cpu_seconds(pid)


def thread_cpu_ns_by_name(pid: int) -> dict:
    """Run time (ns, schedstat) of `pid`'s threads summed per thread name: where an
    exporter's CPU goes (gpuexp-sampler, gpuexp-http, the PMC thread, Python ...)."""
    out: dict = {}
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"/proc/{pid}/task/{tid}/comm") as fh:
                name = fh.read().strip()
            with open(f"/proc/{pid}/task/{tid}/schedstat") as fh:
                ns = int(fh.read().split()[0])
        except (OSError, ValueError, IndexError):
            continue
        out[name] = out.get(name, 0) + ns
    return out


def thread_cpu_seconds(pid: int) -> dict:
    """Per-thread CPU seconds, keyed by thread name (sampler / http / python ...)."""
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    for tid in os.listdir(f"/proc/{pid}/task"):
        try:
            with open(f"/proc/{pid}/task/{tid}/stat") as fh:
                s = fh.read()
        except OSError:
            continue
        name = s[s.index("(") + 1:s.rindex(")")]
        rest = s[s.rindex(")") + 2:].split()
        out[f"{name}:{tid}"] = (int(rest[11]) + int(rest[12])) / tck
    return out


class CpuMeter:
    """Measures CPU% of `pid` between start() and stop()."""

    def __init__(self, pid: int):
        self.pid = pid
        self.c0 = self.t0 = 0.0
        self.percent = float("nan")
        self.cpu_s = 0.0
        self.wall_s = 0.0

    def start(self) -> "CpuMeter":
        self.c0 = cpu_seconds(self.pid)
        self.t0 = time.monotonic()
        return self

    def stop(self) -> float:
        self.cpu_s = cpu_seconds(self.pid) - self.c0
        self.wall_s = time.monotonic() - self.t0
        self.percent = 100.0 * self.cpu_s / self.wall_s if self.wall_s > 0 else float("nan")
        return self.percent
