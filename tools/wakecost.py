#!/usr/bin/env python3
"""CPU a host charges a thread for one sleep -> timer wake-up, and how late the wake-up is.

A sampler or HTTP worker that sleeps between ticks pays this on every tick whatever its own work
is.  On a bare-metal MI355X host it is a few microseconds; on an overcommitted VM (this repo's
build container: 55-70 us of thread CPU per wake-up, 160-180 us late) it can exceed the whole
tick's work at 100 Hz, so tests/test_fakehost.py measures it on the host it runs on and charges
the exporter the MI355X host's figure instead (profiles/r06/host_cpu/).
Usage: python tools/wakecost.py [--hz 10,100] [--seconds 3]
"""
import argparse
import json
import time


def measure(hz: float, seconds: float) -> dict:
    """Thread CPU per wake-up (us) and mean wake-up lateness (us) of a periodic sleeper."""
    period = 1.0 / hz
    n = max(5, int(seconds * hz))
    t = time.monotonic() + period
    late = 0.0
    cpu = 0
    for _ in range(n):
        c0 = time.thread_time_ns()
        time.sleep(max(0.0, t - time.monotonic()))
        late += time.monotonic() - t
        cpu += time.thread_time_ns() - c0
        t += period
    return {"hz": hz, "wakeups": n, "cpu_us_per_wakeup": cpu / n / 1e3, "late_us": late / n * 1e6}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hz", default="10,100")
    ap.add_argument("--seconds", type=float, default=3.0)
    args = ap.parse_args()
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from kubernetes_gpu_exporter_amd._native import load
    native = load()
    for hz in (float(x) for x in args.hz.split(",")):
        r = measure(hz, args.seconds)
        # the sampler's own wait (timerfd + poll in C++), as the exporter pays it
        cpu, late = native.timer_wakeup_cost(hz, max(5, int(args.seconds * hz)))
        r.update({"native_cpu_us_per_wakeup": cpu / 1e3, "native_late_us": late / 1e3})
        r = {("python_" + k if k in ("cpu_us_per_wakeup", "late_us") else k): v for k, v in r.items()}
        print(json.dumps({k: round(v, 2) if isinstance(v, float) else v for k, v in r.items()}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
