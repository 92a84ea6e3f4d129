#!/usr/bin/env python3
"""CPU charged to a thread per sleep/wake-up cycle on this host (schedstat run time of a
child that only sleeps), at 1, 10 and 100 wake-ups per second.

Why: the exporter's CPU at 10 Hz is a few hundred microseconds per tick, and every extra
wake-up per tick (sampler timer, HTTP pre-wake slices, the PMC thread, a Python wait loop)
costs what this host charges for one: a few microseconds on bare metal, ~80-160 us in the
build container (a VM).  profiles/r04/wakeup_cost*.txt.
Usage: python tools/probe_wakeup_cost.py [--seconds 3]
"""
import argparse
import json
import os
import subprocess
import sys
import time

CHILD = "import time\np={p}\nnxt=time.monotonic()\nwhile True:\n    nxt+=p\n    time.sleep(max(0.0,nxt-time.monotonic()))\n"


def run(hz: float, seconds: float) -> dict:
    p = subprocess.Popen([sys.executable, "-c", CHILD.format(p=1.0 / hz)])
    try:
        time.sleep(1.0)

        def snap():
            st = open(f"/proc/{p.pid}/status").read()
            vol = int([l for l in st.splitlines() if l.startswith("voluntary_ctxt")][0].split()[1])
            return vol, int(open(f"/proc/{p.pid}/schedstat").read().split()[0])

        a = snap()
        time.sleep(seconds)
        b = snap()
    finally:
        p.terminate()
        p.wait()
    wakes = max(1, b[0] - a[0])
    return {"hz": hz, "wakeups": wakes, "cpu_us_per_wakeup": round((b[1] - a[1]) / 1e3 / wakes, 2),
            "cpu_percent": round((b[1] - a[1]) / 1e7 / seconds, 4)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    args = ap.parse_args()
    rows = [run(hz, args.seconds) for hz in (1.0, 10.0, 100.0)]
    for r in rows:
        print(f"{r['hz']:>6.0f} Hz: {r['wakeups']:>5} wake-ups, {r['cpu_us_per_wakeup']:>8.2f} us CPU each, "
              f"{r['cpu_percent']:.4f} % of a core", flush=True)
    print("RESULT " + json.dumps({"host": os.uname().nodename, "rows": rows}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
