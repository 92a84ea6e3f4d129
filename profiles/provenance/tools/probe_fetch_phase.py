#!/usr/bin/env python3
"""Does a gpu_metrics fetch cost less CPU at some phase of the PMFW's own table refresh?

A fresh read of gpu_metrics is one SMU message the kernel busy-waits on (130-460 us of CPU on
MI355X, most of the exporter's CPU at one GPU).  The PMFW regenerates the table on its own
period (the firmware timestamp in the blob steps by it); if the SMU answers slower while it is
busy with that, a sampler could phase-lock its fetch to the quiet part of the period.

Reads the real gpu_metrics file at random intervals (2-40 ms) while a child process keeps the
GPU busy with the bf16 GEMM pod kernel; records each read's thread CPU, wall time and the
table's firmware timestamp.  The table's age at each read is the read's host time minus the
firmware timestamp (in the host clock: offset by the smallest such difference, so the freshest
read is age 0); reads are binned by age / PMFW period.
Usage: python tools/probe_fetch_phase.py [--seconds 40] -> table + RESULT json
"""
import argparse
import glob
import json
import os
import random
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=40.0)
    ap.add_argument("--bins", type=int, default=10)
    ap.add_argument("--no-load", action="store_true")
    args = ap.parse_args()
    from kubernetes_gpu_exporter_amd._native import load
    native = load()
    path = sorted(glob.glob("/sys/class/drm/renderD*/device/gpu_metrics"))[0]
    burn = None
    if not args.no_load:
        burn = subprocess.Popen([sys.executable, "-c",
                                 "import sys; sys.path.insert(0, %r)\n"
                                 "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn\n"
                                 "print(gemm_burn(0, 8192, %f), flush=True)" % (ROOT, args.seconds + 8)],
                                stdout=subprocess.PIPE, text=True)
        time.sleep(4.0)
    fd = os.open(path, os.O_RDONLY)
    rng = random.Random(1)
    rows = []
    stop = time.monotonic() + args.seconds
    last_print = time.monotonic()
    while time.monotonic() < stop:
        time.sleep(rng.uniform(0.002, 0.040))
        c0, w0 = time.thread_time_ns(), time.monotonic_ns()
        blob = os.pread(fd, 16384, 0)
        c1, w1 = time.thread_time_ns(), time.monotonic_ns()
        raw = native.decode_gpu_metrics_raw(blob)
        if raw is None:
            continue
        rows.append((w0, (c1 - c0) / 1e3, (w1 - w0) / 1e3, int(raw["firmware_timestamp"])))
        if time.monotonic() - last_print > 10:
            last_print = time.monotonic()
            print(f"{len(rows)} reads", flush=True)
    os.close(fd)
    if burn:
        burn.wait(timeout=120)
    # PMFW period from the firmware timestamp's steps (10 ns units)
    ts = sorted({r[3] for r in rows})
    steps = [b - a for a, b in zip(ts, ts[1:]) if b > a]
    period_ns = statistics.median(steps) * 10 if steps else 0
    # host-minus-firmware clock offset, tracked over the run (the two clocks drift by ppm, which
    # over tens of seconds is more than a period): the freshest read of each of 16 time chunks
    # gives the offset there, interpolated linearly in between
    ages_raw = [r[0] - r[3] * 10 for r in rows]
    nchunk = 16
    t_first, t_last = rows[0][0], rows[-1][0]
    span = max(1, t_last - t_first)
    knots = []
    for k in range(nchunk):
        idx = [i for i, r in enumerate(rows) if k * span // nchunk <= r[0] - t_first < (k + 1) * span // nchunk + (k == nchunk - 1)]
        if idx:
            i0 = min(idx, key=lambda i: ages_raw[i])
            knots.append((rows[i0][0], ages_raw[i0]))

    def offset(t):
        if len(knots) == 1 or t <= knots[0][0]:
            return knots[0][1]
        for (ta, oa), (tb, ob) in zip(knots, knots[1:]):
            if t <= tb:
                return oa + (ob - oa) * (t - ta) / max(1, tb - ta)
        return knots[-1][1]

    ages_raw = [ar - offset(r[0]) for r, ar in zip(rows, ages_raw)]
    a0 = min(ages_raw)
    out = {"path": path, "reads": len(rows), "pmfw_period_us": round(period_ns / 1e3, 1),
           "cpu_us_p50": round(statistics.median(r[1] for r in rows), 1), "bins": []}
    ages = sorted(ar - a0 for ar in ages_raw)
    out["age_us_p10_p50_p90"] = [round(ages[int(q * (len(ages) - 1))] / 1e3, 1) for q in (0.1, 0.5, 0.9)]
    print(f"# {len(rows)} reads, PMFW period {period_ns / 1e3:.1f} us (median firmware-timestamp step), "
          f"cpu p50 {out['cpu_us_p50']} us; table age at the read p10/p50/p90 {out['age_us_p10_p50_p90']} us")
    print("# age/period bin   reads   cpu_us_p50   cpu_us_mean   wall_us_p50")
    if period_ns > 0:
        bins = [[] for _ in range(args.bins)]
        for r, ar in zip(rows, ages_raw):
            ph = ((ar - a0) % period_ns) / period_ns
            bins[min(args.bins - 1, int(ph * args.bins))].append(r)
        for k, b in enumerate(bins):
            if not b:
                continue
            row = {"bin": k, "reads": len(b), "cpu_us_p50": round(statistics.median(x[1] for x in b), 1),
                   "cpu_us_mean": round(statistics.mean(x[1] for x in b), 1),
                   "wall_us_p50": round(statistics.median(x[2] for x in b), 1)}
            out["bins"].append(row)
            print(f"  {k / args.bins:4.1f}-{(k + 1) / args.bins:3.1f}   {row['reads']:6d}   {row['cpu_us_p50']:10.1f}"
                  f"   {row['cpu_us_mean']:11.1f}   {row['wall_us_p50']:11.1f}")
    print("RESULT " + json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
