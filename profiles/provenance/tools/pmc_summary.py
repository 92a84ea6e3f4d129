#!/usr/bin/env python3
"""Summarises a rocprofv3 --pmc rocpd database: median per-dispatch value of every counter
for kernels whose name contains a pattern.  Usage: pmc_summary.py <results.db> <pattern>"""
import sqlite3
import statistics
import sys


def main() -> int:
    db, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(db)
    per: dict = {}
    dur: dict = {}
    for name, disp, ctr, val, d in c.execute(
            "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
        if pat and pat not in str(name):
            continue
        per[(disp, ctr)] = per.get((disp, ctr), 0.0) + float(val)  # sum over dimensions per dispatch
        dur[disp] = d
    if dur:
        print(f"{'dispatch duration (ns)':32s} n={len(dur):5d} median={statistics.median(dur.values()):.6g}")
    by_ctr: dict = {}
    for (_, ctr), v in per.items():
        by_ctr.setdefault(ctr, []).append(v)
    for ctr, vs in sorted(by_ctr.items()):
        print(f"{ctr:32s} n={len(vs):5d} median={statistics.median(vs):.6g}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
