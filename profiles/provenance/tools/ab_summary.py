#!/usr/bin/env python3
"""Summarises tools/devices_ab.sh results (gpurun_out/ab/<arm>.<rep>.json): per arm, the
median over reps of p50 scrape, exporter CPU, the devices stage, sampler CPU per tick, the
devices stage's parts and the CPU of one fresh gpu_metrics fetch.
Usage: python tools/ab_summary.py [gpurun_out/ab]"""
import glob
import json
import os
import statistics
import sys


def main() -> int:
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
    arms: dict = {}
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        arm = os.path.basename(f).split(".")[0]
        try:
            arms.setdefault(arm, []).append(json.load(open(f)))
        except (OSError, ValueError):
            continue

    def med(rows, get):
        v = [get(r) for r in rows]
        v = [x for x in v if x is not None]
        return round(statistics.median(v), 1) if v else None

    print(f"{'arm':>6} {'n':>2} {'p50_us':>7} {'cpu_%':>6} {'devices_us':>10} {'sampler_us/tick':>15} "
          f"{'fetch_cpu_us':>12}  parts_us/tick (median)")
    for arm, rows in arms.items():
        parts = {}
        for r in rows:
            for k, v in (r.get("device_read_mean_us_per_tick") or {}).items():
                parts.setdefault(k, []).append(v)
        pm = {k: round(statistics.median(v), 1) for k, v in sorted(parts.items())}
        print(f"{arm:>6} {len(rows):>2} {med(rows, lambda r: r.get('value')):>7} "
              f"{med(rows, lambda r: r.get('exporter_cpu_percent')):>6} "
              f"{med(rows, lambda r: (r.get('sample_stage_mean_us') or {}).get('devices')):>10} "
              f"{med(rows, lambda r: r.get('sampler_cpu_us_per_tick')):>15} "
              f"{str(med(rows, lambda r: r.get('gpu_metrics_fetch_cpu_us_per_fresh_read_gpu0'))):>12}  {pm}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
