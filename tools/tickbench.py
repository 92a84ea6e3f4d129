#!/usr/bin/env python3
"""Per-tick CPU of the sampler's work on a fake-host node, without the host's wake-up cost.

The engine runs without its sampler thread (EngineConfig.sampler_thread = False); this thread
calls Engine.tick(now) back to back on a simulated clock advancing one period per tick, so every
interval-derived policy (the auto SMU fetch cap and its per-GPU phases, PMC rounds at most every
counters_min_interval, the sentinel at most every sentinel_min_interval) is what the sampler
would run.  What it leaves out is the sleep between ticks: on a VM whose hypervisor charges
50-70 us of thread CPU per timer wake-up (this build container), a 100 Hz tick's work is then
measured apart from the host's idle-exit cost, which tools/wakecost.py measures on its own.

Same fake node as tests/test_fakehost.py (MI355X topology, 4 GPU processes per GPU, full
profile), the SMU fetch's measured CPU burnt per fresh gpu_metrics read, the real PMC read
machine on fake GPUs and a fake sentinel at their silicon per-GPU costs.
Usage: python tools/tickbench.py [--gpus 8] [--hz 100] [--ticks 3000] [--repeat 3]
"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(native, root: str, hz: float, ticks: int, fetch_us: int, sleep_s: float = 0.0) -> dict:
    import test_fakehost as tf
    c = native.EngineConfig()
    c.backend = "sysfs"
    c.host_root = root
    c.interval_s = 1.0 / hz
    c.sampler_thread = False
    c.serve_http = False
    c.series_profile = "full"
    c.fake_metrics_cost_us = fetch_us
    c.enable_counters = c.enable_sentinel = True
    c.fake_pmc_cost_us = tf.PMC_READ_CPU_US
    c.fake_sentinel_cost_us = tf.SENTINEL_RUN_CPU_US
    e = native.Engine(c)
    e.start()
    period = int(1e9 / hz)
    now = time.monotonic_ns()
    try:
        for _ in range(max(50, int(2 * hz))):  # past the exposition's settle and the fetch phases
            now += period
            e.tick(now)
        s0 = e.stats()
        cpu = 0
        for _ in range(ticks):
            now += period
            if sleep_s:
                time.sleep(sleep_s)
            c0 = time.thread_time_ns()
            e.tick(now)
            cpu += time.thread_time_ns() - c0
        s1 = e.stats()
    finally:
        e.stop()
    n = max(1, s1["ticks"] - s0["ticks"])
    stages = {k: (s1["stage_cpu_ns"][k] - s0["stage_cpu_ns"][k]) / n / 1e3 for k in s1["stage_cpu_ns"]}
    return {"cpu_us_per_tick": cpu / n / 1e3,
            "tick_cpu_us": (s1["tick_cpu_ns_total"] - s0["tick_cpu_ns_total"]) / n / 1e3,
            "pct_at_hz": cpu / n / 1e9 * hz * 100.0, "stages": stages}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="8")
    ap.add_argument("--hz", default="100")
    ap.add_argument("--ticks", type=int, default=3000)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--fetch-us", type=int, default=382)
    ap.add_argument("--sleep-ms", type=float, default=0.0,
                    help="sleep between ticks (caches cool down as a sampler's do; its wake-up is not counted)")
    args = ap.parse_args()
    from kubernetes_gpu_exporter_amd._native import load
    import test_fakehost as tf
    native = load()
    print("# tick work only (no wake-ups): median of --repeat runs; stage CPU per tick (us)")
    for g in (int(x) for x in args.gpus.split(",")):
        root = tempfile.mkdtemp(prefix="gpuexp-tb-")
        tf._loaded_node(root, g)
        for hz in (float(x) for x in args.hz.split(",")):
            rs = sorted((run(native, root, hz, args.ticks, args.fetch_us, args.sleep_ms / 1e3) for _ in range(args.repeat)),
                        key=lambda r: r["cpu_us_per_tick"])
            r = rs[len(rs) // 2]
            st = " ".join(f"{k}={v:.1f}" for k, v in r["stages"].items())
            each = ", ".join(f"{x['cpu_us_per_tick']:.1f}" for x in rs)
            print(f"gpus={g} hz={hz:g} tick_cpu={r['cpu_us_per_tick']:.1f} us "
                  f"({r['pct_at_hz']:.2f} % at {hz:g} Hz; runs {each})"
                  f"\n    {st}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
