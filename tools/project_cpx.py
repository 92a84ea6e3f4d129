#!/usr/bin/env python3
"""Tick CPU of a partitioned MI355X node on the fake host: 8 sockets in CPX mode = 64 logical
GPUs (--sockets / --partitions), one GPU process on each, full profile, with the silicon
stand-ins (382 us per fresh SMU fetch, 14 us per PMC read per logical GPU, 4 us per sentinel
run).  Ticks run back to back on a simulated clock (tools/tickbench.py's method: the tick's
own work, warm, without the host's wake-up cost).  Shows that a socket's partitions share one
SMU fetch (fetches per tick ~ sockets / phases, not logical GPUs / phases) and where a 64-GPU
tick's CPU goes.  Usage: python tools/project_cpx.py [--sockets 8] [--partitions 8] [--hz 10,100]
"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sockets", type=int, default=8)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--hz", default="10,100")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--counters-budget", type=float, default=0.75, help="%% of one core (0 = no cap)")
    args = ap.parse_args()
    from kubernetes_gpu_exporter_amd._native import load
    from kubernetes_gpu_exporter_amd.utils.fakehost import kubepods_cgroup, mi355x_cpx_node
    import test_fakehost as tf
    n = load()
    root = tempfile.mkdtemp(prefix="gpuexp-cpx-")
    h = mi355x_cpx_node(root, args.sockets, args.partitions)
    for i, g in enumerate(h.gpus):
        h.set_metrics(g, gfx=50, accum=1000, num_partition=args.partitions)
        h.add_process(5000 + i, kubepods_cgroup(tf.UID, tf.CID), gpus={g.gpu_id: (1 << 30, 8)})
    devs = n.read_backend("sysfs", root)
    print(f"# {len(devs)} logical GPUs on {len({d['bdf'] for d in devs})} sockets, full profile, "
          f"1 process each; tick work on a simulated clock (warm, no wake-ups)")
    for hz in (float(x) for x in args.hz.split(",")):
        c = n.EngineConfig()
        c.backend = "sysfs"
        c.host_root = root
        c.interval_s = 1.0 / hz
        c.sampler_thread = False
        c.serve_http = False
        c.series_profile = "full"
        c.fake_metrics_cost_us = tf.SMU_FETCH_CPU_US
        c.enable_counters = c.enable_sentinel = True
        c.fake_pmc_cost_us = tf.PMC_READ_CPU_US
        c.fake_sentinel_cost_us = tf.SENTINEL_RUN_CPU_US
        c.counters_cpu_budget = args.counters_budget / 100.0
        e = n.Engine(c)
        e.start()
        try:
            now, per = time.monotonic_ns(), int(1e9 / hz)
            for _ in range(int(2 * hz)):
                now += per
                e.tick(now)
            s0, c0, k = e.stats(), time.thread_time_ns(), int(args.seconds * hz)
            per_tick = []
            for _ in range(k):
                now += per
                t = time.thread_time_ns()
                e.tick(now)
                per_tick.append(time.thread_time_ns() - t)
            cpu = (time.thread_time_ns() - c0) / k / 1e3
            s1 = e.stats()
        finally:
            e.stop()
        fake = (s1["fake_cpu_burnt_ns"] - s0["fake_cpu_burnt_ns"]) / k / 1e3
        stages = " ".join(f"{s}={(s1['stage_cpu_ns'][s] - s0['stage_cpu_ns'][s]) / k / 1e3:.1f}"
                          for s in s1["stage_cpu_ns"])
        print(f"{hz:g} Hz: tick {cpu:.0f} us ({cpu * hz / 1e4:.2f} % of a core), of which silicon stand-ins "
              f"{fake:.0f} us; SMU fetches per tick {(s1['fresh_reads'] - s0['fresh_reads']) / k:.2f}; "
              f"PMC rounds every {s1['counters_round_interval_s'] * 1e3:.0f} ms "
              f"({s1['counters_round_cpu_ns'] / 1e3:.0f} us each); heaviest tick {max(per_tick) / (sum(per_tick) / k):.2f}x the mean; {s1['series']} series, {s1['render_bytes']} B body\n    stage us/tick: {stages}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
