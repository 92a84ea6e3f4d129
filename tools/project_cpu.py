#!/usr/bin/env python3
"""Exporter CPU projection for 1/2/4/8 MI355X from a fake-host node (profiles/r04/
cpu_projection.txt; VERDICT r03 task 2).

The engine runs in this process on the sysfs backend over a fake /sys + /proc tree
(utils/fakehost.py: MI355X topology, 4 GPU processes per GPU attributed to a pod), full
series profile, and burns the measured thread CPU of a real SMU fetch on every fresh
gpu_metrics read (--fetch-us, from tools/probe_fetch_cost.py on MI355X).  Whole-process CPU
(getrusage: every thread) over a steady window, with the shipped fetch policy
(metrics_min_interval auto, --budget % of one core for all GPUs' fetches) and, for
comparison, with every tick fetching (metrics_min_interval 0).  A projection of the
per-GPU costs, not a measurement of an 8-GPU node (the driver's SCALE run is that).
Round 6: the GPU-side sources are in the projection too -- the real PMC read machine on fake
GPUs at --pmc-us of CPU per GPU per round and a sentinel at --sentinel-us per GPU per run
(fake_sources.cc) -- so its counters and sentinel stages scale with the GPU count.
Usage: python tools/project_cpu.py [--fetch-us 206,450] [--hz 10,100] [--seconds 4]
"""
import argparse
import os
import resource
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


SCRAPER = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
from kubernetes_gpu_exporter_amd._native import load
n = load()
c = n.ScrapeClient("127.0.0.1", int(sys.argv[2]), "/metrics", sys.argv[4] == "gzip", 5000, "", True)
period = 1.0 / float(sys.argv[3])
t = time.perf_counter()
while True:
    c.scrape()
    t += period
    time.sleep(max(0.0, t - time.perf_counter()))
"""


def measure(native, n_gpus: int, hz: float, fetch_us: int, policy: str, budget: float, seconds: float,
            scrape: str = "none", exposition: str = "compiled", warmup: float = -1.0, pmc_us: int = -1,
            sentinel_us: int = -1, scrape_hz: float = 0.0, render_when_due: bool = True) -> dict:
    # warm-up: long enough for the exposition to settle (a family's real parse comes 8 renders after
    # its last layout; the scraper's first gzip ask starts the gzip copies): 20 ticks, at least 1 s
    if warmup < 0:
        warmup = max(1.0, 20.0 / hz)
    import subprocess
    import test_fakehost as tf
    root = tempfile.mkdtemp(prefix="gpuexp-proj-")
    tf._loaded_node(root, n_gpus)
    c = native.EngineConfig()
    c.backend = "sysfs"
    c.host_root = root
    c.interval_s = 1.0 / hz
    c.serve_http = scrape != "none"
    if c.serve_http:
        h = c.http
        h.port = 0
        h.host = "127.0.0.1"
        c.http = h
    c.series_profile = "full"
    if hasattr(c, "exposition"):  # (an older tree, --root, has only the classic one)
        c.exposition = exposition
    c.fake_metrics_cost_us = fetch_us
    if pmc_us >= 0 and hasattr(c, "fake_pmc_cost_us"):  # the real PMC read machine on fake GPUs
        c.enable_counters = True
        c.fake_pmc_cost_us = pmc_us
    if sentinel_us >= 0 and hasattr(c, "fake_sentinel_cost_us"):
        c.enable_sentinel = True
        c.fake_sentinel_cost_us = sentinel_us
    c.metrics_min_interval_s = -1.0 if policy == "auto" else 0.0
    if hasattr(c, "render_when_due"):
        c.render_when_due = render_when_due
    c.metrics_cpu_budget = budget / 100.0
    e = native.Engine(c)
    e.start()
    scraper = None
    if scrape != "none":  # another process, so its CPU is not the exporter's
        scraper = subprocess.Popen([sys.executable, "-c", SCRAPER, PKG_ROOT, str(e.http_port), str(scrape_hz or hz),
                                    scrape])
    try:
        time.sleep(warmup)
        if hasattr(e, "reset_tick_max"):
            e.reset_tick_max()
        r0, t0, s0 = resource.getrusage(resource.RUSAGE_SELF), time.perf_counter(), e.stats()
        time.sleep(seconds)
        r1, t1, s1 = resource.getrusage(resource.RUSAGE_SELF), time.perf_counter(), e.stats()
    finally:
        if scraper:
            scraper.kill()
            scraper.wait()
        e.stop()
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    ticks = max(1, s1["ticks"] - s0["ticks"])
    stages = {k: round((s1["stage_cpu_ns"][k] - s0["stage_cpu_ns"][k]) / ticks / 1e3, 1) for k in s1["stage_cpu_ns"]}
    return {"gpus": n_gpus, "hz": hz, "fetch_us": fetch_us, "policy": policy, "scrape": scrape,
            "exposition": exposition, "body_bytes": s1.get("render_bytes"),
            "process_cpu_pct": round(100.0 * cpu / (t1 - t0), 2),
            "sampler_us_per_tick": round((s1["sampler_cpu_ns"] - s0["sampler_cpu_ns"]) / ticks / 1e3, 1),
            "stage_us_per_tick": stages,
            "relayouts_per_tick": round((s1.get("relayouts", 0) - s0.get("relayouts", 0)) / ticks, 3),
            "code_builds": s1.get("code_builds", 0) - s0.get("code_builds", 0),
            "tick_wall_mean_us": round((s1.get("tick_ns_total", 0) - s0.get("tick_ns_total", 0)) / ticks / 1e3, 1),
            "tick_wall_max_us": round(s1.get("max_tick_ns", 0) / 1e3, 1),
            # the sampler thread's CPU per tick: the work a tick carries, whatever preempts it
            "tick_cpu_mean_us": round((s1.get("tick_cpu_ns_total", 0) - s0.get("tick_cpu_ns_total", 0)) / ticks / 1e3, 1),
            "tick_cpu_max_us": round(s1.get("max_tick_cpu_ns", 0) / 1e3, 1)}


PKG_ROOT = ROOT


def main() -> int:
    global PKG_ROOT
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=ROOT, help="tree whose built package to measure (e.g. an older round's)")
    ap.add_argument("--fetch-us", default="206,450")
    ap.add_argument("--hz", default="10,100")
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--budget", type=float, default=0.75)
    ap.add_argument("--pmc-us", type=int, default=14,
                    help="CPU per GPU per PMC read round (fake GPUs under the real read machine; -1 = no counters)")
    ap.add_argument("--sentinel-us", type=int, default=4, help="CPU per GPU per sentinel run (-1 = no sentinel)")
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--warmup", type=float, default=-1.0, help="seconds before measuring (default: 20 ticks, >= 1 s)")
    ap.add_argument("--policies", default="auto,every")
    ap.add_argument("--scrape", default="none", help="none | gzip | identity: a scraper process at the tick rate")
    ap.add_argument("--scrape-hz", type=float, default=0.0, help="the scraper's rate (default: the tick rate)")
    ap.add_argument("--render-when-due", default="1", help="1 | 0 | 1,0 (compare)")
    ap.add_argument("--exposition", default="compiled", help="compiled | classic (comma list to compare)")
    ap.add_argument("--stages", action="store_true", help="also print the sampler thread's CPU per stage")
    args = ap.parse_args()
    PKG_ROOT = os.path.abspath(args.root)
    sys.path.insert(0, PKG_ROOT)
    from kubernetes_gpu_exporter_amd._native import load
    native = load()
    print(f"# fake-host projection, full profile, 4 processes/GPU, budget {args.budget} % (auto policy), "
          f"PMC {args.pmc_us} us + sentinel {args.sentinel_us} us CPU per GPU per round / run")
    print(f"{'gpus':>4} {'hz':>5} {'fetch_us':>8} {'policy':>6} {'cpu_%':>7} {'sampler_us/tick':>15} "
          f"{'tick_mean_us':>12} {'tick_max_us':>11} {'cpu_mean_us':>11} {'cpu_max_us':>10}  exposition")
    for fetch in (int(x) for x in args.fetch_us.split(",")):
        for hz in (float(x) for x in args.hz.split(",")):
            for n in (int(x) for x in args.gpus.split(",")):
                for policy in args.policies.split(","):
                  for expo in args.exposition.split(","):
                   for rwd in args.render_when_due.split(","):
                    r = measure(native, n, hz, fetch, policy, args.budget, args.seconds, args.scrape, expo, args.warmup,
                                args.pmc_us, args.sentinel_us, args.scrape_hz, rwd == "1")
                    print(f"{r['gpus']:>4} {r['hz']:>5g} {r['fetch_us']:>8} {r['policy']:>6} "
                          f"{r['process_cpu_pct']:>7.2f} {r['sampler_us_per_tick']:>15.1f} "
                          f"{r['tick_wall_mean_us']:>12.1f} {r['tick_wall_max_us']:>11.1f} "
                          f"{r['tick_cpu_mean_us']:>11.1f} {r['tick_cpu_max_us']:>10.1f}  "
                          f"{expo} scrape={args.scrape}"
                          + (f"@{args.scrape_hz:g}Hz" if args.scrape_hz else "")
                          + ("" if rwd == "1" else " render_when_due=0"), flush=True)
                    if args.stages:
                        print("      stage us/tick: " + " ".join(f"{k}={v}" for k, v in r["stage_us_per_tick"].items())
                              + f"  relayouts/tick={r['relayouts_per_tick']} code_builds={r['code_builds']}"
                              + f" body={r['body_bytes']}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
