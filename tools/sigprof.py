#!/usr/bin/env python3
"""Where the exporter's tick spends CPU, on a fake-host node (no perf in the image).

Drives Engine.tick() in this thread over a fake /sys + /proc tree (utils/fakehost.py,
full profile, 4 GPU processes per GPU) under tools/sigprof.cc's ITIMER_PROF sampler and
prints self and inclusive sample shares per function.  The SMU fetch is not simulated
(fake_metrics_cost_us 0): this profiles everything else a tick does.
Usage: python tools/sigprof.py [--gpus 8] [--ticks 20000] [--top 40] [--gzip] [--backend amdsmi]
(--backend amdsmi: GPU 0 of a GPU box, sentinel and PMC counters on, the SMU fetch real)
"""
import argparse
import bisect
import collections
import ctypes
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def build_lib() -> str:
    out = os.path.join(tempfile.gettempdir(), "libgpuexp_sigprof.so")
    src = os.path.join(ROOT, "tools", "sigprof.cc")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-o", out, src, "-lrt"])
    return out


def leaf_lines(path: str, func: str, top: int = 25):
    """Source lines of the leaf PCs whose innermost frame is `func` (addr2line -i)."""
    samples, maps = [], []
    with open(path) as f:
        in_maps = False
        for line in f:
            if line.startswith("MAPS"):
                in_maps = True
                continue
            if not in_maps:
                samples.append([int(x, 16) for x in line.split()])
            else:
                p = line.split()
                if len(p) >= 6 and "x" in p[1]:
                    a, b = (int(x, 16) for x in p[0].split("-"))
                    maps.append((a, b, int(p[2], 16), p[5]))
    maps.sort()
    starts = [m[0] for m in maps]
    cnt = collections.Counter()
    for s in samples:
        if len(s) < 3:
            continue
        pc = s[2]
        i = bisect.bisect_right(starts, pc) - 1
        if i >= 0 and pc < maps[i][1]:
            cnt[(maps[i][3], pc - maps[i][0] + maps[i][2])] += 1
    by_file = collections.defaultdict(list)
    for (fn, off), k in cnt.items():
        by_file[fn].append((off, k))
    lines = collections.Counter()
    for fn, lst in by_file.items():
        if not fn.startswith("/") or not os.path.exists(fn):
            continue
        r = subprocess.run(["addr2line", "-f", "-C", "-e", fn] + [hex(o) for o, _ in lst],
                           capture_output=True, text=True).stdout.splitlines()
        for j, (o, k) in enumerate(lst):
            if 2 * j + 1 >= len(r):
                break
            name, loc = r[2 * j], r[2 * j + 1]
            if func in name:
                lines[loc.split("/")[-1]] += k
    tot = sum(lines.values()) or 1
    for loc, k in lines.most_common(top):
        print(f"{100 * k / tot:6.1f}  {loc}")


def symbolize(path: str):
    samples, maps = [], []
    with open(path) as f:
        in_maps = False
        for line in f:
            if line.startswith("MAPS"):
                in_maps = True
                continue
            if not in_maps:
                samples.append([int(x, 16) for x in line.split()])
            else:
                p = line.split()
                if len(p) >= 6 and "x" in p[1]:
                    a, b = (int(x, 16) for x in p[0].split("-"))
                    maps.append((a, b, int(p[2], 16), p[5]))
    maps.sort()
    starts = [m[0] for m in maps]
    by_file = collections.defaultdict(set)

    def where(pc):
        i = bisect.bisect_right(starts, pc) - 1
        if i < 0 or pc >= maps[i][1]:
            return None
        return maps[i][3], pc - maps[i][0] + maps[i][2]

    for s in samples:
        for pc in s:
            w = where(pc - 1)
            if w:
                by_file[w[0]].add(w[1])
    names = {}
    for fn, offs in by_file.items():
        offs = sorted(offs)
        try:
            r = subprocess.run(["addr2line", "-f", "-C", "-e", fn] + [hex(o) for o in offs],
                               capture_output=True, text=True, timeout=120).stdout.splitlines()
        except Exception:
            r = []
        for k, o in enumerate(offs):
            nm = r[2 * k] if 2 * k < len(r) else "??"
            names[(fn, o)] = nm if nm != "??" else os.path.basename(fn) + "+" + hex(o)
    out = []
    for s in samples:
        frames = []
        for pc in s:
            w = where(pc - 1)
            frames.append(names.get(w, "?") if w else "?")
        out.append(frames)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--ticks", type=int, default=20000)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--hz", type=int, default=20000)
    ap.add_argument("--sleep-ms", type=float, default=10.0,
                    help="sleep between ticks (a sampler wakes with cold caches; 0 = back-to-back)")
    ap.add_argument("--gzip", action="store_true", help="serve HTTP with a 100 Hz gzip scraper (another process)")
    ap.add_argument("--exposition", default="compiled")
    ap.add_argument("--lines", default="", help="also print the source lines of leaf samples in this function")
    ap.add_argument("--tick-hz", type=float, default=0,
                    help="fake node: run the engine's interval policies for this tick rate (no sampler "
                         "thread; the SMU fetch, PMC reads and sentinel burn their silicon CPU, as in "
                         "tools/tickbench.py); 0 = every source every tick, no fetch cost")
    ap.add_argument("--backend", default="sysfs",
                    help="sysfs: the fake node; mock: simulated devices whose values change every tick; amdsmi: GPU 0 "
                         "of this host, with sentinel and PMC counters "
                         "(a GPU box; the SMU fetch is then real)")
    args = ap.parse_args()
    lib = ctypes.CDLL(build_lib())
    from kubernetes_gpu_exporter_amd._native import load
    native = load()
    c = native.EngineConfig()
    real = args.backend == "amdsmi"
    if real:
        from kubernetes_gpu_exporter_amd._native import rocprof_plugin_path
        c.backend = "amdsmi"
        c.device_filter = [0]
        c.enable_sentinel = True
        c.enable_counters = True
        c.counters_plugin = rocprof_plugin_path("aqlpmc")
        args.gpus = 1
    elif args.backend == "mock":  # simulated telemetry that changes every tick (the fake node's is static)
        import test_fakehost as tf
        c.backend = "mock"
        c.mock_devices = args.gpus
    else:
        import test_fakehost as tf
        root = tempfile.mkdtemp(prefix="gpuexp-prof-")
        tf._loaded_node(root, args.gpus)
        c.backend = "sysfs"
        c.host_root = root
    c.interval_s = 0
    if args.tick_hz and not real:
        c.interval_s = 1.0 / args.tick_hz
        c.sampler_thread = False
        c.enable_counters = c.enable_sentinel = True
        c.fake_pmc_cost_us = tf.PMC_READ_CPU_US
        c.fake_sentinel_cost_us = tf.SENTINEL_RUN_CPU_US
    c.serve_http = args.gzip
    if args.gzip:
        h = c.http
        h.port = 0
        h.host = "127.0.0.1"
        c.http = h
    c.series_profile = "full"
    c.exposition = args.exposition
    if not real:
        c.fake_metrics_cost_us = tf.SMU_FETCH_CPU_US if args.tick_hz else 0
    e = native.Engine(c)
    e.start()
    scraper = None
    if args.gzip:  # a gzip scraper in another process keeps the sampler compressing every tick
        import project_cpu
        scraper = subprocess.Popen([sys.executable, "-c", project_cpu.SCRAPER, ROOT, str(e.http_port), "100", "gzip"])
        time.sleep(1.0)
    now = 1_000_000_000

    step = int(1e9 / args.tick_hz) if args.tick_hz else 10_000_000

    def tick():  # a real device ticks on the real clock (the sentinel's and counters' domain)
        nonlocal now
        now += step
        e.tick() if real else e.tick(now)

    for _ in range(200 if not real else 20):
        tick()
        if real:
            time.sleep(args.sleep_ms / 1e3)
    trace = os.path.join(tempfile.gettempdir(), "gpuexp_sigprof.txt")
    lib.sigprof_start(args.hz)
    t0 = time.process_time()
    for _ in range(args.ticks):
        tick()
        if args.sleep_ms:
            time.sleep(args.sleep_ms / 1e3)
    cpu = time.process_time() - t0
    n = lib.sigprof_stop(trace.encode())
    if scraper:
        scraper.kill()
        scraper.wait()
    e.stop()
    print(f"# {args.ticks} ticks, {args.gpus} GPUs: {cpu / args.ticks * 1e6:.1f} us CPU/tick, {n} samples")
    stacks = symbolize(trace)
    self_c, incl_c = collections.Counter(), collections.Counter()
    for fr in stacks:
        fr = fr[2:] if len(fr) > 2 else fr  # drop the handler + signal trampoline
        if not fr or any("tick_now" in f for f in fr) is False:
            continue  # asleep between ticks (wall-clock timer), or in Python around them
        self_c[fr[0]] += 1
        for f in set(fr):
            incl_c[f] += 1
    tot = max(1, sum(self_c.values()))
    print(f"# {tot} samples inside Engine::tick_now")
    print(f"{'self%':>6}  function")
    for f, k in self_c.most_common(args.top):
        print(f"{100 * k / tot:6.1f}  {f[:150]}")
    print(f"\n{'incl%':>6}  function")
    for f, k in incl_c.most_common(args.top):
        print(f"{100 * k / tot:6.1f}  {f[:150]}")
    if args.lines:
        print(f"\nleaf source lines in {args.lines}:")
        leaf_lines(trace, args.lines)
    return 0


if __name__ == "__main__":
    sys.exit(main())
