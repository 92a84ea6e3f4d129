#!/usr/bin/env python3
"""Runs the amdsmi engine with the HIP sentinel at `hz` for `seconds`, stops it and exits
normally (no os._exit) so a profiler wrapping this process can flush — e.g.
  rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sent -o sent -- \\
      python3 tools/sentinel_profile.py 100 3
Torch-free: the only HIP runtime in the process is the sentinel's.

With a third argument `gemm` (a saturating bf16 MFMA GEMM) or `copy` (HBM-bound device
copies), a child process loads the GPU meanwhile, and the sentinel's per-XCD dispatch
latencies and HBM load latency are summarised idle (first second, before the child
starts) vs loaded — the contention probes the sentinel exists for.
"""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_xcd(samples: list) -> dict:
    out = {}
    for snap in samples:
        for x, v in snap.items():
            out.setdefault(x, []).append(v)
    return {x: {"p50_us": round(statistics.median(v) * 1e6, 2), "max_us": round(max(v) * 1e6, 2), "n": len(v)}
            for x, v in sorted(out.items())}


def main() -> int:
    hz = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    mode = sys.argv[3] if len(sys.argv) > 3 else ""
    load = mode in ("gemm", "copy")
    from kubernetes_gpu_exporter_amd._native import load as load_native
    from kubernetes_gpu_exporter_amd.utils import promtext
    n = load_native()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 1.0 / hz
    c.serve_http = False
    c.enable_sentinel = True
    c.series_profile = "full"
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    phases = {"idle": [], "load": []}
    first = {"idle": [], "load": []}
    hbm = {"idle": [], "load": []}
    child = None
    t0 = time.time()
    last_runs = -1
    while time.time() - t0 < secs:
        phase = "load" if child is not None else "idle"
        if load and child is None and time.time() - t0 > 1.0:
            dur = max(1.0, secs - 1.5)
            code = ("import sys; sys.path.insert(0, %r);"
                    "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                    "print(gemm_burn(0, 8192, %f, 4), flush=True)" % (ROOT, dur)) if mode == "gemm" else (
                "import time, torch; x = torch.empty(1 << 31, dtype=torch.uint8, device='cuda');"
                "y = torch.empty_like(x); n = 0; t = time.time()\n"
                "while time.time() - t < %f:\n"
                "    for _ in range(20): y.copy_(x)\n"
                "    torch.cuda.synchronize(); n += 20\n"
                "print({'copy_TBps': 2 * n * x.numel() / (time.time() - t) / 1e12}, flush=True)" % dur)
            child = subprocess.Popen([sys.executable, "-c", code],
                                     stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
            time.sleep(0.5)  # let the GEMM ramp up before sampling the loaded phase
            continue
        fams = promtext.parse(e.snapshot_text())
        runs = promtext.samples(fams, "amd_gpu_sentinel_runs_total")
        r = runs[0][2] if runs else -1
        if r != last_runs:  # one sample per completed run
            last_runs = r
            lat = {lab["xcc"]: v for _, lab, v in
                   promtext.samples(fams, "amd_gpu_sentinel_xcc_dispatch_latency_seconds")}
            if lat:
                phases[phase].append(lat)
            f = promtext.samples(fams, "amd_gpu_sentinel_dispatch_latency_seconds")
            if f:
                first[phase].append(f[0][2])
            hb = promtext.samples(fams, "amd_gpu_sentinel_memory_latency_seconds")
            if hb:
                hbm[phase].append(hb[0][2])
        time.sleep(1.0 / hz)
    fams = promtext.parse(e.snapshot_text())
    out = {"status": e.source_status(), "ticks": e.stats()["ticks"]}
    for name in ("amd_gpu_sentinel_runs_total", "amd_gpu_sentinel_sclk_hz", "amd_gpu_sentinel_dispatch_latency_seconds"):
        v = promtext.samples(fams, name)
        out[name] = v[0][2] if v else None
    out["xcc_clock_hz"] = {lab["xcc"]: v for _, lab, v in promtext.samples(fams, "amd_gpu_xcc_clock_hz")}
    e.stop()
    out["mode"] = mode or "idle"
    for ph in ("idle", "load"):
        if first[ph]:
            out[f"{ph}_first_wave_p50_us"] = round(statistics.median(first[ph]) * 1e6, 2)
            out[f"{ph}_per_xcd"] = per_xcd(phases[ph])
        if hbm[ph]:
            out[f"{ph}_memory_latency_p50_ns"] = round(statistics.median(hbm[ph]) * 1e9, 1)
            out[f"{ph}_memory_latency_max_ns"] = round(max(hbm[ph]) * 1e9, 1)
    if child is not None:
        o, _ = child.communicate(timeout=120)
        out["load_child"] = o.strip()[-300:]
    print("RESULT " + json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
