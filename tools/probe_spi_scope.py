#!/usr/bin/env python3
"""Scope and calibration of the SPI occupancy-limiter counters on one MI355X
(profiles/r04/spi_scope.txt; VERDICT r03 task 3).

The exporter engine runs in THIS process (aqlprofile counters, continuous, 10 Hz, sentinel
on the PMC queue).  The load runs in a CHILD process, so a counter that only counts this
process's VMID (the SQ wave counters do for an unprivileged client, profiles/r02/
pmc_scope.txt) sees nothing of it; the same kernels from this process are the control.
Per tick the derived values come straight from the plugin (gpuexp_rp_sample outputs 13-17:
dispatch stall %, LDS / wave-slot / VGPR limiter %) and the raw window deltas from its
debug line, whatever the engine's export gating.

Cases (each `--seconds` long, 4 generations of blocks queued):
  idle           no kernel
  lds_other      occupancy_hog kind lds   (1 wave + 64 KiB LDS per block) in the child
  waves_other    occupancy_hog kind waves (8 waves, no LDS per block)      in the child
  vgpr_other     occupancy_hog kind vgpr (1 wave of 400 registers per lane) in the child (--kinds)
  sgpr_other     occupancy_hog kind sgpr (1 wave of 108 SGPRs)             in the child (--kinds)
  lds_self       the lds kernel from this process (control: VMID-matched)
  waves_self     the waves kernel from this process
Usage: python tools/probe_spi_scope.py [--seconds 2.0] -> RESULT json
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r"""
import sys, time
sys.path.insert(0, {root!r})
import torch
from kubernetes_gpu_exporter_amd.ops.gemm import occupancy_hog
torch.zeros(1, device="cuda:0")
kind, seconds, stream_no = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
# HIP gives each new stream its own hardware queue, round robin over GPU_MAX_HW_QUEUES (4):
# stream k > 0 is the k-th created stream, 0 the null stream
streams = [torch.cuda.Stream() for _ in range(stream_no)]
s = streams[-1] if streams else torch.cuda.current_stream()
torch.cuda.synchronize()
print("ready", flush=True)
sys.stdin.readline()  # go
t = time.perf_counter()
with torch.cuda.stream(s):
    out = occupancy_hog(0, kind, seconds / 4, generations=4, stream=s.cuda_stream)
torch.cuda.synchronize()
print("done", round(time.perf_counter() - t, 3), flush=True)
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--hz", type=float, default=10.0)
    ap.add_argument("--streams", default="0", help="comma-separated stream numbers to run every case on "
                    "(0 = the null stream, k = the k-th new stream: a different hardware queue each)")
    ap.add_argument("--kinds", default="lds,waves")
    ap.add_argument("--no-self", action="store_true", help="only the other-process cases")
    ap.add_argument("--exported", action="store_true",
                    help="also record the engine's exported amd_gpu_occupancy_limiter_percent per case")
    args = ap.parse_args()

    import torch
    torch.zeros(1, device="cuda:0")
    from kubernetes_gpu_exporter_amd._native import load, rocprof_plugin_path
    from kubernetes_gpu_exporter_amd.ops.gemm import occupancy_hog

    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 1.0 / args.hz
    c.serve_http = False
    c.series_profile = "full"
    c.enable_counters = True
    c.enable_sentinel = True
    c.counters_plugin = rocprof_plugin_path("aqlpmc")
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    status = e.source_status()
    print("status:", status, flush=True)
    if "counters=unavailable" in status:
        print("RESULT " + json.dumps({"status": status}), flush=True)
        e.stop()
        return 0
    plugin = ctypes.CDLL(rocprof_plugin_path("aqlpmc"))
    plugin.gpuexp_rp_sample.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
    out = (ctypes.c_double * 32)()  # >= the plugin ABI's output count (counter_model.h kNumOut)
    buf = ctypes.create_string_buffer(8192)

    def window():
        plugin.gpuexp_rp_debug(0, buf, 8192)
        kv = dict(x.split("=", 1) for x in buf.value.decode().split(";") if "=" in x)
        raw = {k: kv.get(k) for k in ("SPI_RA_RES_STALL_CSN", "SPI_RA_LDS_CU_FULL_CSN", "SPI_RA_WAVE_SIMD_FULL_CSN",
                                      "SPI_RA_VGPR_SIMD_FULL_CSN", "SPI_RA_SGPR_SIMD_FULL_CSN", "GRBM_COUNT",
                                      "GRBM_GUI_ACTIVE", "SQ_WAVES")}
        ok = plugin.gpuexp_rp_sample(0, 0.0, out) == 0
        w = {"stall": out[13] if ok else None, "lds": out[14] if ok else None, "waves": out[15] if ok else None,
             "vgpr": out[16] if ok else None, "sgpr": out[17] if ok else None, "gui": out[2] if ok else None, "raw": raw,
             "window_s": float(kv.get("window_s", "nan"))}
        if args.exported:
            from kubernetes_gpu_exporter_amd.utils import promtext
            fams = promtext.parse(e.snapshot_text())
            w["exported"] = {lab["resource"]: v for _, lab, v in
                             promtext.samples(fams, "amd_gpu_occupancy_limiter_percent") if lab.get("gpu") == "0"}
            st = [v for _, lab, v in promtext.samples(fams, "amd_gpu_dispatch_stall_percent") if lab.get("gpu") == "0"]
            w["exported"]["stall"] = st[0] if st else None
        return w

    def record(seconds, skip=0.3):
        rows = []
        t_end = time.perf_counter() + seconds
        time.sleep(skip)
        last = None
        while time.perf_counter() < t_end:
            time.sleep(1.0 / args.hz)
            w = window()
            if w["raw"] != last:
                rows.append(w)
                last = w["raw"]
        return rows

    def summary(rows):
        def med(k):
            v = [r[k] for r in rows if r[k] is not None]
            return round(statistics.median(v), 2) if v else None
        def tot(k):  # sum over the recorded windows of a raw counter ("value/instances")
            v = [float(r["raw"][k].split("/")[0]) for r in rows if r["raw"].get(k)]
            return round(sum(v)) if v else None
        out = {"windows": len(rows), "sum_sq_waves": tot("SQ_WAVES"),
               "stall_median": med("stall"), "lds_median": med("lds"),
               "waves_median": med("waves"), "vgpr_median": med("vgpr"), "sgpr_median": med("sgpr"),
               "gui_median": med("gui"),
               "raw_example": rows[len(rows) // 2]["raw"] if rows else None}
        if args.exported and rows:
            ex = [r["exported"] for r in rows]
            out["exported_median"] = {k: (round(statistics.median([x[k] for x in ex if x.get(k) is not None]), 2)
                                          if any(x.get(k) is not None for x in ex) else None)
                                      for k in ("stall", "lds", "wave_slots", "vgpr", "sgpr")}
        return out

    res = {"status": status, "cases": {}}
    time.sleep(0.5)
    res["cases"]["idle"] = summary(record(1.5))
    print("idle", res["cases"]["idle"], flush=True)
    own_streams: list = []
    for sn in (int(x) for x in args.streams.split(",")):
        while len(own_streams) < sn:
            own_streams.append(torch.cuda.Stream())
        sfx = "" if sn == 0 else f"_s{sn}"
        for kind in args.kinds.split(","):
            p = subprocess.Popen([sys.executable, "-c", CHILD.format(root=ROOT), kind, str(args.seconds), str(sn)],
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
            assert p.stdout.readline().strip() == "ready"
            p.stdin.write("go\n")
            p.stdin.flush()
            rows = record(args.seconds * 0.9)
            done = p.stdout.readline().strip()
            p.wait(timeout=60)
            key = f"{kind}_other{sfx}"
            res["cases"][key] = dict(summary(rows), child=done)
            print(key, res["cases"][key], flush=True)
            time.sleep(0.5)
            if args.no_self:
                continue
            t = time.perf_counter()
            st = own_streams[sn - 1] if sn else torch.cuda.current_stream()
            occupancy_hog(0, kind, args.seconds / 4, generations=4, stream=st.cuda_stream)
            rows = record(args.seconds * 0.9)
            torch.cuda.synchronize()
            key = f"{kind}_self{sfx}"
            res["cases"][key] = dict(summary(rows), run_s=round(time.perf_counter() - t, 3))
            print(key, res["cases"][key], flush=True)
            time.sleep(0.5)
    e.stop()
    print("RESULT " + json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
