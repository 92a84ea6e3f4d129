#!/usr/bin/env python3
"""MFMA-busy ground truth on one MI355X (tests/test_gpu.py::test_mfma_busy_calibration).

The exporter engine samples at 10 Hz with the aqlprofile counters in `counters_mode`
(default continuous) while this process runs the MFMA duty-cycle kernel
(ops.gemm.mfma_duty: 2 waves per SIMD alternating back-to-back v_mfma_f32_32x32x16_bf16
with s_sleep on the 100 MHz s_memrealtime clock) at known duties, on torch's HIP queue.
SQ_VALU_MFMA_BUSY_CYCLES and the GRBM clocks are chip-global for any client
(profiles/r02/pmc_scope.txt), so no special queue is needed.

Cases:
  resident d : the kernel stays resident the whole run, matrix cores busy d of the time:
               amd_gpu_mfma_busy_percent (over elapsed cycles) and amd_gpu_mfma_util_percent
               (over GUI-active cycles) should both read ~100 d.
  gated d    : the host runs 100 % MFMA kernels for d of every 20 ms and leaves the GPU idle
               in between: busy ~100 d, GUI active ~100 d, util ~100.
  idle       : no kernel at all: busy ~0.
  xcc x      : (--xcc-cases) the resident kernel at --xcc-duty on XCC x only (its other
               blocks exit at once): amd_gpu_xcc_mfma_busy_percent{xcc=x} ~100 d, the other
               XCCs ~0, the chip value ~100 d / 8 = the mean of the XCCs.
Every tick of a case is recorded, so "changes every tick" is checked too.
Usage: python tools/mfma_calibration.py [--mode continuous|duty] [--hz 10] [--xcc-cases 0,5]
  -> RESULT json
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="continuous")
    ap.add_argument("--hz", type=float, default=10.0)
    ap.add_argument("--seconds", type=float, default=2.6, help="kernel run per resident case")
    ap.add_argument("--duties", default="0,0.25,0.5,0.75,1")
    ap.add_argument("--no-sentinel", action="store_true")
    ap.add_argument("--xcc-cases", default="", help="comma-separated XCCs to run the XCC-targeted case on")
    ap.add_argument("--xcc-duty", type=float, default=0.9)
    ap.add_argument("--no-gated", action="store_true")
    ap.add_argument("--sentinel-impl", default="auto", help="auto (on the PMC queue) | hip (its own HIP stream)")
    ap.add_argument("--starve", type=float, default=0.0,
                    help="seconds of a 100 %% MFMA kernel that leaves the sentinel no slot (pending gauge case)")
    args = ap.parse_args()

    import torch  # one HIP runtime per process: torch's, loaded before the exporter's plugins
    torch.zeros(1, device="cuda:0")
    from kubernetes_gpu_exporter_amd._native import load, rocprof_plugin_path
    from kubernetes_gpu_exporter_amd.ops.gemm import mfma_duty
    from kubernetes_gpu_exporter_amd.utils import promtext

    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 1.0 / args.hz
    c.serve_http = False
    c.series_profile = "full"
    c.enable_counters = True
    c.enable_sentinel = not args.no_sentinel
    c.sentinel_impl = args.sentinel_impl
    c.counters_plugin = rocprof_plugin_path("aqlpmc")
    c.counters_mode = args.mode
    c.counters_window_ms = 20
    c.counters_interval_ms = int(1000 / args.hz) if args.mode == "duty" else 1000
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    status = e.source_status()
    print("status:", status, flush=True)
    if "counters=unavailable" in status:
        print("RESULT " + json.dumps({"status": status}), flush=True)
        e.stop()
        return 0
    simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    import ctypes
    plugin = ctypes.CDLL(rocprof_plugin_path("aqlpmc"))

    def raw():
        """The plugin's last window: raw per-counter deltas (reduced) + window length."""
        buf = ctypes.create_string_buffer(8192)
        plugin.gpuexp_rp_debug(0, buf, 8192)
        return buf.value.decode()

    def val(fams, name, **kw):
        try:
            return promtext.value(fams, name, **kw)
        except KeyError:
            return None

    def ticks_during(seconds, skip=0.5, work=None):
        """Per-tick (mfma busy, util, gui, sclk) exported while `work` runs (or sleeping)."""
        rows, last = [], None
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            if work is not None:
                work()
            else:
                time.sleep(0.01)
            fams = promtext.parse(e.snapshot_text())
            tk = val(fams, "gpuexp_ticks_total")
            if tk == last or time.perf_counter() - t0 < skip:
                last = tk
                continue
            last = tk
            row = {k: val(fams, f, gpu=0) for k, f in (
                ("busy", "amd_gpu_mfma_busy_percent"), ("util", "amd_gpu_mfma_util_percent"),
                ("gui", "amd_gpu_gui_active_percent"), ("clk", "amd_gpu_sentinel_sclk_hz"))}
            row["xcc"] = {int(lab["xcc"]): v for _, lab, v in promtext.samples(fams, "amd_gpu_xcc_mfma_busy_percent")
                          if lab.get("gpu") == "0"}
            rows.append(row)
        return rows

    def summary(rows, expect_busy, expect_util=None, extra=None):
        def med(k):
            v = [r[k] for r in rows if r[k] is not None]
            return statistics.median(v) if v else None
        busy = [r["busy"] for r in rows if r["busy"] is not None]
        changed = sum(1 for a, b in zip(busy, busy[1:]) if a != b)
        out = {"ticks": len(rows), "busy_median": med("busy"), "busy_min": min(busy) if busy else None,
               "busy_max": max(busy) if busy else None, "util_median": med("util"), "gui_median": med("gui"),
               "sclk_median": med("clk"), "expected_busy": expect_busy, "expected_util": expect_util,
               "changed_fraction": changed / max(1, len(busy) - 1), "per_tick_busy": [round(x, 2) for x in busy]}
        if extra:
            out.update(extra)
        return out

    res = {"status": status, "mode": args.mode, "hz": args.hz, "simds": simds, "cases": {}}
    time.sleep(1.0)
    idle_rows = ticks_during(1.5)
    res["cases"]["idle"] = summary(idle_rows, 0.0, None, {"raw_window": raw()})
    print("idle", res["cases"]["idle"]["busy_median"], flush=True)
    for d in [float(x) for x in args.duties.split(",") if x.strip()]:
        def cum_mfma():
            kv = dict(x.split("=", 1) for x in raw().split(";") if "=" in x)
            return float(kv["cum_MFMA"]) if "cum_MFMA" in kv else None
        time.sleep(0.25)  # idle: the next reads carry nothing but this kernel
        cum0 = cum_mfma()
        t_launch = time.perf_counter()
        out, counts = mfma_duty(0, d, args.seconds, period_s=0.002)
        rows = ticks_during(args.seconds - 0.35, skip=0.45)
        raw_window = raw()
        torch.cuda.synchronize()
        run_s = time.perf_counter() - t_launch
        mf = int(counts.sum().item())
        time.sleep(0.35)  # let a read after the kernel's end land
        cum1 = cum_mfma()
        # SQ_VALU_MFMA_BUSY_CYCLES over the kernel's life vs 32 cycles per issued
        # v_mfma_f32_32x32x16_bf16 (MI355X_MICROARCH.md cycle constants): exact ground truth
        cycles_ratio = (cum1 - cum0) / (32.0 * mf) if cum0 is not None and cum1 is not None and mf else None
        clk = statistics.median([r["clk"] for r in rows if r["clk"]] or [0])
        # MFMA cycles issued (32 per v_mfma_f32_32x32x16_bf16, microarch guide) over the
        # kernel's SIMD-cycles at the measured shader clock: what the counters should see
        from_count = 100.0 * mf * 32 / (args.seconds * clk * simds) if clk else None
        key = f"resident_{d:g}"
        res["cases"][key] = summary(rows, 100.0 * d, 100.0 * d,
                                    {"mfma_issued": mf, "busy_from_mfma_count": from_count, "run_s": run_s,
                                     "mfma_busy_cycles_over_32x_issued": cycles_ratio,
                                     "raw_window": raw_window})
        print(key, res["cases"][key]["busy_median"], res["cases"][key]["util_median"], "from count", from_count,
              "busy cycles / (32 x MFMAs issued)", cycles_ratio, flush=True)
    def xcc_medians(rows):
        xs = sorted({x for r in rows for x in r["xcc"]})
        return {str(x): statistics.median([r["xcc"][x] for r in rows if x in r["xcc"]]) for x in xs}

    res["cases"]["idle"]["xcc_median"] = xcc_medians(idle_rows)
    for x in [int(v) for v in args.xcc_cases.split(",") if v.strip()]:
        time.sleep(0.25)
        t_launch = time.perf_counter()
        out, counts = mfma_duty(0, args.xcc_duty, args.seconds, period_s=0.002, xcc_mask=1 << x)
        rows = ticks_during(args.seconds - 0.35, skip=0.45)
        raw_window = raw()
        torch.cuda.synchronize()
        run_s = time.perf_counter() - t_launch
        c = counts.cpu()
        key = f"xcc_{x}"
        res["cases"][key] = summary(rows, 100.0 * args.xcc_duty / 8, None, {
            "xcc": x, "xcc_duty": args.xcc_duty, "xcc_median": xcc_medians(rows), "run_s": run_s,
            "waves_that_ran": int((c > 0).sum().item()), "waves": int(c.numel()), "mfma_issued": int(c.sum().item()),
            "raw_window": raw_window})
        print(key, "chip", res["cases"][key]["busy_median"], "per-XCC", res["cases"][key]["xcc_median"],
              "waves ran", res["cases"][key]["waves_that_ran"], "/", res["cases"][key]["waves"], flush=True)
    # gated: kernel at 100 % for on_ms of every 20 ms, idle in between
    for on_ms in (() if args.no_gated else (10.0, 5.0)):
        period = 0.020

        def step(on=on_ms / 1000.0):
            t = time.perf_counter()
            mfma_duty(0, 1.0, on, period_s=0.001)
            torch.cuda.synchronize()
            rest = period - (time.perf_counter() - t)
            if rest > 0:
                time.sleep(rest)

        d = on_ms / 20.0
        key = f"gated_{d:g}"
        res["cases"][key] = summary(ticks_during(2.5, skip=0.5, work=step), 100.0 * d, 100.0,
                                    {"raw_window": raw()})
        print(key, res["cases"][key]["busy_median"], res["cases"][key]["util_median"], res["cases"][key]["gui_median"],
              flush=True)
    if args.starve > 0:
        # 8 blocks of 4 waves per CU = every wave slot of every SIMD, each wave issuing MFMAs
        # back to back for `starve` s (the grid's later blocks wait for the first ones): the
        # one-wave sentinel run cannot start, so amd_gpu_sentinel_pending_seconds must grow,
        # and drop to 0 once the kernel is gone
        def pend(with_busy=False):
            fams = promtext.parse(e.snapshot_text())
            p = val(fams, "amd_gpu_sentinel_pending_seconds", gpu=0)
            if with_busy:
                ticks.append(val(fams, "gpuexp_ticks_total"))
                return p, val(fams, "amd_gpu_mfma_busy_percent", gpu=0)
            return p
        ticks = []

        def rss_mib():  # this process holds the engine, so its queues' pinned areas
            with open("/proc/self/status") as fh:
                return int([l for l in fh if l.startswith("VmRSS:")][0].split()[1]) / 1024.0
        rss = {"before": rss_mib()}
        time.sleep(0.3)
        before = pend()
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        ev = torch.cuda.Event()
        t0 = time.perf_counter()
        mfma_duty(0, 1.0, args.starve, period_s=0.002, blocks=8 * cus)
        ev.record()
        seen, busy = [], []
        rss_during = []
        while not ev.query() and time.perf_counter() - t0 < 4 * args.starve + 5:
            time.sleep(0.1)
            p, b = pend(True)
            seen.append(p)
            busy.append(b)
            rss_during.append(rss_mib())
        torch.cuda.synchronize()
        run_s = time.perf_counter() - t0
        time.sleep(0.5)
        # the rescue queue is released once reads complete on the first queue again
        # (kProbationRounds ticks after the abandoned read ran): wait for that, bounded
        t_rel = time.perf_counter()
        while time.perf_counter() - t_rel < 5.0:
            kv = dict(x.split("=", 1) for x in raw().split(";") if "=" in x)
            if kv.get("rescue_active") == "0" and kv.get("rescues") == kv.get("rescue_releases"):
                break
            time.sleep(0.1)
        released_after_s = round(time.perf_counter() - t_rel + 0.5, 2)
        time.sleep(0.3)
        rss["during_max"] = max(rss_during) if rss_during else None
        rss["after"] = rss_mib()
        kv = dict(x.split("=", 1) for x in raw().split(";") if "=" in x)
        fams_after = promtext.parse(e.snapshot_text())
        events = {lab["event"]: v for _, lab, v in promtext.samples(fams_after, "gpuexp_counters_events_total")
                  if lab.get("gpu") == "0"}
        active = [v for _, lab, v in promtext.samples(fams_after, "gpuexp_counters_rescue_active") if lab.get("gpu") == "0"]
        res["cases"]["starve"] = {"seconds": args.starve, "kernel_s": run_s, "pending_before": before,
                                  "pmc_read_stalls": int(kv.get("stalls", -1)), "rescued": kv.get("rescued"),
                                  "rescue_active_after": kv.get("rescue_active"), "rescues": kv.get("rescues"),
                                  "rescue_releases": kv.get("rescue_releases"),
                                  "released_after_kernel_s": released_after_s,
                                  "rss_mib": {k: round(v, 1) if v is not None else None for k, v in rss.items()},
                                  "counters_events": events, "rescue_active_metric": active[0] if active else None,
                                  "busy_during": [round(v, 2) if v is not None else None for v in busy],
                                  "ticks_during": ticks,
                                  "pending_during": [round(v, 3) if v is not None else None for v in seen],
                                  "pending_max": max([v for v in seen if v is not None] or [0]),
                                  "pending_after": pend()}
        print("starve", res["cases"]["starve"], flush=True)
    res["raw_counters"] = raw()
    res["stage_counters_ms_last"] = e.stats()["stage_ns"]["counters"] / 1e6
    e.stop()
    print("RESULT " + json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
