"""Calibrates the device-scope PMC families (counter_model.h derivations) against
workloads with known HBM bytes, LDS bank conflicts and wave counts, on one MI355X.

An unprivileged process's agent-mode SQ/TCC counters count only the dispatches of the
queue that programs them (profiles/r02/pmc_scope.txt), so the calibration workloads
(csrc/kernels/probe_device.h) are dispatched by the aqlprofile plugin on its own PMC queue
(gpuexp_rp_calibrate) while the exporter engine's counting windows run; with
GPUEXP_PMC_ASSUME_DEVICE_SCOPE=1 the device-scope families are exported and compared:

  copy      stream copy of 1 GiB per launch: HBM read = write = 1 GiB / t_launch,
            waves/s = 16384 / t_launch
  lds_clean ds_read_b32, 32 distinct banks per lane group: bank-conflict % ~ 0
  lds_32way the same reads, all 32 lanes of a group on one bank: 31 of 32 cycles extra
  mfma_bf16 / mfma_fp8  a fixed number of v_mfma_f32_32x32x16_{bf16,fp8_fp8} per wave:
            FLOP/s of that type = FLOPs per launch / t_launch, the other type ~ 0

Prints one line `RESULT {json}` (run by tests/test_gpu.py::test_device_scope_pmc_calibration).
Never imports torch: the plugin's HSA runtime is the only GPU runtime in the process.
"""
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FAMILIES = ("amd_gpu_hbm_read_bytes_per_second", "amd_gpu_hbm_write_bytes_per_second", "amd_gpu_waves_per_second",
            "amd_gpu_lds_active_percent", "amd_gpu_lds_bank_conflict_percent", "amd_gpu_gui_active_percent",
            "amd_gpu_sq_busy_percent", "amd_gpu_mfma_busy_percent", "amd_gpu_remote_read_bytes_per_second",
            "amd_gpu_remote_write_bytes_per_second", "amd_gpu_hbm_bandwidth_bytes_per_second",
            "amd_gpu_umc_activity_percent")
WORKLOADS = (("copy", 0), ("lds_clean", 1), ("lds_32way", 2), ("mfma_bf16", 3), ("mfma_fp8", 4))


def main() -> int:
    os.environ["GPUEXP_PMC_ASSUME_DEVICE_SCOPE"] = "1"
    from kubernetes_gpu_exporter_amd._native import load, rocprof_plugin_path
    from kubernetes_gpu_exporter_amd.utils import promtext
    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0
    c.serve_http = False
    c.series_profile = "full"
    c.enable_counters = True
    plugin = rocprof_plugin_path("aqlpmc")
    c.counters_plugin = plugin
    c.counters_window_ms = 100
    c.counters_interval_ms = 100
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    lib = ctypes.CDLL(plugin)  # the engine's already-loaded copy
    lib.gpuexp_rp_calibrate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    lib.gpuexp_rp_calibrate.restype = ctypes.c_int
    out = {"status": e.source_status()}
    try:
        for name, kind in WORKLOADS:
            probe = (ctypes.c_double * 3)()
            if lib.gpuexp_rp_calibrate(0, kind, 20, probe) != 0:
                out[name] = {"error": "calibration dispatch failed"}
                continue
            per_launch = probe[0] / 20
            # ~3 s of work: the last tick (at 1.5 s) must read a window inside the busy period
            # even when the 20-launch probe overestimated the per-launch time
            launches = max(20, int(3.0 / per_launch))
            res = (ctypes.c_double * 3)()
            rc = [None]
            th = threading.Thread(target=lambda: rc.__setitem__(0, lib.gpuexp_rp_calibrate(0, kind, launches, res)))
            t0 = time.monotonic()
            th.start()
            time.sleep(1.2)  # several complete counting windows inside the busy period
            e.tick()
            time.sleep(0.3)
            e.tick()
            busy_s = time.monotonic() - t0
            fams = promtext.parse(e.snapshot_text())
            th.join()
            got = {"launches": launches, "rc": rc[0], "seconds": res[0], "ticked_at_s": round(busy_s, 3),
                   "busy_at_tick": bool(res[0] > busy_s)}
            for fam in FAMILIES:
                v = promtext.samples(fams, fam)
                got[fam] = v[0][2] if v else None
            sc = promtext.samples(fams, "gpuexp_counters_device_scope")
            got["device_scope"] = sc[0][2] if sc else None
            t = res[0] / launches if res[0] else float("nan")
            got["per_launch_s"] = t
            got["expected_waves_per_second"] = res[1] / t
            if kind == 0:
                got["expected_Bps"] = res[2] / t
            if kind >= 3:
                got["expected_flops_per_second"] = res[2] / t
                for _, lab, v in promtext.samples(fams, "amd_gpu_mfma_flops_per_second"):
                    got["flops_" + lab["dtype"]] = v
            dbg = ctypes.create_string_buffer(4096)
            lib.gpuexp_rp_debug(0, dbg, 4096)
            got["raw"] = dbg.value.decode()
            out[name] = got
            time.sleep(0.3)
    finally:
        e.stop()
    print("RESULT " + json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    os._exit(rc)
