#!/usr/bin/env python3
"""Runs the exporter engine in its shipped default GPU configuration (amdsmi backend, raw
gpu_metrics path, aqlprofile PMC counters in continuous mode, sentinel dispatched as raw AQL
on the counters' queue, full profile) at `hz` for `seconds`, then stops it and exits
normally, so a profiler wrapping this process can flush:
  rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o exporter -- python3 tools/exporter_profile.py 10 5
(a third argument `nocounters` runs the same without the PMC plugin: the HIP sentinel then)
Torch-free: the sentinel's and the PMC programs' queue is the only GPU queue the exporter
creates.  Prints the engine's source status and how many sentinel runs completed, so the
profile's dispatch count can be checked against it.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    hz = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    from kubernetes_gpu_exporter_amd._native import load, rocprof_plugin_path
    from kubernetes_gpu_exporter_amd.utils import promtext
    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 1.0 / hz
    c.serve_http = False
    c.series_profile = "full"
    c.enable_sentinel = True
    c.enable_counters = "nocounters" not in sys.argv[3:]
    c.counters_plugin = rocprof_plugin_path("aqlpmc")
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    print("status:", e.source_status(), flush=True)
    time.sleep(secs)
    fams = promtext.parse(e.snapshot_text())
    st = e.stats()
    import ctypes
    dbg = ctypes.create_string_buffer(4096)
    if c.enable_counters:
        ctypes.CDLL(rocprof_plugin_path("aqlpmc")).gpuexp_rp_debug(0, dbg, 4096)
    print("plugin:", ";".join(x for x in dbg.value.decode().split(";") if x.startswith(("round", "rounds", "mode",
                                                                                         "stalls", "window"))))
    cpu = [v for _, _, v in promtext.samples(fams, "gpuexp_sampler_cpu_seconds_total")]
    print(f"sampler CPU per tick {cpu[0] / st['ticks'] * 1e6:.0f} us" if cpu and st["ticks"] else "", flush=True)
    e.stop()
    runs = sum(v for _, _, v in promtext.samples(fams, "amd_gpu_sentinel_runs_total"))
    late = [v for _, _, v in promtext.samples(fams, "gpuexp_counters_late_ticks_total")]
    print(f"ticks {st['ticks']}, sentinel runs completed {runs:.0f}, counter reads late {late}, "
          f"counters stage mean {st['stage_ns']['counters'] / 1e3:.1f} us (last tick)", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
