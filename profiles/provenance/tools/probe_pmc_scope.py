"""Probe: which waves do the agent-mode (aqlprofile) SQ/TCC counters see for an
unprivileged process?  Runs the engine with counters + the sentinel (queue | hip) at 10 Hz
and prints the plugin's raw per-window counters: idle, then while this process streams
copies on torch's queue.  usage: probe_pmc_scope.py queue|hip"""
import ctypes
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    impl = sys.argv[1] if len(sys.argv) > 1 else "queue"
    import torch
    torch.zeros(1, device="cuda:0")
    from kubernetes_gpu_exporter_amd._native import load, rocprof_plugin_path
    from kubernetes_gpu_exporter_amd.ops.gemm import stream_copy
    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0.1
    c.serve_http = False
    c.enable_counters = True
    plugin = rocprof_plugin_path("aqlpmc")
    c.counters_plugin = plugin
    c.counters_window_ms = 100
    c.counters_interval_ms = 100
    c.enable_sentinel = True
    c.sentinel_impl = impl
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    print("status:", e.source_status(), flush=True)
    lib = ctypes.CDLL(plugin)
    dbg = ctypes.create_string_buffer(4096)

    def show(tag):
        lib.gpuexp_rp_debug(0, dbg, 4096)
        print(tag, dbg.value.decode(), flush=True)

    time.sleep(1.0)
    show("idle+sentinel:")
    src = torch.ones(1 << 28, device="cuda:0")
    dst = torch.empty_like(src)
    stop = threading.Event()

    def loop():
        while not stop.is_set():
            stream_copy(src, dst)

    th = threading.Thread(target=loop)
    th.start()
    time.sleep(1.0)
    show("copy+sentinel:")
    stop.set()
    th.join()
    torch.cuda.synchronize()
    e.stop()


if __name__ == "__main__":
    main()
    sys.stdout.flush()
    os._exit(0)
