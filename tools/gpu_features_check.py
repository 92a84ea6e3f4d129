"""GPU-box checks that need a clean process (run as subprocesses by tests/test_gpu.py).

  counters : exporter engine with a device-counter plugin (PLUGIN=aqlpmc|rocprof) while a
             GEMM child keeps the GPU busy; prints the counter series, per-thread CPU and
             the plugin's raw readings as JSON.  Never imports torch (the rocprofiler plugin
             must register before HSA loads).
  rccl     : a torch.distributed (RCCL, world_size 1) child with the RCCL tracer injected
             via ROCP_TOOL_LIBRARIES; prints the per-op counters from its shm file.
"""
import ctypes
import json
import os
import socket
import struct
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counters(seconds: float) -> dict:
    child = subprocess.Popen([sys.executable, "-c",
                              f"import sys; sys.path.insert(0, {ROOT!r});"
                              "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                              # long enough to outlast a slow plugin start; stopped after the snapshot
                              f"print(gemm_burn(0, 8192, {seconds + 20}, 4), flush=True)"],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    time.sleep(2.0)  # let the child start its GEMM loop
    from kubernetes_gpu_exporter_amd._native import load
    from kubernetes_gpu_exporter_amd.utils import promtext
    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0.1
    c.serve_http = False
    c.enable_counters = True
    from kubernetes_gpu_exporter_amd._native import rocprof_plugin_path
    plugin = rocprof_plugin_path(os.environ.get("PLUGIN", "aqlpmc"))
    c.counters_plugin = plugin
    c.counters_window_ms = int(os.environ.get("WINDOW_MS", "20"))
    c.counters_interval_ms = int(os.environ.get("INTERVAL_MS", "500"))
    c.enable_sentinel = os.environ.get("SENTINEL", "1") == "1"
    c.enable_counters = os.environ.get("COUNTERS", "1") == "1"
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    from kubernetes_gpu_exporter_amd.utils.procstat import thread_cpu_seconds
    time.sleep(0.5)
    cpu0 = thread_cpu_seconds(os.getpid())
    time.sleep(seconds)
    cpu1 = thread_cpu_seconds(os.getpid())
    hot = sorted(((cpu1[k] - cpu0.get(k, 0.0)) / seconds * 100, k) for k in cpu1)[-6:]
    print("per-thread CPU% over the window:", [(round(p, 1), k) for p, k in hot], flush=True)
    tid = hot[-1][1].split(":")[-1]
    for _ in range(2):  # what is the hottest thread doing? (syscall nr 24 = sched_yield)
        try:
            sc = open(f"/proc/self/task/{tid}/syscall").read().split()[0]
            wc = open(f"/proc/self/task/{tid}/wchan").read()
            print(f"hot thread {tid}: syscall={sc} wchan={wc}", flush=True)
        except OSError as ex:
            print("hot thread probe failed", ex)
        time.sleep(0.05)
    text = e.snapshot_text()
    status = e.source_status()
    gemm_running = child.poll() is None  # the snapshot's window lies inside the GEMM's run

    dbg = ctypes.create_string_buffer(4096)
    try:
        ctypes.CDLL(plugin).gpuexp_rp_debug(0, dbg, 4096)
    except OSError:
        pass
    e.stop()
    fams = promtext.parse(text)
    out = {"status": status, "raw_counters": dbg.value.decode(), "hot_threads": [(round(p, 1), k) for p, k in hot],
           "gemm_running_at_snapshot": gemm_running}
    for name in ("amd_gpu_mfma_busy_percent", "amd_gpu_sq_busy_percent", "amd_gpu_gui_active_percent",
                 "amd_gpu_waves_per_second", "amd_gpu_lds_active_percent", "amd_gpu_lds_bank_conflict_percent",
                 "amd_gpu_hbm_read_bytes_per_second", "amd_gpu_hbm_write_bytes_per_second",
                 "amd_gpu_gfx_activity_percent", "amd_gpu_sentinel_sclk_hz"):
        v = promtext.samples(fams, name)
        out[name] = v[0][2] if v else None
    sc = promtext.samples(fams, "gpuexp_counters_device_scope")
    out["device_scope"] = sc[0][2] if sc else None
    per_gpu = 0
    for name, fam in fams.items():
        if name.startswith("amd_gpu_") and not name.startswith("amd_gpu_process_"):
            per_gpu += sum(1 for s in fam.samples if s[1].get("gpu") == "0")
    out["series_gpu0"] = per_gpu
    child.terminate()
    child.wait(timeout=60)
    return out


def rccl() -> dict:
    from kubernetes_gpu_exporter_amd._native import rccl_tracer_path
    d = tempfile.mkdtemp(prefix="gpuexp-rccl-")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, ROCP_TOOL_LIBRARIES=rccl_tracer_path(), GPUEXP_RCCL_DIR=d, GPUEXP_RCCL_KEEP="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    code = (
        "import torch, torch.distributed as dist\n"
        "dist.init_process_group('nccl', rank=0, world_size=1)\n"
        "torch.cuda.set_device(0)\n"
        "x = torch.ones(1 << 20, device='cuda', dtype=torch.bfloat16)\n"
        "for _ in range(20): dist.all_reduce(x)\n"
        "out = [torch.empty_like(x)]\n"
        "for _ in range(5): dist.all_gather(out, x)\n"
        "for _ in range(5): dist.reduce_scatter_tensor(torch.empty_like(x), x)\n"
        "for _ in range(5): dist.all_to_all_single(torch.empty_like(x), x)\n"
        "torch.cuda.synchronize(); dist.destroy_process_group(); print('child done', flush=True)\n")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    # per-strategy parity: tracer deltas vs the generators' TrafficStats, in a second child
    d2 = tempfile.mkdtemp(prefix="gpuexp-rccl-parity-")
    env2 = dict(env, GPUEXP_RCCL_DIR=d2, MASTER_PORT=str(port + 1 if port < 65535 else port - 1))
    r2 = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_parity_child.py")], env=env2,
                        capture_output=True, text=True, timeout=240)
    parity_line = [l for l in r2.stdout.splitlines() if l.startswith("PARITY ")]
    parity = json.loads(parity_line[-1][7:]) if parity_line else {"rc": r2.returncode, "stderr": r2.stderr[-1500:]}
    files = [f for f in os.listdir(d) if f.startswith("gpuexp-rccl-")]
    ops = {}
    comm = []
    names = ["allreduce", "allgather", "reducescatter", "alltoall", "alltoallv", "broadcast", "reduce", "send",
             "recv", "gather", "scatter"]
    for f in files:
        b = open(os.path.join(d, f), "rb").read()
        magic, ver, ns_pid, ino, rank, nranks = struct.unpack_from("<QIiQii", b, 0)
        comm.append({"rank": rank, "nranks": nranks})
        for i, nm in enumerate(names):
            calls, nbytes = struct.unpack_from("<QQ", b, 64 + 16 * i)
            if calls:
                ops[nm] = {"calls": calls, "bytes": nbytes}
    return {"rc": r.returncode, "files": files, "ops": ops, "communicator": comm, "parity": parity,
            "stdout": r.stdout[-500:], "stderr": r.stderr[-1500:]}


if __name__ == "__main__":
    mode = sys.argv[1]
    res = counters(float(sys.argv[2]) if len(sys.argv) > 2 else 3.0) if mode == "counters" else rccl()
    print("RESULT " + json.dumps(res), flush=True)
    sys.stdout.flush()
    os._exit(0)
