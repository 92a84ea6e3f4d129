#!/usr/bin/env python3
"""GPU-box probe: cost of each KFD per-process sysfs read while a GEMM child runs.
Times (wall and thread CPU, p50 over N reps) of: listing /sys/class/kfd/kfd/proc, and
reading vram_<gpu_id>, stats_<gpu_id>/cu_occupancy and sdma_<gpu_id> for every process.
Decides which reads the sampler may do every tick and which at a lower rate.
Usage: python tools/probe_kfd_cost.py [reps]
"""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KFD = "/sys/class/kfd/kfd/proc"


def timed(fn, reps):
    w, c = [], []
    for _ in range(reps):
        c0, w0 = time.thread_time_ns(), time.perf_counter_ns()
        fn()
        w.append((time.perf_counter_ns() - w0) / 1e3)
        c.append((time.thread_time_ns() - c0) / 1e3)
    return {"wall_us_p50": round(statistics.median(w), 2), "cpu_us_p50": round(statistics.median(c), 2)}


def read(path):
    try:
        with open(path, "rb", buffering=0) as fh:
            return fh.read()
    except OSError:
        return b""


def main() -> int:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    child = subprocess.Popen([sys.executable, "-c",
                              f"import sys; sys.path.insert(0, {ROOT!r});"
                              "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                              "print(gemm_burn(0, 8192, 12.0, 4), flush=True)"],
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    time.sleep(3.0)
    out = {"list": timed(lambda: os.listdir(KFD), reps)}
    pids = os.listdir(KFD)
    out["pids"] = len(pids)
    for pid in pids[:4]:
        files = sorted(os.listdir(f"{KFD}/{pid}"))
        ent = {"files": files}
        for f in files:
            p = f"{KFD}/{pid}/{f}"
            if f.startswith("vram_") or f.startswith("sdma_"):
                ent[f] = timed(lambda p=p: read(p), reps)
            elif f.startswith("stats_"):
                for sub in sorted(os.listdir(p)):
                    ent[f"{f}/{sub}"] = timed(lambda q=f"{p}/{sub}": read(q), reps)
                    ent[f"{f}/{sub}:value"] = read(f"{p}/{sub}").decode(errors="replace").strip()
        out[pid] = ent
    # DRM fdinfo of the GEMM child's render-node fds: does KFD compute show up in
    # drm-engine-* (it does not go through the DRM scheduler)?
    fdi = {}
    try:
        for fd in os.listdir(f"/proc/{child.pid}/fd"):
            try:
                tgt = os.readlink(f"/proc/{child.pid}/fd/{fd}")
            except OSError:
                continue
            if tgt.startswith("/dev/dri/") or tgt == "/dev/kfd":
                fdi[f"{fd}->{tgt}"] = read(f"/proc/{child.pid}/fdinfo/{fd}").decode(errors="replace")
    except OSError as ex:
        fdi["error"] = str(ex)
    out["gemm_child_fdinfo"] = fdi
    child.kill()
    child.wait()
    print("RESULT " + json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
