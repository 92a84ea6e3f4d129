#!/usr/bin/env python3
"""Per-process cost of GPU process discovery and pod attribution on real KFD sysfs: K child
processes hold VRAM on the GPU (no compute), each attributed to its own fake pod through a
cgroup override; the engine (amdsmi raw path, 10 Hz, full profile, no PMC / sentinel) runs
for a few seconds per K and reports the processes / attribution / series stage CPU per tick
and what it exported.  K <= 12 (the box allows 16 GPU processes per run).
profiles/r04/many_procs.txt.

Usage: python tools/probe_many_procs.py [--counts 1,4,8,12] [--seconds 3]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r"""
import sys, time
sys.path.insert(0, {root!r})
import torch
from kubernetes_gpu_exporter_amd.utils.kfdself import find_own_kfd_pid
salt = int(sys.argv[1])
hostpid = find_own_kfd_pid(0, salt=salt)
keep = torch.empty((64 + salt) << 20, dtype=torch.uint8, device="cuda:0")
keep.fill_(1)
torch.cuda.synchronize()
print("ready", hostpid, flush=True)
sys.stdin.readline()
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", default="1,4,8,12")
    ap.add_argument("--seconds", type=float, default=3.0)
    args = ap.parse_args()
    counts = [min(12, int(x)) for x in args.counts.split(",")]
    from kubernetes_gpu_exporter_amd._native import load
    from kubernetes_gpu_exporter_amd.utils import promtext
    n = load()
    kids, pids = [], []
    rows = []
    try:
        for k in counts:
            while len(kids) < k:  # add children up to k
                i = len(kids)
                p = subprocess.Popen([sys.executable, "-c", CHILD.format(root=ROOT), str(i)], stdin=subprocess.PIPE,
                                     stdout=subprocess.PIPE, text=True)
                line = p.stdout.readline().split()
                assert line and line[0] == "ready", line
                kids.append(p)
                pids.append(int(line[1]) if line[1] != "None" else p.pid)
            c = n.EngineConfig()
            c.backend = "amdsmi"
            c.interval_s = 0.1
            c.serve_http = False
            c.series_profile = "full"
            c.enable_counters = False
            c.enable_sentinel = False
            c.device_filter = [0]
            e = n.Engine(c)
            e.start()
            pods = []
            for i, hp in enumerate(pids):
                uid = f"00000000-0000-4000-8000-{i:012d}"
                cid = f"{i:064x}"
                pods.append({"uid": uid, "namespace": "probe", "name": f"pod-{i}", "containers": {cid: "main"}})
                e.set_pid_cgroup(hp, f"/kubepods.slice/kubepods-pod{uid.replace('-', '_')}.slice/"
                                     f"cri-containerd-{cid}.scope")
            e.set_pods(pods, True)
            time.sleep(1.0)
            s0 = e.stats()
            time.sleep(args.seconds)
            s1 = e.stats()
            fams = promtext.parse(e.snapshot_text())
            e.stop()
            ticks = s1["ticks"] - s0["ticks"]
            st = {k2: round((s1["stage_cpu_ns"][k2] - s0["stage_cpu_ns"][k2]) / max(1, ticks) / 1e3, 1)
                  for k2 in ("processes", "attribution", "series", "render")}
            attributed = {lab["pod"] for _, lab, _ in promtext.samples(fams, "pod_gpu_memory_usage")}
            procs = {lab["pid"] for _, lab, _ in promtext.samples(fams, "amd_gpu_process_vram_bytes")}
            row = {"children": k, "ticks": ticks, "stage_cpu_us_per_tick": st,
                   "sampler_cpu_us_per_tick": round((s1["sampler_cpu_ns"] - s0["sampler_cpu_ns"]) / max(1, ticks) / 1e3, 1),
                   "gpu_processes_exported": len(procs), "pods_attributed": len(attributed)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    finally:
        for p in kids:
            try:
                p.stdin.write("\n")
                p.stdin.flush()
            except OSError:
                pass
        for p in kids:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    print("RESULT " + json.dumps(rows), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
