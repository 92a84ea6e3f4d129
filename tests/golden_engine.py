"""A deterministic mock 8-GPU node for the engine's golden exposition (test_engine_golden.py):
full profile, sentinel + counters, GPU processes in two pods (one on two GPUs), device owners,
KFD SMI events (no RCCL tracer), ticked on an injected clock.

Families whose values come from the host's clocks (stage durations, CPU seconds, wall time,
fetch-cost-driven caps) are masked: their sample lines keep name + labels, the value becomes
`X`.  Everything else is compared byte for byte."""
from __future__ import annotations

import re

MASKED = (
    "gpuexp_sample_stage_duration_seconds", "gpuexp_device_read_seconds_total", "gpuexp_sampler_cpu_seconds_total",
    "gpuexp_gpu_metrics_fetch_cpu_seconds_total", "gpuexp_startup_seconds", "gpuexp_last_sample_timestamp_seconds",
    "gpuexp_render_bytes", "gpuexp_gpu_metrics_min_interval_seconds", "gpuexp_build_info",
)
UID_A = "aaaaaaaa-0000-4000-8000-00000000000a"
UID_B = "bbbbbbbb-0000-4000-8000-00000000000b"
CID_A, CID_B = "a" * 64, "b" * 64


def cgroup(uid: str, cid: str) -> str:
    return ("/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod" + uid.replace("-", "_") +
            ".slice/cri-containerd-" + cid + ".scope")


def run(native, exposition: str, ticks: int = 6, render_every: int = 0) -> str:
    c = native.EngineConfig()
    c.render_every_ticks = render_every
    c.backend = "mock"
    c.mock_devices = 8
    c.interval_s = 0
    c.serve_http = False
    c.series_profile = "full"
    c.enable_sentinel = True
    c.enable_counters = True
    c.exposition = exposition
    c.version = "golden"
    e = native.Engine(c)
    e.start()
    try:
        e.set_pods([dict(uid=UID_A, namespace="ml", name="trainer-0", containers={CID_A: "main"}),
                    dict(uid=UID_B, namespace="ml", name="serve-1", containers={CID_B: "srv"})])
        for pid, uid, cid in ((4242, UID_A, CID_A), (4243, UID_A, CID_A), (5151, UID_B, CID_B)):
            e.set_pid_cgroup(pid, cgroup(uid, cid))
        e.mock_set_processes(0, [dict(pid=4242, vram_bytes=30.5e9, cu_occupancy=64, name="python3")])
        e.mock_set_processes(1, [dict(pid=4242, vram_bytes=12.25e9, cu_occupancy=32, name="python3"),
                                 dict(pid=4243, vram_bytes=1.0e9, cu_occupancy=8, name="worker")])
        e.mock_set_processes(5, [dict(pid=5151, vram_bytes=8.0e9, cu_occupancy=16, name="serve")])
        for t in range(1, ticks + 1):
            if t == 3:  # KFD SMI events: a VM fault + an eviction of 4242 (trainer-0) on GPU 1, a throttle on 0
                e.inject_kfd_events(1, b"1 1092:python3\n9 100 -4242 0 2\n")
                e.inject_kfd_events(0, b"2 0:1\n")
            e.tick(t * 100_000_000)
        return e.snapshot_text()
    finally:
        e.stop()


def mask(text: str) -> str:
    out = []
    for line in text.split("\n"):
        if line and not line.startswith("#"):
            name = re.match(r"[a-zA-Z_:][a-zA-Z0-9_:]*", line).group(0)
            base = re.sub(r"_(bucket|sum|count)$", "", name)
            if name in MASKED or base in MASKED:
                line = re.sub(r"(\}|^[a-zA-Z0-9_:]+)\s+\S+$", r"\1 X", line)
        out.append(line)
    return "\n".join(out)
