"""Synthetic GPU pod workloads — the "models" the exporter is benchmarked and tested under.

The exporter observes workloads; it runs none.  BASELINE.json's configs are defined by
what runs in the pods ("8 synthetic HIP-GEMM pods", "DP/TP/PP/SP/EP collectives visible
per pod"), so each workload class here reproduces one pod type's GPU signature:

  GemmPod       bf16 MFMA GEMM bursts (our gfx950 kernel, csrc/kernels/gemm_bf16.hip)
                -> gfx/MFMA busy, power, HBM traffic, VRAM held by one process
  TrainerPod    a GemmPod's compute + one parallelism strategy's collectives per step
                (parallel/collectives.py: dp tp pp sp ep cp ulysses) -> xGMI per-link
                traffic + RCCL per-op calls/bytes attributable to the pod

Every workload has the same interface: step() runs one step and returns its stats;
`run()` does warmup + timed steps.  On a host without a GPU the GEMM falls back to an
fp32 torch matmul of the same shape so the multi-process (gloo) tests exercise the same
code path; on a GPU box the HIP kernel is mandatory (ops.gemm fails loudly if missing).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

from ..parallel import collectives


@dataclass
class StepStats:
    seconds: float = 0.0
    flops: float = 0.0
    comm_bytes: dict = field(default_factory=dict)  # op -> bytes (RCCL tracer accounting)
    comm_calls: dict = field(default_factory=dict)


class GemmPod:
    """`iters` size^3 bf16 GEMMs per step on one device (HIP kernel on GPU)."""

    name = "gemm"

    def __init__(self, size: int = 8192, iters: int = 4, device=None):
        import torch
        self.size, self.iters = int(size), int(iters)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.gpu = self.device.type == "cuda"
        dt = torch.bfloat16 if self.gpu else torch.float32
        g = torch.Generator(device="cpu").manual_seed(1234)
        self.a = (torch.rand(self.size, self.size, generator=g) - 0.5).to(self.device, dt)
        self.b = (torch.rand(self.size, self.size, generator=g) - 0.5).to(self.device, dt)
        self.c = torch.empty(self.size, self.size, device=self.device, dtype=dt)
        if self.gpu:
            from ..ops.gemm import kernels
            self._k = kernels()
            self._stream = torch.cuda.current_stream(self.device).cuda_stream

    def compute(self) -> float:
        import torch
        for _ in range(self.iters):
            if self.gpu:
                self._k.gemm_bf16(self.a.data_ptr(), self.b.data_ptr(), self.c.data_ptr(), self.size, self.size,
                                  self.size, self._stream)
            else:
                torch.matmul(self.a, self.b.T, out=self.c)
        return 2.0 * self.size ** 3 * self.iters

    def sync(self) -> None:
        import torch
        if self.gpu:
            torch.cuda.synchronize(self.device)

    def step(self) -> StepStats:
        t0 = time.perf_counter()
        flops = self.compute()
        self.sync()
        return StepStats(seconds=time.perf_counter() - t0, flops=flops)


class TrainerPod(GemmPod):
    """GemmPod compute + `strategy`'s collectives (default process group) every step."""

    def __init__(self, strategy: str = "dp", size: int = 4096, iters: int = 2, comm_bytes: int = 16 << 20,
                 layers: int = 2, device=None):
        if strategy not in collectives.STRATEGIES:
            raise ValueError(f"unknown strategy {strategy}; choose from {collectives.STRATEGIES}")
        super().__init__(size, iters, device)
        self.name = strategy
        self.strategy, self.comm_bytes, self.layers = strategy, int(comm_bytes), int(layers)

    def step(self) -> StepStats:
        t0 = time.perf_counter()
        flops = self.compute()
        tr = collectives.run(self.strategy, 1, self.comm_bytes, device=self.device if self.gpu else None,
                             layers=self.layers)
        self.sync()
        return StepStats(seconds=time.perf_counter() - t0, flops=flops, comm_bytes=dict(tr.bytes),
                         comm_calls=dict(tr.calls))


WORKLOADS = ("gemm",) + collectives.STRATEGIES


def make(name: str, **kw):
    """Workload by name: "gemm" or a parallelism strategy (dp tp pp sp ep cp ulysses)."""
    if name == "gemm":
        return GemmPod(**{k: v for k, v in kw.items() if k in ("size", "iters", "device")})
    return TrainerPod(name, **kw)


def run(workload, steps: int, warmup: int = 1) -> dict:
    """Warmup + timed steps; returns totals per rank (TFLOP/s, per-op comm bytes/calls)."""
    for _ in range(warmup):
        workload.step()
    tot = StepStats()
    for _ in range(steps):
        s = workload.step()
        tot.seconds += s.seconds
        tot.flops += s.flops
        for op, b in s.comm_bytes.items():
            tot.comm_bytes[op] = tot.comm_bytes.get(op, 0) + b
        for op, c in s.comm_calls.items():
            tot.comm_calls[op] = tot.comm_calls.get(op, 0) + c
    return {"workload": workload.name, "steps": steps, "seconds": tot.seconds,
            "tflops": tot.flops / tot.seconds / 1e12 if tot.seconds else 0.0,
            "comm_bytes": tot.comm_bytes, "comm_calls": tot.comm_calls,
            "device": str(workload.device)}
