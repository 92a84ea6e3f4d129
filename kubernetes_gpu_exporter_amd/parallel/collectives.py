"""Synthetic collective-traffic generators, one per parallelism strategy.

The exporter never issues collectives; it OBSERVES them (xGMI per-link accumulators,
the RCCL tracer).  These generators produce each strategy's wire signature with
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X; "gloo" for CPU tests) and
return the per-rank payload the tracer must report, so tests and the bench can check
the exporter's per-pod numbers against ground truth:

  dp       all-reduce of a gradient bucket                       (every link, symmetric)
  tp       per layer: all-reduce (row-parallel) + all-gather      (small, frequent)
  pp       send to next stage / recv from previous                (asymmetric, neighbours)
  sp       all-gather + reduce-scatter on the sequence dimension
  ep       all-to-all of token blocks (MoE dispatch)              (every pair)
  cp       ring attention: KV blocks passed around a ring         (2 neighbour links)
  ulysses  2 x all-to-all per attention layer                     (every pair)
  bcast    parameter broadcast from rank 0 + metric reduce to rank 0 (rooted trees)

Bytes follow the RCCL tracer's accounting (csrc/gpuexp/rccl_tracer.cc header comment).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

STRATEGIES = ("dp", "tp", "pp", "sp", "ep", "cp", "ulysses", "bcast")


@dataclass
class TrafficStats:
    strategy: str
    world: int
    steps: int
    calls: dict = field(default_factory=dict)   # op -> calls per rank
    bytes: dict = field(default_factory=dict)   # op -> payload bytes per rank (tracer accounting)
    seconds: float = 0.0
    # peer rank -> payload bytes this rank sent it directly (point-to-point and all-to-all
    # patterns, whose peers the pattern fixes; a collective's per-peer split is RCCL's choice)
    peer_bytes: dict = field(default_factory=dict)

    def add(self, op: str, nbytes: int, n: int = 1) -> None:
        self.calls[op] = self.calls.get(op, 0) + n
        self.bytes[op] = self.bytes.get(op, 0) + nbytes * n

    def add_peer(self, peer: int, nbytes: int) -> None:
        self.peer_bytes[peer] = self.peer_bytes.get(peer, 0) + nbytes


def _elems(nbytes: int, world: int, esize: int) -> int:
    """Element count for a buffer of ~nbytes that splits evenly across `world` ranks."""
    n = max(world, nbytes // esize)
    return n - n % world


def run(strategy: str, steps: int = 1, nbytes: int = 1 << 20, device=None, dtype=None, layers: int = 2,
        check: bool = True) -> TrafficStats:
    """Runs `steps` steps of `strategy` on the default process group.  With check=True the
    collectives' results are verified (catches a broken transport, not just a slow one)."""
    import torch
    import torch.distributed as dist
    if strategy not in STRATEGIES:
        raise ValueError(f"unknown strategy {strategy}; choose from {STRATEGIES}")
    world, rank = dist.get_world_size(), dist.get_rank()
    dtype = dtype or (torch.bfloat16 if device is not None and torch.device(device).type == "cuda" else torch.float32)
    esize = torch.tensor([], dtype=dtype).element_size()
    n = _elems(nbytes, world, esize)
    st = TrafficStats(strategy, world, steps)
    t0 = time.perf_counter()

    def full(v):
        return torch.full((n,), float(v), device=device, dtype=dtype)

    for _ in range(steps):
        if strategy == "dp":
            g = full(rank + 1)
            dist.all_reduce(g)
            st.add("allreduce", n * esize)
            if check:
                assert float(g[0]) == world * (world + 1) / 2
        elif strategy == "tp":
            for _ in range(layers):
                x = full(1)
                dist.all_reduce(x)
                st.add("allreduce", n * esize)
                shard = full(rank)[: n // world].contiguous()
                out = torch.empty(n // world * world, device=device, dtype=dtype)
                dist.all_gather_into_tensor(out, shard)
                st.add("allgather", (n // world) * esize * world)
                if check:
                    assert float(x[0]) == world and float(out[(world - 1) * (n // world)]) == world - 1
        elif strategy == "sp":
            shard = full(rank)[: n // world].contiguous()
            out = torch.empty(n, device=device, dtype=dtype)
            dist.all_gather_into_tensor(out, shard)
            st.add("allgather", (n // world) * esize * world)
            red = torch.empty(n // world, device=device, dtype=dtype)
            dist.reduce_scatter_tensor(red, full(1))
            st.add("reducescatter", (n // world) * esize * world)
            if check:
                assert float(red[0]) == world
        elif strategy in ("ep", "ulysses"):
            reps = 2 if strategy == "ulysses" else 1
            for _ in range(reps * (layers if strategy == "ulysses" else 1)):
                x = full(rank)
                y = torch.empty_like(x)
                dist.all_to_all_single(y, x)
                st.add("alltoall", (n // world) * esize * world)
                for p in range(world):
                    if p != rank:
                        st.add_peer(p, (n // world) * esize)
                if check:
                    assert float(y[(world - 1) * (n // world)]) == world - 1
        elif strategy == "pp":
            if world > 1:
                buf = full(rank)
                recv = torch.empty_like(buf)
                ops = []
                if rank + 1 < world:
                    ops.append(dist.P2POp(dist.isend, buf, rank + 1))
                if rank > 0:
                    ops.append(dist.P2POp(dist.irecv, recv, rank - 1))
                for r in dist.batch_isend_irecv(ops):
                    r.wait()
                if rank + 1 < world:
                    st.add("send", n * esize)
                    st.add_peer(rank + 1, n * esize)
                if rank > 0:
                    st.add("recv", n * esize)
                    if check:
                        assert float(recv[0]) == rank - 1
        elif strategy == "bcast":
            p = full(7 if rank == 0 else 0)
            dist.broadcast(p, src=0)
            st.add("broadcast", n * esize)
            m = full(rank + 1)
            dist.reduce(m, dst=0)
            st.add("reduce", n * esize)
            if check:
                assert float(p[0]) == 7
                if rank == 0:
                    assert float(m[0]) == world * (world + 1) / 2
        elif strategy == "cp":
            if world > 1:
                kv = full(rank)
                for hop in range(world - 1):
                    recv = torch.empty_like(kv)
                    ops = [dist.P2POp(dist.isend, kv, (rank + 1) % world),
                           dist.P2POp(dist.irecv, recv, (rank - 1) % world)]
                    for r in dist.batch_isend_irecv(ops):
                        r.wait()
                    st.add("send", n * esize)
                    st.add("recv", n * esize)
                    st.add_peer((rank + 1) % world, n * esize)
                    kv = recv
                if check:
                    assert float(kv[0]) == (rank + 1) % world  # after world-1 hops
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    st.seconds = time.perf_counter() - t0
    return st


def ring_allreduce_link_bytes(nbytes: int, world: int) -> float:
    """Bytes each rank sends on ITS outgoing ring link for one ring all-reduce of `nbytes`
    (reduce-scatter + all-gather): 2 (N-1)/N * nbytes.  On an 8-GPU fully connected xGMI
    mesh RCCL spreads channels over the 7 links, but the per-rank total is the same; at
    ~153 GB/s per link the all-reduce is per-link bound (task brief)."""
    return 0.0 if world <= 1 else 2.0 * (world - 1) / world * nbytes
