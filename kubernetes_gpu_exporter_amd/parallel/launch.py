"""Multi-process launch helpers: one process per rank, 127.0.0.1 rendezvous.

`spawn(fn, world, backend)` runs fn(rank, world, *args) in `world` fresh processes with an
initialised default process group ("gloo" on CPU, "nccl" = RCCL on GPUs) and returns the
per-rank results.  `traffic_worker` drives a strategy from parallel/collectives.py.
Command line (one rank per GPU of a node, e.g. as synthetic RCCL pods):
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
      -m kubernetes_gpu_exporter_amd.parallel.launch --strategy ep --steps 100 --mb 64
"""
from __future__ import annotations

import argparse
import json
import os
import socket


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, backend, fn, args, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world, *args)))
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, e))
    finally:
        dist.destroy_process_group()


def spawn(fn, world: int, backend: str = "gloo", args: tuple = (), timeout: float = 120.0) -> list:
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, backend, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, v = q.get(timeout=timeout)
            out[r] = v
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    errs = [v for v in out.values() if isinstance(v, Exception)]
    if errs:
        raise errs[0]
    return [out[r] for r in range(world)]


def traffic_worker(rank: int, world: int, strategy: str, steps: int, nbytes: int, device: str | None = None):
    from .collectives import run
    st = run(strategy, steps=steps, nbytes=nbytes, device=device)
    return {"calls": st.calls, "bytes": st.bytes, "seconds": st.seconds}


def workload_worker(rank: int, world: int, name: str, steps: int, kw: dict):
    from ..models import make, run
    return run(make(name, **kw), steps, warmup=1)


def main() -> int:
    import torch
    import torch.distributed as dist
    from .collectives import STRATEGIES, run
    ap = argparse.ArgumentParser()
    ap.add_argument("--strategy", choices=STRATEGIES, default="dp")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mb", type=float, default=16.0)
    a = ap.parse_args()
    gpu = torch.cuda.is_available()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if gpu:
        torch.cuda.set_device(local)
    dist.init_process_group("nccl" if gpu else "gloo")
    st = run(a.strategy, steps=a.steps, nbytes=int(a.mb * (1 << 20)), device=f"cuda:{local}" if gpu else None)
    if dist.get_rank() == 0:
        print(json.dumps({"strategy": a.strategy, "world": st.world, "calls": st.calls, "bytes": st.bytes,
                          "seconds": round(st.seconds, 4)}))
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
