"""`python -m kubernetes_gpu_exporter_amd.models <workload>` — run a synthetic pod workload.

Single process: `... gemm --steps 100`.  Multi-GPU: under torchrun (one rank per GPU,
RCCL over xGMI), e.g. `torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m
kubernetes_gpu_exporter_amd.models dp --steps 50`.  Prints one JSON line per rank.
"""
import argparse
import json
import os
import sys

from . import WORKLOADS, make, run


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="gpuexp-workload")
    ap.add_argument("workload", choices=WORKLOADS)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--comm-mb", type=float, default=16.0)
    args = ap.parse_args(argv)
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    gpu = torch.cuda.device_count() > 0
    if gpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    if args.workload != "gemm":
        import torch.distributed as dist
        if world == 1 and "MASTER_ADDR" not in os.environ:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29531", RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl" if gpu else "gloo")
    kw = {"size": args.size, "iters": args.iters}
    if args.workload != "gemm":
        kw["comm_bytes"] = int(args.comm_mb * (1 << 20))
    res = run(make(args.workload, **kw), args.steps, args.warmup)
    res["rank"] = int(os.environ.get("RANK", "0"))
    print(json.dumps(res), flush=True)
    if args.workload != "gemm":
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
