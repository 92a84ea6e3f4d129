"""RCCL tracer parity on one GPU (run by tools/gpu_features_check.py `rccl` with the tracer
injected through ROCP_TOOL_LIBRARIES).  For every generator strategy that moves data at
world size 1 it reads this process's own tracer file before and after the strategy's
steps, and reports the per-op (calls, bytes) deltas next to the generator's TrafficStats
(the ground truth the tracer must reproduce byte for byte)."""
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

OPS = ["allreduce", "allgather", "reducescatter", "alltoall", "alltoallv", "broadcast", "reduce", "send", "recv",
       "gather", "scatter"]


def counters(path):
    with open(path, "rb") as fh:
        b = fh.read()
    return {nm: struct.unpack_from("<QQ", b, 64 + 16 * i) for i, nm in enumerate(OPS)}


def main():
    import torch
    import torch.distributed as dist
    from kubernetes_gpu_exporter_amd.parallel.collectives import run
    dist.init_process_group("nccl", rank=0, world_size=1)
    torch.cuda.set_device(0)
    ino = os.stat("/proc/self/ns/pid").st_ino
    path = os.path.join(os.environ["GPUEXP_RCCL_DIR"], f"gpuexp-rccl-{ino}-{os.getpid()}")
    warm = torch.ones(16, device="cuda")
    dist.all_reduce(warm)  # communicator up before the first measured strategy
    torch.cuda.synchronize()
    out = {}
    for strategy in ("dp", "tp", "sp", "ep", "ulysses", "bcast"):
        before = counters(path)
        st = run(strategy, steps=3, nbytes=1 << 20, device="cuda", check=True)
        torch.cuda.synchronize()
        after = counters(path)
        delta = {op: [after[op][0] - before[op][0], after[op][1] - before[op][1]] for op in OPS
                 if after[op] != before[op]}
        out[strategy] = {"traced": delta, "expected": {op: [st.calls[op], st.bytes[op]] for op in st.calls}}
    dist.destroy_process_group()
    print("PARITY " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
