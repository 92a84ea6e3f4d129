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


def rccl_lib():
    """The librccl this process already runs (torch's), so the tracer sees the same API table."""
    import ctypes
    with open("/proc/self/maps") as fh:
        for line in fh:
            p = line.split()[-1]
            if os.path.basename(p).startswith("librccl.so"):
                return ctypes.CDLL(p)
    raise RuntimeError("librccl not mapped")


def p2p_ops(torch, nbytes=1 << 20, steps=3):
    """PP/CP point-to-point and root-based ops at world size 1, through RCCL's C API (torch
    refuses a send to its own rank): a grouped ncclSend + ncclRecv to self (RCCL's local p2p
    copy), ncclGather and ncclScatter with root 0.  Returns (traced-op expectations, ok)."""
    import ctypes
    lib = rccl_lib()
    class UniqueId(ctypes.Structure):  # passed by value (a bare ctypes array would decay to a pointer)
        _fields_ = [("internal", ctypes.c_char * 128)]

    uid = UniqueId()
    comm = ctypes.c_void_p()
    assert lib.ncclGetUniqueId(ctypes.byref(uid)) == 0
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UniqueId, ctypes.c_int]
    rc = lib.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0)
    assert rc == 0, f"ncclCommInitRank: {rc}"
    n = nbytes // 4
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    src = torch.arange(n, device="cuda", dtype=torch.float32)
    dst = torch.zeros_like(src)
    F32 = 7  # ncclFloat32
    sz = ctypes.c_size_t
    for f in ("ncclSend", "ncclRecv"):
        getattr(lib, f).argtypes = [ctypes.c_void_p, sz, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    for f in ("ncclGather", "ncclScatter"):
        getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, sz, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p]
    ok = True
    for _ in range(steps):
        dst.zero_()
        assert lib.ncclGroupStart() == 0
        assert lib.ncclSend(ctypes.c_void_p(src.data_ptr()), n, F32, 0, comm, stream) == 0
        assert lib.ncclRecv(ctypes.c_void_p(dst.data_ptr()), n, F32, 0, comm, stream) == 0
        assert lib.ncclGroupEnd() == 0
        torch.cuda.synchronize()
        ok = ok and bool(torch.equal(dst, src))
        dst.zero_()
        assert lib.ncclGather(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), n, F32, 0, comm,
                              stream) == 0
        torch.cuda.synchronize()
        ok = ok and bool(torch.equal(dst, src))
        dst.zero_()
        assert lib.ncclScatter(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), n, F32, 0, comm,
                               stream) == 0
        torch.cuda.synchronize()
        ok = ok and bool(torch.equal(dst, src))
    lib.ncclCommDestroy(comm)
    return {op: [steps, steps * nbytes] for op in ("send", "recv", "gather", "scatter")}, ok


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
    before = counters(path)
    expected, data_ok = p2p_ops(torch)
    after = counters(path)
    out["p2p"] = {"traced": {op: [after[op][0] - before[op][0], after[op][1] - before[op][1]] for op in OPS
                             if after[op] != before[op]}, "expected": expected, "data_ok": data_ok}
    dist.destroy_process_group()
    print("PARITY " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
