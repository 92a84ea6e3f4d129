#!/usr/bin/env python3
"""Runs `iters` dispatches of ONE GEMM arm (our kernel variant `vN`, or `blas` =
torch.matmul / hipBLASLt) at n^3 bf16 on uniform random operands, for `rocprofv3 --pmc`
passes that compare the arms counter by counter:
  rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES ... -d gpurun_out/pmc -o v8 -- python3 tools/gemm_arm.py v8 8192 20
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    arm = sys.argv[1] if len(sys.argv) > 1 else "v8"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    import torch
    from kubernetes_gpu_exporter_amd.ops.gemm import kernels
    k = kernels()
    s = torch.cuda.current_stream().cuda_stream
    a = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    b = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    k.fill_bf16(a.data_ptr(), a.numel(), 11, s)
    k.fill_bf16(b.data_ptr(), b.numel(), 29, s)
    if arm == "blas":
        fn = lambda: torch.matmul(a, b.t(), out=c)  # noqa: E731
    else:
        v = int(arm.lstrip("v"))
        fn = lambda: k.gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), n, n, n, s, v)  # noqa: E731
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    print(f"{arm} {n}^3 x {iters} done", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
