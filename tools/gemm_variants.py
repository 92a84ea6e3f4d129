#!/usr/bin/env python3
"""A/B of the synthetic pod's GEMM kernel variants against hipBLASLt (torch.matmul) on one
MI355X, in one process, interleaved: C = A @ B^T, bf16 in / fp32 accumulate / bf16 out,
uniform random operands (cdna_hip_programming.md rule 25).  Each variant's output is first
checked bit-for-bit against the 128x128 kernel (same K order) and against an fp32 reference.

  python3 tools/gemm_variants.py [sizes=4096,8192] [variants=7,8] [rounds=3] [iters=30]

Prints one line per (size, variant, round) and a median summary; kernel time from GPU events
over `iters` back-to-back dispatches after a warm-up.
"""
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch
    from kubernetes_gpu_exporter_amd.ops.gemm import kernels
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4096,8192").split(",")]
    variants = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "7,8").split(",")]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    k = kernels()
    s = torch.cuda.current_stream().cuda_stream
    summary = {}
    for n in sizes:
        a = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        b = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        k.fill_bf16(a.data_ptr(), a.numel(), 11, s)
        k.fill_bf16(b.data_ptr(), b.numel(), 29, s)
        c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        ref = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        k.gemm_bf16(a.data_ptr(), b.data_ptr(), ref.data_ptr(), n, n, n, s, 1)
        torch.cuda.synchronize()
        ref32 = a[:512].float() @ b.float().T  # fp32 reference on a row slice
        for v in variants:
            for rep in range(3):
                c.fill_(float("nan"))
                k.gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), n, n, n, s, v)
                torch.cuda.synchronize()
                same = torch.equal(c, ref)
                if rep == 0:
                    first = c.clone()
                elif not torch.equal(c, first):
                    print(f"RUN-TO-RUN MISMATCH n={n} variant={v} rep={rep}", flush=True)
                    return 1
                if not same and v != 9:  # 9 sums K in 16-deep MFMA steps: not bitwise
                    print(f"MISMATCH n={n} variant={v} rep={rep}: max diff "
                          f"{(c.float() - ref.float()).abs().max().item()}", flush=True)
                    return 1
            err = ((c[:512].float() - ref32).abs() / (ref32.abs() + 1.0)).max().item()
            if err > 2e-2:
                print(f"n={n} variant={v}: max rel err vs fp32 {err:.2e} TOO LARGE", flush=True)
                return 1
            print(f"n={n} variant={v}: {'bitwise == 128x128 kernel, ' if same else ''}"
                  f"max rel err vs fp32 {err:.2e}", flush=True)

        def run(fn):
            for _ in range(10):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / iters
            return ms, 2.0 * n ** 3 / (ms * 1e-3) / 1e12

        arms = {"hipblaslt": lambda: torch.matmul(a, b.t(), out=c)}
        for v in variants:
            arms[f"v{v}"] = (lambda v=v: k.gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), n, n, n, s, v))
        for r in range(rounds):
            for name, fn in arms.items():
                ms, tf = run(fn)
                summary.setdefault((n, name), []).append(tf)
                print(f"n={n} round={r} {name}: {ms * 1e3:.1f} us  {tf:.1f} TFLOP/s", flush=True)
    print("--- median TFLOP/s")
    for n in sizes:
        base = statistics.median(summary[(n, "hipblaslt")])
        for name in ["hipblaslt"] + [f"v{v}" for v in variants]:
            m = statistics.median(summary[(n, name)])
            print(f"n={n} {name:10s} {m:8.1f}  ({m / base * 100:.1f} % of hipBLASLt)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
