import sys, time, torch
sys.path.insert(0, "/root/repo")
from kubernetes_gpu_exporter_amd.ops.gemm import gemm_bf16, gemm_burn
N = 8192
a = torch.randn(N, N, device="cuda", dtype=torch.bfloat16)
b = torch.randn(N, N, device="cuda", dtype=torch.bfloat16)
def bench(fn, iters=30):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize()
    return 2 * N**3 * iters / (time.perf_counter() - t) / 1e12
c = torch.empty(N, N, device="cuda", dtype=torch.bfloat16)
print("hipBLASLt (torch.matmul a @ b.T) TFLOP/s:", round(bench(lambda: torch.matmul(a, b.t(), out=c)), 1))
print("ours (gemm_bf16 256x256) TFLOP/s:", round(bench(lambda: gemm_bf16(a, b, out=c)), 1))
print("hipBLASLt again:", round(bench(lambda: torch.matmul(a, b.t(), out=c)), 1))
print("ours again:", round(bench(lambda: gemm_bf16(a, b, out=c)), 1))
