"""bf16 MFMA GEMM (hand-written HIP for gfx950, csrc/kernels/gemm_bf16.hip) — the
synthetic "HIP-GEMM pod" workload of BASELINE configs 3-5.

`_gpuexp_kernels` links a HIP runtime.  torch ROCm wheels bundle their own
libamdhip64.so.7 (same SONAME as /opt/rocm's), so when torch is installed it is imported
FIRST: the kernels module's DT_NEEDED then binds to torch's already-loaded runtime
instead of loading a second one into the process.
"""
from __future__ import annotations

import importlib

_mod = None


def kernels():
    global _mod
    if _mod is None:
        try:
            import torch  # noqa: F401  (load torch's HIP runtime first)
        except ImportError:
            pass
        _mod = importlib.import_module("kubernetes_gpu_exporter_amd._gpuexp_kernels")
    return _mod


def gemm_bf16(a, b, out=None, stream=None, variant: int = 0):
    """out[M,N] = a[M,K] @ b[N,K]^T for contiguous bf16 torch tensors on one GPU.
    Shapes must satisfy M%128 == N%128 == K%64 == 0 (checked by the native op).
    variant 0 picks the 256x256-tile kernel when M%256 == N%256 == 0 and K >= 128, else
    the 128x128 one; 1 / 2 force the 128x128 / 256x256 kernel."""
    import torch
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise TypeError("gemm_bf16 expects bf16 tensors")
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[1]:
        raise ValueError(f"shape mismatch {tuple(a.shape)} x {tuple(b.shape)}^T")
    if not (a.is_contiguous() and b.is_contiguous()):
        raise ValueError("operands must be contiguous (row-major, K innermost)")
    if a.device != b.device or a.device.type != "cuda":
        raise ValueError("operands must be on the same GPU")
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
    elif out.shape != (M, N) or out.dtype != torch.bfloat16 or not out.is_contiguous():
        raise ValueError("bad output tensor")
    s = stream if stream is not None else torch.cuda.current_stream(a.device).cuda_stream
    kernels().gemm_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, s, variant)
    return out


def gemm_burn(device: int = 0, size: int = 8192, seconds: float = 1.0, iters_per_sync: int = 4,
              variant: int = 0) -> dict:
    """Torch-free GPU load: keeps `device` busy with size^3 GEMMs for `seconds`."""
    return kernels().gemm_burn(device, size, size, size, seconds, iters_per_sync, variant)


def stream_copy(src, dst, stream=None, blocks: int = 4096):
    """dst <- src (same nbytes, contiguous, one GPU) with the calibration copy kernel:
    reads and writes each byte of HBM exactly once."""
    import torch
    n = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != n or not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("src and dst must be contiguous and of equal size")
    if src.device != dst.device or src.device.type != "cuda":
        raise ValueError("tensors must be on the same GPU")
    s = stream if stream is not None else torch.cuda.current_stream(src.device).cuda_stream
    kernels().stream_copy(src.data_ptr(), dst.data_ptr(), n, blocks, s)


def lds_probe(out, blocks: int, iters: int, conflicts: bool, stream=None):
    """`blocks` x 256 threads of LDS reads; conflicts=True makes every read 32-way
    bank-conflicted, False conflict-free.  `out`: float32 tensor with >= blocks elements."""
    import torch
    if out.dtype != torch.float32 or out.numel() < blocks or out.device.type != "cuda":
        raise ValueError("out must be a float32 GPU tensor with >= blocks elements")
    s = stream if stream is not None else torch.cuda.current_stream(out.device).cuda_stream
    kernels().lds_probe(out.data_ptr(), blocks, iters, 32 if conflicts else 1, s)


def mfma_duty(device: int, duty: float, seconds: float, period_s: float = 0.002, stream=None,
              blocks: int | None = None, xcc_mask: int = 0):
    """Launches the MFMA duty-cycle calibration kernel on `device` (non-blocking): 2 blocks
    of 4 waves per CU (2 waves per SIMD) alternate back-to-back v_mfma_f32_32x32x16_bf16 for
    duty x period_s with s_sleep for the rest, for `seconds`.  xcc_mask != 0 runs only the
    blocks that land on those XCCs (bit x = HW_REG_XCC_ID x); the others exit at once.
    Returns (out, counts) tensors; counts[w] = MFMAs wave w issued (valid after the kernel
    finished; 0 for the waves of skipped blocks)."""
    import torch
    if not (0.0 <= duty <= 1.0) or not (0 < seconds <= 60) or not (1e-5 <= period_s <= 1.0):
        raise ValueError("duty in [0,1], 0 < seconds <= 60, 1e-5 <= period_s <= 1")
    if not (0 <= xcc_mask < 1 << 32):
        raise ValueError("xcc_mask is a 32-bit XCC bit set")
    dev = torch.device(f"cuda:{device}")
    if blocks is None:
        blocks = 2 * torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.zeros(blocks, dtype=torch.float32, device=dev)
    counts = torch.zeros(blocks * 4, dtype=torch.int64, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    kernels().mfma_duty(out.data_ptr(), counts.data_ptr(), blocks, float(duty), float(period_s), float(seconds), s,
                        int(xcc_mask))
    return out, counts


_HOG_KINDS = {"lds": (0, 2), "waves": (1, 4), "vgpr": (2, 4), "sgpr": (3, 28)}  # kernel, blocks per CU that fit


def occupancy_hog(device: int, kind: str, seconds: float, generations: int = 4, stream=None):
    """Launches blocks that each hold a resource for `seconds` (non-blocking), `generations`
    times as many as fit at once, so ready waves queue in the dispatcher for a known reason:
    kind "lds" = 1 wave + 64 KiB LDS per block (2 per CU fit: LDS-limited), "waves" = 8 waves
    per block, no LDS (4 per CU fit: wave-slot-limited), "vgpr" = 1 wave of 400 registers per
    lane (1 per SIMD fits: VGPR-limited), "sgpr" = 1 wave of 108 SGPRs (7 per SIMD fit, of 8
    slots: SGPR-limited).  Returns the sink tensor."""
    import torch
    if kind not in _HOG_KINDS or not (0 < seconds <= 10) or not (1 <= generations <= 64):
        raise ValueError("kind lds|waves|vgpr|sgpr, 0 < seconds <= 10, 1 <= generations <= 64")
    code, per_cu = _HOG_KINDS[kind]
    dev = torch.device(f"cuda:{device}")
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    blocks = cus * per_cu * generations
    out = torch.zeros(blocks, dtype=torch.float32, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    kernels().occupancy_hog(code, out.data_ptr(), blocks, float(seconds), s)
    return out
