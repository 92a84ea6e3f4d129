"""Host-side checks of the HIP workload-kernel module (no GPU needed): which GEMM kernel a
launch resolves to.  The numerics of every variant are GPU tests (tests/test_gpu.py)."""
import pytest

from kubernetes_gpu_exporter_amd.ops.gemm import kernels


@pytest.mark.parametrize("M,N,K,variant,want", [
    (8192, 8192, 8192, 0, 8),   # the bench's pod GEMM: the ping-pong 256x256 kernel
    (4096, 4096, 1024, 0, 8),
    (256, 256, 128, 0, 8),
    (256, 256, 64, 0, 1),       # K < 128: the 256x256 pipeline needs two K-tiles
    (384, 256, 512, 0, 1),      # M % 256 != 0
    (128, 128, 64, 0, 1),
    (8192, 8192, 8192, 7, 7),
    (8192, 8192, 8192, 9, 9),
    (384, 256, 512, 9, -1),     # explicit 256x256 variant on a shape it cannot run
    (100, 128, 64, 0, -1),
    (256, 256, 128, 10, -1),
])
def test_gemm_variant_resolution(native, M, N, K, variant, want):
    assert kernels().gemm_variant(M, N, K, variant) == want
