// Synthetic "HIP-GEMM pod" workload: C[M,N] (bf16) = A[M,K] . B[N,K]^T (bf16 in, fp32 acc).
//
// This is the load generator behind BASELINE configs 3-5 ("synthetic HIP-workload pods")
// — the exporter itself issues no GEMMs.  Written for CDNA4 directly:
//   * v_mfma_f32_16x16x32_bf16 (gfx950), 4 waves of 64 lanes, 128x128 block tile, BK=64;
//     each wave owns a 64x64 sub-tile = 4x4 MFMA tiles (acc[mi][ni], never indexed by
//     wave position — cdna_hip_programming.md §5 "Wave->output-tile decomposition").
//   * global->LDS with __builtin_amdgcn_global_load_lds (16 B/lane, lane-linear 1 KiB per
//     wave-instruction); the LDS image is XOR-swizzled by pre-swizzling the GLOBAL source
//     chunk (both-sides rule 21), chunk' = chunk ^ ((row>>1)&7) so the 16 rows one
//     ds_read_b128 group touches spread over the 16 slots of a 256-B bank row.
//   * double-buffered K loop (one barrier per K-step), all LDS in one __shared__ array
//     (trap 4(a)), bijective XCD-aware block remap (T1).
// Requirements (checked on the host before launch): M%128 == N%128 == K%64 == 0.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace gpuexp {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gptr_t;

constexpr int kBM = 128, kBN = 128, kBK = 64, kThreads = 256;
constexpr int kTileElems = 128 * kBK;  // one operand tile (A or B) in bf16 elements

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Issues this wave's 4 glds for one 128x64 operand tile: wave-instruction i covers rows
// [(w*4+i)*8, +8); lane l -> row +(l>>3), LDS chunk position l&7, which holds global
// chunk swz(row, l&7) (swz is an involution).
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ g, int ld, int row0, int k0,
                                           uint16_t* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int rblk = (wave * 4 + i) * 8;
    int row = rblk + (lane >> 3);
    int c = swz(row, lane & 7);
    const uint16_t* src = g + size_t(row0 + row) * size_t(ld) + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lds_ptr_t)(lds_tile + rblk * kBK), 16, 0, 0);
  }
}

__global__ void __launch_bounds__(kThreads, 2)
gemm_bf16_tn_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                    int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 2 * kTileElems];  // 64 KiB: [buf][A|B]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // Bijective XCD-aware remap: blocks sharing blockIdx%8 (one XCD under round-robin
  // dispatch) get a contiguous range of tiles, i.e. the same A row panels in their L2.
  const int nbn = N / kBN;
  const int nwg = (M / kBM) * nbn;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int bm = wgid / nbn, bn = wgid % nbn;
  const int row_a = bm * kBM, row_b = bn * kBN;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / kBK;
  stage_tile(A, K, row_a, 0, smem, wave, lane);
  stage_tile(B, K, row_b, 0, smem + kTileElems, wave, lane);

  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // tile kt landed for every wave; buffer (kt+1)&1 is free
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      uint16_t* nxt = smem + ((kt + 1) & 1) * 2 * kTileElems;
      stage_tile(A, K, row_a, (kt + 1) * kBK, nxt, wave, lane);
      stage_tile(B, K, row_b, (kt + 1) * kBK, nxt + kTileElems, wave, lane);
    }
    const uint16_t* As = smem + cur * 2 * kTileElems;
    const uint16_t* Bs = As + kTileElems;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        int row = wm * 64 + mi * 16 + (lane & 15);
        af[mi] = *reinterpret_cast<const bf16x8*>(As + row * kBK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        int row = wn * 64 + ni * 16 + (lane & 15);
        bfr[ni] = *reinterpret_cast<const bf16x8*>(Bs + row * kBK + swz(row, chunk) * 8);
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
  }

  // Epilogue: C/D map of 16x16x32: col = lane&15, row = (lane>>4)*4 + j.
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int row = row_a + wm * 64 + mi * 16 + (lane >> 4) * 4 + j;
        int col = row_b + wn * 64 + ni * 16 + (lane & 15);
        __bf16 v = (__bf16)acc[mi][ni][j];
        C[size_t(row) * size_t(N) + col] = *reinterpret_cast<uint16_t*>(&v);
      }
}

// Fills a bf16 buffer with uniform [-1, 1) values from a counter hash (random operands:
// zero-filled GEMMs run at an unrepresentative clock, cdna_hip_programming.md rule 25).
__global__ void fill_bf16_kernel(uint16_t* __restrict__ p, size_t n, uint32_t seed) {
  size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  size_t stride = size_t(gridDim.x) * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t x = uint32_t(i) * 2654435761u ^ seed;
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    float f = float(x & 0xFFFFFF) / float(0x1000000) * 2.f - 1.f;
    __bf16 v = (__bf16)f;
    p[i] = *reinterpret_cast<uint16_t*>(&v);
  }
}

bool gemm_shape_ok(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && M % kBM == 0 && N % kBN == 0 && K % kBK == 0;
}

hipError_t launch_gemm_bf16_tn(const void* A, const void* B, void* C, int M, int N, int K, hipStream_t stream) {
  if (!gemm_shape_ok(M, N, K)) return hipErrorInvalidValue;
  dim3 grid((M / kBM) * (N / kBN)), block(kThreads);
  hipLaunchKernelGGL(gemm_bf16_tn_kernel, grid, block, 0, stream, static_cast<const uint16_t*>(A),
                     static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M, N, K);
  return hipGetLastError();
}

hipError_t launch_fill_bf16(void* p, size_t n, uint32_t seed, hipStream_t stream) {
  hipLaunchKernelGGL(fill_bf16_kernel, dim3(1024), dim3(256), 0, stream, static_cast<uint16_t*>(p), n, seed);
  return hipGetLastError();
}

}  // namespace gpuexp
