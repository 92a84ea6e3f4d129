// Synthetic "HIP-GEMM pod" workload: C[M,N] (bf16) = A[M,K] . B[N,K]^T (bf16 in, fp32 acc).
// Two kernels: the 256x256 one below the 128x128 one is the default whenever the shape
// allows (M,N multiples of 256); its default form is the ping-pong variant 8: MI355X,
// random operands, 8192^3 1497 TFLOP/s (91 % of torch.matmul / hipBLASLt; 93 % at 4096^3) vs
// 1357 for the previous one-barrier-per-phase form (profiles/r03/gemm_variants.log).
//
// 128x128 kernel:
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
#include <type_traits>

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

// ---------------------------------------------------------------------------------------
// 256x256 tile, 8 waves (2 along M x 4 along N), BK=64, loads that stay in flight across
// barriers.  Each wave owns a 128x64 output block = 2x2 quadrants of 64x32; one K-tile is
// four phases, one quadrant per phase (16 MFMA 16x16x32 each), ordered so that each phase
// reads ONE new row group of the LDS tile and the group it finished with is free for the
// K-tile two ahead:
//   phase 1: ds_read A rows M0 (wave-row's first 64) + B rows N0 (wave-col's first 32) -> Q00
//   phase 2: ds_read B rows N1                      -> Q01;  stage t+2: A-M0 + B-N0 groups
//   phase 3: ds_read A rows M1 (over the M0 frags)  -> Q11;  stage t+2: B-N1 group
//   phase 4: (registers only)                       -> Q10;  stage t+2: A-M1 group
// A "group" is 128 tile rows x 64 K (16 KiB) = 2 global_load_lds x 16 B per thread.  Every
// phase ends in one raw s_barrier after the wave's own ds_reads retired (lgkmcnt(0)), so a
// group staged in phase p+1 never overwrites rows still being read (WAR).  K-tile t+1 was
// staged during phases 2-4 of K-tile t-1; the counted wait before phase 4's barrier,
// vmcnt(8), retires it while t+2's 8 loads stay in flight (RAW: read one barrier after the
// wait).  No __syncthreads() in the loop (its fence would drain vmcnt to 0) and all LDS is
// one __shared__ array (cdna_hip_programming.md §5 "Pipelining across barriers", 4(a)).
// Epilogue: the 256x256 bf16 C tile goes through the (then idle) 128 KiB of LDS so every
// global store is a full 16-B chunk of a 512-B row.
// Requirements (host-checked): M%256 == N%256 == 0, K%64 == 0, K >= 128.
// ---------------------------------------------------------------------------------------
constexpr int kBM2 = 256, kBN2 = 256, kThreads2 = 512;
constexpr int kTile2 = 256 * kBK;  // one operand K-tile (bf16 elements), 32 KiB

// Stages one 128-row group of a 256x64 operand tile: row-block rb (8 rows) of the group
// starts at tile row  run * run_stride + off + (rb % blocks_per_run) * 8.
template <int kBlocksPerRun, int kRunStride>
__device__ __forceinline__ void stage_group(const uint16_t* __restrict__ g, int ld, int row0, int k0, int off,
                                            uint16_t* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rb = wave * 2 + i;  // 0..15
    const int trow = (rb / kBlocksPerRun) * kRunStride + off + (rb % kBlocksPerRun) * 8;
    const int row = trow + (lane >> 3);
    const int c = swz(row, lane & 7);
    const uint16_t* src = g + size_t(row0 + row) * size_t(ld) + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lds_ptr_t)(lds_tile + trow * kBK), 16, 0, 0);
  }
}

// A groups: M0 = rows {wr*128 + 0..63}, M1 = {wr*128 + 64..127}  (2 runs of 8 blocks)
// B groups: N0 = rows {wc*64 + 0..31},  N1 = {wc*64 + 32..63}    (4 runs of 4 blocks)
#define GEMM2_STAGE_A(half, t)                                                                      \
  stage_group<8, 128>(A, K, row_a, (t) * kBK, (half) * 64, smem + ((t) & 1) * 2 * kTile2, wave, lane)
#define GEMM2_STAGE_B(half, t)                                                                      \
  stage_group<4, 64>(B, K, row_b, (t) * kBK, (half) * 32, smem + ((t) & 1) * 2 * kTile2 + kTile2, wave, lane)

__device__ __forceinline__ void read_frags(const uint16_t* tile, int row_base, int lane, bf16x8 (&f)[4][2],
                                           int n) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= n) break;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int row = row_base + i * 16 + (lane & 15);
      const int chunk = kk * 4 + (lane >> 4);
      f[i][kk] = *reinterpret_cast<const bf16x8*>(tile + row * kBK + swz(row, chunk) * 8);
    }
  }
}

// kPrio 0: raise the wave's priority around each 16-MFMA cluster (T5); 1: no setprio;
// 2: static — wave row 1 (the later half) runs at priority 1 throughout, set once.
template <int kPrio>
__device__ __forceinline__ void mfma_quadrant(f32x4 (&acc)[4][2], const bf16x8 (&af)[4][2],
                                              const bf16x8 (&bf)[4][2]) {
  if (kPrio == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][kk], bf[ni][kk], acc[mi][ni], 0, 0, 0);
  if (kPrio == 0) __builtin_amdgcn_s_setprio(0);
}

// Ends a phase: this wave's ds_reads have landed (so the rows they read may be restaged
// once every wave passes the barrier), then the barrier itself.
__device__ __forceinline__ void phase_end() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // keep the next phase's LDS accesses below the barrier
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Wave-row stagger: the two wave rows (waves 0-3 and 4-7; every SIMD holds one of each)
// run one phase apart — wave row 1 passes one extra barrier before the loop and row 0 one
// after it — so on each SIMD one wave issues its phase's ds_reads while the other keeps
// the MFMA pipe busy.  Because a barrier interval now holds phase p of row 0 and p-1 of
// row 1, a group read in phase p is restaged in phase p+2 at the earliest (row 1 may still
// be reading it during row 0's p+1):
//   phase 1: read A-M0 + B-N0 -> Q00;  stage A-M1 of K-tile t+1
//   phase 2: read B-N1        -> Q01
//   phase 3: read A-M1        -> Q11;  stage A-M0 + B-N0 of t+2
//   phase 4: (registers)      -> Q10;  stage B-N1 of t+2
// Counted waits, placed for the EARLIER row (row 1 reads one barrier after row 0 arrives,
// so every wave waits before the barrier that precedes row 0's read): end of phase 3
// retires t+1's A-M0/B-N0/B-N1 (then in flight: t+1's A-M1, t+2's first 4), end of phase 1
// retires t's A-M1 (then in flight: t+1's first 6 + A-M1).
template <int kGroupM, int kPrio, bool kSnake = false>
__global__ void __launch_bounds__(kThreads2, 1)
gemm_bf16_tn_256_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                        int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 2 * kTile2];  // 128 KiB: [buf][A|B][256][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR: branches on it are scalar
  const int wr = wave >> 2, wc = wave & 3;

  const int nbn = N / kBN2, nbm = M / kBM2;
  const int nwg = nbm * nbn;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  // Grouped tile order inside each XCD's contiguous range: kGroupM row panels x all
  // column panels, column-major within the group, so the ~32 blocks an XCD runs at once
  // cover a kGroupM x (32/kGroupM) patch and share its A and B panels in that XCD's L2.
  const int in_group = kGroupM * nbn;
  const int first_m = (wgid / in_group) * kGroupM;
  const int gsize = nbm - first_m < kGroupM ? nbm - first_m : kGroupM;
  const int bm = first_m + (wgid % in_group) % gsize;
  const int bn = (wgid % in_group) / gsize;
  const int row_a = bm * kBM2, row_b = bn * kBN2;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / kBK;  // >= 2
  bf16x8 af[4][2], b0[4][2], b1[4][2];
  const int a_row = wr * 128, b_row = wc * 64;
  if constexpr (kSnake) {
    // Balanced reads (8/4/8/4 per phase instead of 12/4/8/0): phase 4 prefetches the B
    // group the NEXT K-tile starts with into the B registers phase 4 does not use, and the
    // quadrant order alternates with K-tile parity to make that possible:
    //   even t: P1 read A-M0 -> Q00(b0) | P2 read B-N1 -> Q01 | P3 read A-M1 -> Q11 | P4 read B-N1(t+1) -> Q10(b0)
    //   odd  t: P1 read A-M0 -> Q01(b1) | P2 read B-N0 -> Q00 | P3 read A-M1 -> Q10 | P4 read B-N0(t+1) -> Q11(b1)
    // Staging of t+2 (buffer t&1), every group >= 2 phases after its last read under the
    // stagger: P1 A-M1 of t+1; P3 A-M0 + the B group read at P4(t-1); P4 the B group read
    // at P2.  Waits (before the barrier that precedes row 0's read): end of P1 retires
    // t's A-M1; end of P2 t+1's first 4 loads (A-M0 + the prefetched B); end of P4 t+1's
    // other B group.
    GEMM2_STAGE_A(0, 0); GEMM2_STAGE_B(0, 0); GEMM2_STAGE_B(1, 0); GEMM2_STAGE_A(1, 0);
    GEMM2_STAGE_A(0, 1); GEMM2_STAGE_B(1, 1); GEMM2_STAGE_B(0, 1);  // tile 1 (odd) order
    wait_vm<6>();  // K-tile 0 landed
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger: row 1 one phase behind
    if (kPrio == 2 && wr == 1) __builtin_amdgcn_s_setprio(1);
    asm volatile("" ::: "memory");
    read_frags(smem + kTile2, b_row, lane, b0, 2);  // B-N0 of tile 0 ("phase 4 of tile -1")
    auto tile = [&](int t, auto odd_tag) {
      constexpr bool odd = decltype(odd_tag)::value;
      const uint16_t* As = smem + (odd ? 2 * kTile2 : 0);
      const uint16_t* Bs = As + kTile2;
      const uint16_t* Bn = smem + (odd ? 0 : 2 * kTile2) + kTile2;
      const bool has1 = t + 1 < nk, has2 = t + 2 < nk;
      // phase 1
      read_frags(As, a_row, lane, af, 4);
      if (has1) GEMM2_STAGE_A(1, t + 1);
      if constexpr (odd) mfma_quadrant<kPrio>(acc[0][1], af, b1); else mfma_quadrant<kPrio>(acc[0][0], af, b0);
      if (has1) wait_vm<8>(); else wait_vm<0>();  // this tile's A-M1 landed
      phase_end();
      // phase 2
      if constexpr (odd) {
        read_frags(Bs, b_row, lane, b0, 2);
        mfma_quadrant<kPrio>(acc[0][0], af, b0);
      } else {
        read_frags(Bs, b_row + 32, lane, b1, 2);
        mfma_quadrant<kPrio>(acc[0][1], af, b1);
      }
      if (has1) wait_vm<4>(); else wait_vm<0>();  // t+1's A-M0 + first B group landed
      phase_end();
      // phase 3
      read_frags(As, a_row + 64, lane, af, 4);
      if (has2) {
        GEMM2_STAGE_A(0, t + 2);
        if constexpr (odd) GEMM2_STAGE_B(1, t + 2); else GEMM2_STAGE_B(0, t + 2);
      }
      if constexpr (odd) mfma_quadrant<kPrio>(acc[1][0], af, b0); else mfma_quadrant<kPrio>(acc[1][1], af, b1);
      phase_end();
      // phase 4
      if constexpr (odd) {
        if (has1) read_frags(Bn, b_row, lane, b0, 2);
        if (has2) GEMM2_STAGE_B(0, t + 2);
        mfma_quadrant<kPrio>(acc[1][1], af, b1);
      } else {
        if (has1) read_frags(Bn, b_row + 32, lane, b1, 2);
        if (has2) GEMM2_STAGE_B(1, t + 2);
        mfma_quadrant<kPrio>(acc[1][0], af, b0);
      }
      if (has2) wait_vm<8>(); else if (has1) wait_vm<2>(); else wait_vm<0>();  // t+1's second B group
      phase_end();
    };
    for (int t = 0; t < nk; t += 2) {
      tile(t, std::false_type{});
      if (t + 1 < nk) tile(t + 1, std::true_type{});
    }
  } else {
  GEMM2_STAGE_A(0, 0); GEMM2_STAGE_B(0, 0); GEMM2_STAGE_B(1, 0); GEMM2_STAGE_A(1, 0);
  GEMM2_STAGE_A(0, 1); GEMM2_STAGE_B(0, 1); GEMM2_STAGE_B(1, 1);
  wait_vm<6>();  // K-tile 0 landed; tile 1's first three groups in flight
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger: row 1 one phase behind
  if (kPrio == 2 && wr == 1) __builtin_amdgcn_s_setprio(1);
  asm volatile("" ::: "memory");

  for (int t = 0; t < nk; ++t) {
    const uint16_t* As = smem + (t & 1) * 2 * kTile2;
    const uint16_t* Bs = As + kTile2;
    const bool has1 = t + 1 < nk, has2 = t + 2 < nk;
    // phase 1
    read_frags(As, a_row, lane, af, 4);
    read_frags(Bs, b_row, lane, b0, 2);
    if (has1) GEMM2_STAGE_A(1, t + 1);
    mfma_quadrant<kPrio>(acc[0][0], af, b0);
    if (has1) wait_vm<8>(); else wait_vm<0>();  // this tile's A-M1 landed
    phase_end();
    // phase 2
    read_frags(Bs, b_row + 32, lane, b1, 2);
    mfma_quadrant<kPrio>(acc[0][1], af, b1);
    phase_end();
    // phase 3
    read_frags(As, a_row + 64, lane, af, 4);
    if (has2) { GEMM2_STAGE_A(0, t + 2); GEMM2_STAGE_B(0, t + 2); }
    mfma_quadrant<kPrio>(acc[1][1], af, b1);
    if (has2) wait_vm<6>(); else if (has1) wait_vm<2>(); else wait_vm<0>();  // t+1's first 3 groups landed
    phase_end();
    // phase 4
    if (has2) GEMM2_STAGE_B(1, t + 2);
    mfma_quadrant<kPrio>(acc[1][0], af, b0);
    phase_end();
  }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // close the stagger: row 1's last phase is done
  asm volatile("" ::: "memory");

  // Epilogue through LDS: every wave's reads retired before its last barrier and the last
  // K-tiles waited vmcnt(0), so the 128 KiB are free.
  // C/D map of 16x16x32: col = lane&15, row = (lane>>4)*4 + j.
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = wr * 128 + qm * 64 + mi * 16 + (lane >> 4) * 4 + j;
            const int col = wc * 64 + qn * 32 + ni * 16 + (lane & 15);
            __bf16 v = (__bf16)acc[qm][qn][mi][ni][j];
            smem[row * kBN2 + col] = *reinterpret_cast<uint16_t*>(&v);
          }
  __syncthreads();
#pragma unroll 4
  for (int p = 0; p < (kBM2 * kBN2 / 8) / kThreads2; ++p) {  // 16 passes of 512 x 16 B
    const int idx = p * kThreads2 + threadIdx.x;
    const int row = idx >> 5, chunk = idx & 31;
    const uint4 v = *reinterpret_cast<const uint4*>(smem + row * kBN2 + chunk * 8);
    *reinterpret_cast<uint4*>(C + size_t(row_a + row) * size_t(N) + row_b + chunk * 8) = v;
  }
}
// ---------------------------------------------------------------------------------------
// Ping-pong form of the 256x256 kernel (variant 8, the default): same tile, waves, LDS
// image, snake-B read order and epilogue, but every phase is
//   ds_reads of this phase's group -> stage ONE group (2 glds) -> counted vmcnt ->
//   s_barrier -> lgkmcnt(0) -> 16 MFMA -> s_barrier
// and wave row 1 runs one barrier behind row 0, so on every SIMD one wave's MFMA cluster
// runs while the other wave's reads and DMA issue run (cdna_hip_programming.md, "The 256²
// 8-phase template").  With two barriers per phase a group is restaged >= 2 phases after
// its last read and read >= 1 phase after the wait that retires it.  Numbering phases
// g = 4t + p - 1, the group reads of K-tile t are
//   Bf(t) at 4t-1 (read ahead into the idle B registers), A-M0 at 4t, Bs(t) at 4t+1,
//   A-M1 at 4t+2        (Bf = B-N0 for even t, B-N1 for odd t; Bs the other half)
// and one group is staged per phase:
//   P1 A-M1(t+1),  P2 Bf(t+2),  P3 A-M0(t+2),  P4 Bs(t+2)
// (its DMA issued before the phase's ds_reads) so every group is issued 2 phases after its last read in the same buffer, and 6 phases
// before its first read: each phase waits for the group issued 5 phases earlier (vmcnt =
// 2 x the groups issued since, 10 in steady state; pp_wait below), 1 phase before the read.
// ---------------------------------------------------------------------------------------
// s_waitcnt through the builtin, not inline asm, so the compiler's own wait tracking sees
// it (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8]); otherwise it
// re-waits lgkmcnt(0) for reads these waits already retired.
constexpr int waitcnt_vm(int n) { return (n & 0xF) | (0x7 << 4) | (0xF << 8) | (((n >> 4) & 3) << 14); }
constexpr int kWaitLgkm0 = 0xF | (0x7 << 4) | (0x3 << 14);

template <int N>
__device__ __forceinline__ void pp_vm() {
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(N));
}

__device__ __forceinline__ void pp_wait(int p, bool has1, bool has2) {
  // groups issued in the 4 phases before this one and in this one (see the table above)
  if (has2) { pp_vm<10>(); return; }
  if (!has1) {
    if (p == 1) pp_vm<2>(); else pp_vm<0>();
    return;
  }
  switch (p) {
    case 1: pp_vm<10>(); break;
    case 2: pp_vm<8>(); break;
    case 3: pp_vm<6>(); break;
    default: pp_vm<4>(); break;
  }
}

// barrier A of a phase: every wave's counted wait is behind it; this wave's reads retire
__device__ __forceinline__ void pp_barrier_a() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
  __builtin_amdgcn_sched_barrier(0);
}

// barrier B: the MFMA cluster is issued; the next phase's LDS traffic stays below it
__device__ __forceinline__ void pp_barrier_b() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <bool kSetPrio = true>
__device__ __forceinline__ void pp_mfma(f32x4 (&acc)[4][2], const bf16x8 (&af)[4][2], const bf16x8 (&bf)[4][2]) {
  if (kSetPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi][kk], bf[ni][kk], acc[mi][ni], 0, 0, 0);
  if (kSetPrio) __builtin_amdgcn_s_setprio(0);
}

template <int kGroupM, bool kSetPrio = true, bool kNtStore = false>
__global__ void __launch_bounds__(kThreads2, 1)
gemm_bf16_tn_256pp_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                          int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 2 * kTile2];  // 128 KiB: [buf][A|B][256][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int nbn = N / kBN2, nbm = M / kBM2;
  const int nwg = nbm * nbn;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int in_group = kGroupM * nbn;
  const int first_m = (wgid / in_group) * kGroupM;
  const int gsize = nbm - first_m < kGroupM ? nbm - first_m : kGroupM;
  const int bm = first_m + (wgid % in_group) % gsize;
  const int bn = (wgid % in_group) / gsize;
  const int row_a = bm * kBM2, row_b = bn * kBN2;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / kBK;  // >= 2
  bf16x8 af[4][2], b0[4][2], b1[4][2];
  const int a_row = wr * 128, b_row = wc * 64;
  // prologue: K-tile 0 whole, then K-tile 1's Bf, A-M0, Bs (the groups steady state stages
  // at phases -3..-1); wait for tile 0, then row 1 falls one barrier behind
  GEMM2_STAGE_B(0, 0); GEMM2_STAGE_A(0, 0); GEMM2_STAGE_B(1, 0); GEMM2_STAGE_A(1, 0);
  GEMM2_STAGE_B(1, 1); GEMM2_STAGE_A(0, 1); GEMM2_STAGE_B(0, 1);
  wait_vm<6>();
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  read_frags(smem + kTile2, b_row, lane, b0, 2);  // Bf(0) = B-N0 of tile 0, "phase -1"

  // Each phase issues its DMA before its ds_reads (reads after the DMA need no wait; the
  // other order makes the compiler drain the reads before the DMA).
  auto tile = [&](int t, auto odd_tag) {
    constexpr bool odd = decltype(odd_tag)::value;
    const bool has1 = t + 1 < nk, has2 = t + 2 < nk;
    const uint16_t* As = smem + (odd ? 2 * kTile2 : 0);
    const uint16_t* Bs = As + kTile2;
    const uint16_t* Bn = smem + (odd ? 0 : 2 * kTile2) + kTile2;  // K-tile t+1's B
    // P1: stage A-M1(t+1); read A-M0; quadrant (M0, Bf)
    if (has1) GEMM2_STAGE_A(1, t + 1);
    read_frags(As, a_row, lane, af, 4);
    pp_wait(1, has1, has2);
    pp_barrier_a();
    if constexpr (odd) pp_mfma<kSetPrio>(acc[0][1], af, b1); else pp_mfma<kSetPrio>(acc[0][0], af, b0);
    pp_barrier_b();
    // P2: stage Bf(t+2) (same half as Bf(t)); read Bs(t); quadrant (M0, Bs)
    if (has2) { if constexpr (odd) GEMM2_STAGE_B(1, t + 2); else GEMM2_STAGE_B(0, t + 2); }
    if constexpr (odd) read_frags(Bs, b_row, lane, b0, 2); else read_frags(Bs, b_row + 32, lane, b1, 2);
    pp_wait(2, has1, has2);
    pp_barrier_a();
    if constexpr (odd) pp_mfma<kSetPrio>(acc[0][0], af, b0); else pp_mfma<kSetPrio>(acc[0][1], af, b1);
    pp_barrier_b();
    // P3: stage A-M0(t+2); read A-M1; quadrant (M1, Bs)
    if (has2) GEMM2_STAGE_A(0, t + 2);
    read_frags(As, a_row + 64, lane, af, 4);
    pp_wait(3, has1, has2);
    pp_barrier_a();
    if constexpr (odd) pp_mfma<kSetPrio>(acc[1][0], af, b0); else pp_mfma<kSetPrio>(acc[1][1], af, b1);
    pp_barrier_b();
    // P4: stage Bs(t+2); read Bf(t+1) into the B registers this phase does not use; (M1, Bf)
    if (has2) { if constexpr (odd) GEMM2_STAGE_B(0, t + 2); else GEMM2_STAGE_B(1, t + 2); }
    if (has1) {
      if constexpr (odd) read_frags(Bn, b_row, lane, b0, 2); else read_frags(Bn, b_row + 32, lane, b1, 2);
    }
    pp_wait(4, has1, has2);
    pp_barrier_a();
    if constexpr (odd) pp_mfma<kSetPrio>(acc[1][1], af, b1); else pp_mfma<kSetPrio>(acc[1][0], af, b0);
    pp_barrier_b();
  };
  for (int t = 0; t < nk; t += 2) {
    tile(t, std::false_type{});
    if (t + 1 < nk) tile(t + 1, std::true_type{});
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // close the stagger: row 1's last MFMA cluster is issued
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // no DMA in flight, every wave's reads retired: the 128 KiB are free

#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = wr * 128 + qm * 64 + mi * 16 + (lane >> 4) * 4 + j;
            const int col = wc * 64 + qn * 32 + ni * 16 + (lane & 15);
            __bf16 v = (__bf16)acc[qm][qn][mi][ni][j];
            smem[row * kBN2 + col] = *reinterpret_cast<uint16_t*>(&v);
          }
  __syncthreads();
#pragma unroll 4
  for (int p = 0; p < (kBM2 * kBN2 / 8) / kThreads2; ++p) {
    const int idx = p * kThreads2 + threadIdx.x;
    const int row = idx >> 5, chunk = idx & 31;
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4v;
    const u32x4v v = *reinterpret_cast<const u32x4v*>(smem + row * kBN2 + chunk * 8);
    u32x4v* dst = reinterpret_cast<u32x4v*>(C + size_t(row_a + row) * size_t(N) + row_b + chunk * 8);
    if constexpr (kNtStore) __builtin_nontemporal_store(v, dst); else *dst = v;
  }
}
#undef GEMM2_STAGE_A
#undef GEMM2_STAGE_B

// ---------------------------------------------------------------------------------------
// 4-wave form of the 256x256 tile (variant 9): one wave per SIMD, each wave owns a 128x128
// output block (8x8 MFMA tiles, 256 fp32 accumulators per lane, in AGPRs), so a K-tile
// costs every wave (128 + 128) rows of LDS reads instead of 8 waves x (128 + 64): a third
// fewer ds_reads per tile.  With no SIMD partner to ping-pong with, a wave hides its own
// reads: a K-tile is two K=32 slices, and while one slice's 64 MFMAs run (row mi of the
// 8x8 block = 8 MFMAs), the other slice's fragments are read into place: A row mi's new
// fragment into the register row mi just finished with, the B fragments into a second B
// set (A 32 + 2 x B 32 = 96 fragment VGPRs):
//   slice 0 (A0, B0) || read A1 in place, B1      (tile t, k 32-63)
//   lgkmcnt(0); vmcnt(0) [tile t+1 landed]; s_barrier [every wave is done with tile t]
//   stage tile t+2 (16 glds) into tile t's buffer
//   slice 1 (A1, B1) || read A0 in place, B0      (tile t+1, k 0-31)
// One barrier per K-tile; tile t+2's DMA has one K-tile of MFMA work to land.
// Same LDS image and swizzle as the kernels above; same K order, so bit-identical output.
// Measured (profiles/r03/gemm_variants.log): 1246-1286 TFLOP/s at 8192^3 against 1434-1441
// for the ping-pong variant 8 on the same boxes, with a third fewer LDS instructions, no
// bank conflicts and 7x fewer LDS-wait cycles (profiles/r03/gemm_pmc_4wave.txt); spreading
// the reads and the DMA between MFMAs and spacing accumulator chains 8 MFMAs apart moved
// it < 4 %.
// Kept as an A/B arm, not the default.  (The 16x16x32 form of this layout, 64 f32x4
// accumulators, makes hipcc shuttle accumulators between AGPRs and VGPRs every K-tile.)
// ---------------------------------------------------------------------------------------
constexpr int kThreads4 = 256;

// Stages one 256x64 operand K-tile: wave-instruction i covers rows [(i*4 + wave)*8, +8);
// the per-lane source differs between instructions only by i*32 rows (swz does not depend
// on i), so one address register pair serves all 8.
__device__ __forceinline__ void stage_tile_w4(const uint16_t* __restrict__ lane_src, size_t row32, uint16_t* lds_tile,
                                              int wave) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rblk = i * 4 + wave;
    __builtin_amdgcn_global_load_lds((gptr_t)(lane_src + size_t(i) * row32), (lds_ptr_t)(lds_tile + rblk * 8 * kBK),
                                     16, 0, 0);
  }
}

typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int kGroupM>
__global__ void __launch_bounds__(kThreads4, 1)
gemm_bf16_tn_256w4_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                          int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * 2 * kTile2];  // 128 KiB: [buf][A|B][256][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int nbn = N / kBN2, nbm = M / kBM2;
  const int nwg = nbm * nbn;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int in_group = kGroupM * nbn;
  const int first_m = (wgid / in_group) * kGroupM;
  const int gsize = nbm - first_m < kGroupM ? nbm - first_m : kGroupM;
  const int bm = first_m + (wgid % in_group) % gsize;
  const int bn = (wgid % in_group) / gsize;
  const int row_a = bm * kBM2, row_b = bn * kBN2;

  // 128x128 per wave as 4x4 tiles of v_mfma_f32_32x32x16_bf16: 16 accumulators of 16 fp32
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = K / kBK;  // >= 2
  const int srow = wave * 8 + (lane >> 3);
  const int schunk = swz(srow, lane & 7);
  const uint16_t* a_src = A + size_t(row_a + srow) * size_t(K) + schunk * 8;
  const uint16_t* b_src = B + size_t(row_b + srow) * size_t(K) + schunk * 8;
  const size_t row32 = size_t(32) * size_t(K);
  // 32x32x16 operand fragment: lane l holds row l%32, K elements (l/32)*8..+8 of a 16-deep
  // step; fragment (tile i, step k16) of slice kk reads chunk kk*4 + k16*2 + l/32 of row
  // base + i*32 + l%32, and the swizzle ((row>>1)&7) depends only on l%32: one offset per
  // (operand, kk, k16), tiles as i*32 rows of immediate offset
  const int l31 = lane & 31;
  const int rsw = (l31 >> 1) & 7;
  int a_off[2][2], b_off[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int k16 = 0; k16 < 2; ++k16) {
      const int c = ((kk * 4 + k16 * 2 + (lane >> 5)) ^ rsw) * 8;
      a_off[kk][k16] = (wm * 128 + l31) * kBK + c;
      b_off[kk][k16] = kTile2 + (wn * 128 + l31) * kBK + c;
    }

  bf16x8 a[4][2], b0[4][2], b1[4][2];
  stage_tile_w4(a_src, row32, smem, wave);
  stage_tile_w4(b_src, row32, smem + kTile2, wave);
  stage_tile_w4(a_src + kBK, row32, smem + 2 * kTile2, wave);
  stage_tile_w4(b_src + kBK, row32, smem + 3 * kTile2, wave);
  pp_vm<16>();  // K-tile 0 landed (tile 1's 16 loads may be in flight)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k16 = 0; k16 < 2; ++k16) {
      a[i][k16] = *reinterpret_cast<const bf16x8*>(smem + a_off[0][k16] + i * 32 * kBK);
      b0[i][k16] = *reinterpret_cast<const bf16x8*>(smem + b_off[0][k16] + i * 32 * kBK);
    }

  // two rows of a slice (16 MFMAs): both rows' first 16-deep step, then both rows' second,
  // so the two MFMAs that chain through one accumulator are 8 MFMAs apart
  auto rows = [&](int m0, const bf16x8 (&bb)[4][2]) {
#pragma unroll
    for (int k16 = 0; k16 < 2; ++k16)
#pragma unroll
      for (int m = m0; m < m0 + 2; ++m)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[m][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m][k16], bb[ni][k16], acc[m][ni], 0, 0, 0);
  };
  // one fragment (both 16-deep steps of a slice) of B tile n / A tile m: 2 ds_read_b128
  auto rb = [&](const uint16_t* buf, int kk, int n, bf16x8 (&bb)[4][2]) {
#pragma unroll
    for (int k16 = 0; k16 < 2; ++k16)
      bb[n][k16] = *reinterpret_cast<const bf16x8*>(buf + b_off[kk][k16] + n * 32 * kBK);
  };
  auto ra = [&](const uint16_t* buf, int kk, int m) {
#pragma unroll
    for (int k16 = 0; k16 < 2; ++k16)
      a[m][k16] = *reinterpret_cast<const bf16x8*>(buf + a_off[kk][k16] + m * 32 * kBK);
  };
  // Per slice, the next slice's B fragments are read first (every row of the next slice
  // needs all of them) and its A fragments after, each into rows already finished (A rows
  // 2-3 only once their MFMAs are issued), spread between the MFMAs (bunched, the 4 waves'
  // reads fill the LDS queue together and stall MFMA issue).  The barrier sits after rows
  // 0-1 of slice 1: by then every read of tile t has long been issued.
#define W4_SPREAD(per, n)                                 \
  for (int i_ = 0; i_ < (n); ++i_) {                      \
    __builtin_amdgcn_sched_group_barrier(0x008, per, 0);  \
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    \
  }
  for (int t = 0; t < nk; ++t) {
    const uint16_t* cur = smem + (t & 1) * 2 * kTile2;
    const uint16_t* nxt = smem + ((t + 1) & 1) * 2 * kTile2;
    // slice 0: (a = k 0-31, b0); read k 32-63 of tile t: b1, then a
    rows(0, b0);
#pragma unroll
    for (int n = 0; n < 4; ++n) rb(cur, 1, n, b1);
    W4_SPREAD(2, 8)
    rows(2, b0); ra(cur, 1, 0); ra(cur, 1, 1); ra(cur, 1, 2); ra(cur, 1, 3);
    W4_SPREAD(4, 4)
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
    // slice 1: (a = k 32-63, b1)
    rows(0, b1);
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // this wave is done reading tile t
    pp_vm<0>();                              // tile t+1 landed (the only DMA in flight)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // Tile t+2's 16 DMA instructions go out one per MFMA of the last two rows (a burst of
    // them stalls the wave at issue).  Past the end the last tile is restaged into a buffer
    // nothing reads any more (in bounds, no branch in the loop).
    {
      uint16_t* dst = smem + (t & 1) * 2 * kTile2;
      const int ts = t + 2 < nk ? t + 2 : nk - 1;
      stage_tile_w4(a_src + ts * kBK, row32, dst, wave);
      stage_tile_w4(b_src + ts * kBK, row32, dst + kTile2, wave);
    }
    // read k 0-31 of tile t+1 (after the last tile: the other buffer's stale rows, in
    // bounds and unused)
    rows(2, b1);
#pragma unroll
    for (int n = 0; n < 4; ++n) rb(nxt, 0, n, b0);
    ra(nxt, 0, 0); ra(nxt, 0, 1);
    for (int i_ = 0; i_ < 12; ++i_) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    for (int i_ = 0; i_ < 4; ++i_) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
    }
    ra(nxt, 0, 2); ra(nxt, 0, 3);
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
  }
#undef W4_SPREAD
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's reads retired, no DMA in flight: the 128 KiB are free

  // C/D map of 32x32x16: col = lane%32, row = (e/4)*8 + (lane/32)*4 + e%4
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wm * 128 + mi * 32 + (e >> 2) * 8 + (lane >> 5) * 4 + (e & 3);
        const int col = wn * 128 + ni * 32 + l31;
        __bf16 v = (__bf16)acc[mi][ni][e];
        smem[row * kBN2 + col] = *reinterpret_cast<uint16_t*>(&v);
      }
  __syncthreads();
#pragma unroll 4
  for (int p = 0; p < (kBM2 * kBN2 / 8) / kThreads4; ++p) {  // 32 passes of 256 x 16 B
    const int idx = p * kThreads4 + threadIdx.x;
    const int row = idx >> 5, chunk = idx & 31;
    const uint4 v = *reinterpret_cast<const uint4*>(smem + row * kBN2 + chunk * 8);
    *reinterpret_cast<uint4*>(C + size_t(row_a + row) * size_t(N) + row_b + chunk * 8) = v;
  }
}

bool gemm_shape_ok(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && M % kBM == 0 && N % kBN == 0 && K % kBK == 0;
}

bool gemm256_shape_ok(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 2 * kBK && M % kBM2 == 0 && N % kBN2 == 0 && K % kBK == 0;
}

// variant: 0 = auto (256x256 kernel when the shape allows it), 1 = 128x128, 2 = 256x256
// with row-major tile order per XCD, 3 / 4 = 256x256 with 4 / 8 row panels per group,
// 5-7 priority / read-schedule forms, 8 = ping-pong phases (two barriers per phase),
// 9 = 4 waves of 128x128.
// The kernel a launch with `variant` runs (0 = auto), or -1 if the shape does not fit it.
// auto = 8 (256x256 ping-pong) when M%256 == N%256 == 0 and K >= 128, else 1 (128x128):
// 8 runs at 1436-1459 vs 1361 TFLOP/s for 7 at 8192^3 (1319-1365 vs 1190 at 4096^3;
// profiles/r03/gemm_variants.log).  7: 8-row tile groups (1355 vs 1265 TFLOP/s row-major),
// per-cluster setprio (5 / 6 without it / static form: -5 %), balanced snake-B reads
// (+0.3-1 % over 4).  9: 4 waves of 128x128 (1246-1274).
int resolve_gemm_variant(int M, int N, int K, int variant) {
  if (!gemm_shape_ok(M, N, K) || variant < 0 || variant > 9) return -1;
  if (variant == 0) return gemm256_shape_ok(M, N, K) ? 8 : 1;
  if (variant >= 2 && !gemm256_shape_ok(M, N, K)) return -1;
  return variant;
}

hipError_t launch_gemm_bf16_tn(const void* A, const void* B, void* C, int M, int N, int K, hipStream_t stream,
                               int variant) {
  variant = resolve_gemm_variant(M, N, K, variant);
  if (variant < 0) return hipErrorInvalidValue;
  if (variant >= 2) {
    if (variant == 9) {
      hipLaunchKernelGGL(gemm_bf16_tn_256w4_kernel<8>, dim3((M / kBM2) * (N / kBN2)), dim3(kThreads4), 0, stream,
                         static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C),
                         M, N, K);
      return hipGetLastError();
    }
    // 4-row tile groups: 1456 vs 1444 (8 rows), 1398 (16) at 8192^3, 1355 vs 1318 at 4096^3;
    // no s_setprio around the MFMA clusters (the wave rows alternate by barrier anyway):
    // +2.2 % at 4096^3, +0.2 % at 8192^3 over raising it; C written with non-temporal stores
    // (written once, never read here): +1.7 % / +1.3 % at 4096^3 / 8192^3
    if (variant == 8) {
      auto k8 = gemm_bf16_tn_256pp_kernel<4, false, true>;
      hipLaunchKernelGGL(k8, dim3((M / kBM2) * (N / kBN2)), dim3(kThreads2), 0, stream,
                         static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C),
                         M, N, K);
      return hipGetLastError();
    }
    auto k = variant == 2   ? gemm_bf16_tn_256_kernel<1, 0>
             : variant == 3 ? gemm_bf16_tn_256_kernel<4, 0>
             : variant == 4 ? gemm_bf16_tn_256_kernel<8, 0>
             : variant == 5 ? gemm_bf16_tn_256_kernel<8, 1>
             : variant == 6 ? gemm_bf16_tn_256_kernel<8, 2>
                            : gemm_bf16_tn_256_kernel<8, 0, true>;
    hipLaunchKernelGGL(k, dim3((M / kBM2) * (N / kBN2)), dim3(kThreads2), 0, stream,
                       static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M,
                       N, K);
  } else {
    hipLaunchKernelGGL(gemm_bf16_tn_kernel, dim3((M / kBM) * (N / kBN)), dim3(kThreads), 0, stream,
                       static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M,
                       N, K);
  }
  return hipGetLastError();
}

hipError_t launch_fill_bf16(void* p, size_t n, uint32_t seed, hipStream_t stream) {
  hipLaunchKernelGGL(fill_bf16_kernel, dim3(1024), dim3(256), 0, stream, static_cast<uint16_t*>(p), n, seed);
  return hipGetLastError();
}

}  // namespace gpuexp
