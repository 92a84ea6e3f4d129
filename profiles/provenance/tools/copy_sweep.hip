// Sweep of the PMC calibration stream-copy shape on one MI355X (1 GiB, hipEvent timing):
// load/store cache policy x vectors in flight per lane x grid size.  Picks the shape
// kernels/probe_device.h uses.  Build: hipcc -O3 --offload-arch=gfx950 copy_sweep.hip -o copy_sweep
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int kUnroll, bool kNtLoad, bool kNtStore>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (kUnroll - 1) * stride < n; i += kUnroll * stride) {
    u32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) v[u] = kNtLoad ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (kNtStore)
        __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else
        dst[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

// Contiguous chunk per workgroup (instead of a grid-wide stride): each workgroup streams its
// own [b*chunk, (b+1)*chunk) range, kUnroll vectors in flight per lane.
template <int kUnroll>
__global__ __launch_bounds__(256) void chunk_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t chunk = (n + gridDim.x - 1) / gridDim.x;
  const size_t beg = size_t(blockIdx.x) * chunk;
  const size_t end = beg + chunk < n ? beg + chunk : n;
  size_t i = beg + threadIdx.x;
  for (; i + (kUnroll - 1) * 256 < end; i += kUnroll * 256) {
    u32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) v[u] = __builtin_nontemporal_load(src + i + u * 256);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) __builtin_nontemporal_store(v[u], dst + i + u * 256);
  }
  for (; i < end; i += 256) dst[i] = src[i];
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

template <typename K>
void run_k(const char* name, K kern, const u32x4* s, u32x4* d, size_t n) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int blocks : {256, 512, 768, 1024, 1536, 2048, 4096, 8192}) {
    for (int w = 0; w < 3; ++w) kern<<<blocks, 256>>>(s, d, n);
    CK(hipEventRecord(a));
    const int iters = 20;
    for (int it = 0; it < iters; ++it) kern<<<blocks, 256>>>(s, d, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double bytes = 2.0 * double(n) * 16 * iters;
    std::printf("%-16s blocks %6d  %.3f ms/copy  %.2f TB/s (read+write)\n", name, blocks, ms / iters,
                bytes / (ms * 1e-3) / 1e12);
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

template <int U, bool NL, bool NS>
void run(const char* name, const u32x4* s, u32x4* d, size_t n) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int blocks : {1024, 2048, 4096, 8192, 16384, 32768}) {
    for (int w = 0; w < 3; ++w) copy_kernel<U, NL, NS><<<blocks, 256>>>(s, d, n);
    CK(hipEventRecord(a));
    const int iters = 20;
    for (int it = 0; it < iters; ++it) copy_kernel<U, NL, NS><<<blocks, 256>>>(s, d, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double bytes = 2.0 * double(n) * 16 * iters;
    std::printf("%-16s blocks %6d  %.3f ms/copy  %.2f TB/s (read+write)\n", name, blocks, ms / iters,
                bytes / (ms * 1e-3) / 1e12);
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main() {
  const size_t bytes = size_t(1) << 30;
  const size_t n = bytes / 16;
  u32x4 *s = nullptr, *d = nullptr;
  CK(hipMalloc(&s, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(s, 1, bytes));
  CK(hipMemset(d, 0, bytes));
  run_k("chunk u4 nt", chunk_kernel<4>, s, d, n);
  run_k("chunk u8 nt", chunk_kernel<8>, s, d, n);
  run_k("chunk u16 nt", chunk_kernel<16>, s, d, n);
  run_k("stride u1 plain", copy_kernel<1, false, false>, s, d, n);
  run_k("stride u4 nt", copy_kernel<4, true, true>, s, d, n);
  CK(hipDeviceSynchronize());
  CK(hipFree(s));
  CK(hipFree(d));
  return 0;
}
