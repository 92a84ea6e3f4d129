// Device bodies of the PMC calibration workloads, shared by the HIP-launched kernels
// (probe_kernels.hip, bound in _gpuexp_kernels) and the raw-AQL code object the aqlprofile
// plugin dispatches on its own PMC queue (calib_hsaco.hip -> gpuexp_calib.hsaco).
//
// No blockDim/gridDim: a raw AQL dispatch fills no implicit kernel arguments, so the block
// size is the compile-time kProbeBlock and the grid's thread count is an explicit argument.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels/probe_args.h"

namespace gpuexp {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// dst[i] = src[i] over n 16-byte vectors: every byte read once and written once, with
// nontemporal hints so the copy streams through L2 instead of parking in it.  Grid-stride
// (`stride` = threads in the grid) with 4 vectors in flight per lane.
__device__ inline void stream_copy_body(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n,
                                        size_t stride) {
  size_t i = size_t(blockIdx.x) * kProbeBlock + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    u32x4 a = __builtin_nontemporal_load(src + i);
    u32x4 b = __builtin_nontemporal_load(src + i + stride);
    u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    u32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + stride);
    __builtin_nontemporal_store(c, dst + i + 2 * stride);
    __builtin_nontemporal_store(d, dst + i + 3 * stride);
  }
  for (; i < n; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// Every lane reads `iters` dwords from LDS (ds_read_b32: lane groups {0-31} {32-63}, bank =
// word mod 32).  stride 1: the 32 lanes of a group hit 32 distinct banks (conflict-free);
// stride 32: all of them hit one bank at 32 distinct addresses (32-way: 31 extra cycles per
// group).  The sum goes to global memory so nothing is optimised away.
__device__ inline void lds_probe_body(float* out, int iters, int stride) {
  __shared__ float table[kLdsWords];
  for (int w = threadIdx.x; w < kLdsWords; w += kProbeBlock) table[w] = float(w & 7);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  float acc = 0.f;
  const int base = lane * stride;
#pragma unroll 8
  for (int i = 0; i < iters; ++i) acc += table[(base + i) & (kLdsWords - 1)];
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

}  // namespace gpuexp
