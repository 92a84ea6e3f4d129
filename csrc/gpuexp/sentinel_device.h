// Device code of the sentinel (sentinel_common.h has the layout), shared by the HIP
// plugin's __global__ kernels (sentinel.hip) and the HSACO that the aqlprofile plugin
// dispatches as raw AQL (sentinel_hsaco.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "gpuexp/sentinel_common.h"

namespace gpuexp {

// Writes the pointer-chase links in place (one lane per hop): a kernel, not a copy, so no
// blit/copy queue (each with its own context save area) is ever created for it.
__device__ __forceinline__ void sentinel_init_chase_body(uint32_t* __restrict__ chase, int hops) {
  const int h = int(threadIdx.x);
  if (h < hops) chase[size_t(h) * kChaseStride] = uint32_t((h + 1) % hops);
}

// ring[run_slot * kSentinelMaxWaves + blockIdx.x]
__device__ __forceinline__ void sentinel_body(SentinelSlot* __restrict__ ring, uint32_t slot, uint64_t seq, int spin,
                                              const uint32_t* chase, int hops) {
  // Highest wave priority for the few microseconds this runs: next to workload waves that
  // issue MFMAs back-to-back for seconds (a persistent GEMM / attention kernel), a
  // priority-0 sentinel wave lost every VALU issue slot and never finished, and the PMC read
  // packets queued behind its dispatch stalled with it (measured on MI355X with the MFMA
  // duty kernel at 100 %: tools/mfma_calibration.py, profiles/r03/mfma_calibration.txt).
  __builtin_amdgcn_s_setprio(3);
  if (threadIdx.x != 0) return;
  uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
  uint64_t mt0 = __builtin_amdgcn_s_memtime();
  // Dependent integer chain: the compiler cannot shorten it; its length only sets the
  // timing window (~spin*8 shader cycles).
  uint32_t x = uint32_t(seq) | 1u;
  for (int i = 0; i < spin; ++i) {
    x = x * 1664525u + 1013904223u;
    asm volatile("" : "+v"(x));
  }
  uint64_t mt1 = __builtin_amdgcn_s_memtime();
  uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
  // HBM load latency under whatever the GPU is doing now: a chain of dependent loads.
  uint32_t idx = 0;
  uint64_t rt2 = __builtin_amdgcn_s_memrealtime();
  for (int h = 0; h < hops; ++h) idx = reinterpret_cast<const volatile uint32_t*>(chase)[size_t(idx) * kChaseStride];
  uint64_t rt3 = __builtin_amdgcn_s_memrealtime();
  uint32_t xcc, hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  SentinelSlot* s = ring + size_t(slot) * kSentinelMaxWaves + blockIdx.x;
  s->rt0 = rt0;
  s->rt1 = rt1;
  s->mt0 = mt0;
  s->mt1 = mt1;
  s->xcc_id = xcc;
  s->hw_id = hwid ^ (x & 0u);  // keep x live without changing hw_id
  s->chase_rt = rt3 - rt2;
  s->hops = uint32_t(hops);
  s->chase_end = idx;
  __atomic_thread_fence(__ATOMIC_RELEASE);  // orders the payload before seq (system scope below)
  __hip_atomic_store(&s->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace gpuexp
