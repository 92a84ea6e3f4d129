// Host-visible launch parameters of the PMC calibration workloads (probe_device.h): the
// argument structs are passed by value as the kernels' whole kernarg segment, by HIP
// launches and by raw AQL dispatches from the aqlprofile plugin (compiled by g++) alike.
#pragma once

#include <cstdint>

namespace gpuexp {

constexpr int kProbeBlock = 256;  // threads per block: 4 waves
constexpr int kLdsWords = 4096;   // 16 KiB LDS table

struct CalibCopyArgs {
  const void* src;  // 16-byte vectors
  void* dst;
  uint64_t n;       // 16-byte vectors to copy
  uint64_t blocks;  // workgroups in the grid (each copies one contiguous chunk)
};

struct CalibLdsArgs {
  float* out;  // >= blocks floats
  int iters;
  int stride;  // 1 (conflict-free) or 32 (32-way bank conflicts)
};

// MFMA duty-cycle workload (mfma_duty_body): every wave alternates `on_ticks` of
// back-to-back v_mfma_f32_32x32x16_bf16 with `period_ticks - on_ticks` of s_sleep, for
// `total_ticks`, on the 100 MHz s_memrealtime clock.  Launched with 2 waves per SIMD the
// matrix cores are busy for on/period of the wall time while the kernel stays resident.
struct CalibMfmaArgs {
  float* out;             // >= blocks floats (sink, keeps the MFMAs live)
  uint64_t* mfma_count;   // >= blocks * 4 counters: MFMAs issued per wave
  uint64_t period_ticks;  // s_memrealtime ticks (10 ns) per on/off period
  uint64_t on_ticks;      // MFMA phase of each period (<= period_ticks)
  uint64_t total_ticks;   // run length
  uint32_t xcc_mask;      // XCCs (HW_REG_XCC_ID bits) whose blocks run; 0 = every XCC
};
constexpr int kMfmaPerCheck = 32;  // MFMAs between two clock reads (32 x 32 cycles)

// Fixed MFMA work for the FLOP-counter calibration (mfma_count_body): every wave issues
// exactly 4 x iters v_mfma_f32_32x32x16 of one operand type, 32768 FLOPs each.
struct CalibMfmaCountArgs {
  float* out;      // >= blocks floats (sink, keeps the MFMAs live)
  uint32_t iters;
  uint32_t type;   // 0 bf16 (v_mfma_f32_32x32x16_bf16), 1 fp8 (v_mfma_f32_32x32x16_fp8_fp8)
};
constexpr int kMfmaCountChains = 4;
constexpr double kMfma32x32x16Flops = 2.0 * 32 * 32 * 16;

}  // namespace gpuexp
