// Calibration kernels for the device PMC families, launched through HIP (bound in
// _gpuexp_kernels as stream_copy / lds_probe): workloads whose HBM bytes, LDS bank
// conflicts and wave counts are known in advance.  The same device code is dispatched as
// raw AQL on the PMC queue by the aqlprofile plugin (calib_hsaco.hip), where the
// exporter's own counters see it (tools/pmc_validate.py).
#include "kernels/probe_device.h"

namespace gpuexp {

namespace {

__global__ __launch_bounds__(kProbeBlock) void stream_copy_kernel(CalibCopyArgs a) {
  stream_copy_body(static_cast<const u32x4*>(a.src), static_cast<u32x4*>(a.dst), a.n, a.blocks);
}

__global__ __launch_bounds__(kProbeBlock) void lds_probe_kernel(CalibLdsArgs a) {
  lds_probe_body(a.out, a.iters, a.stride);
}

__global__ __launch_bounds__(kProbeBlock) void mfma_duty_kernel(CalibMfmaArgs a) { mfma_duty_body(a); }

// Occupancy-limiter calibration (tools/probe_spi_scope.py, amd_gpu_occupancy_limiter_percent):
// blocks that only hold resources for `ticks` of the 100 MHz s_memrealtime clock, launched in
// more generations than fit, so ready waves queue in the dispatcher for a known reason.
//   lds:   1 wave per block + 64 KiB of LDS: LDS (160 KiB per CU) admits 2 blocks = 2 waves per
//          CU while 30 wave slots stay free -> the limiter is LDS
//   waves: 8 waves per block, no LDS, few VGPRs: 4 blocks fill a CU's 32 wave slots -> the
//          limiter is wave slots
constexpr int kHogLdsBytes = 64 * 1024;

__device__ inline void hold_for(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ __launch_bounds__(64) void occupancy_hog_lds_kernel(float* out, uint64_t ticks) {
  __shared__ float lds[kHogLdsBytes / sizeof(float)];
  const int t = int(threadIdx.x);
  for (int i = t; i < kHogLdsBytes / int(sizeof(float)); i += 64) lds[i] = float(i + blockIdx.x);
  __syncthreads();
  hold_for(ticks);
  // the allocation must be live: one value read back per block
  if (t == 0) out[blockIdx.x] = lds[(blockIdx.x * 97) % (kHogLdsBytes / sizeof(float))];
}

__global__ __launch_bounds__(512) void occupancy_hog_waves_kernel(float* out, uint64_t ticks) {
  hold_for(ticks);
  if (threadIdx.x == 0) out[blockIdx.x] = float(blockIdx.x);
}

}  // namespace

hipError_t launch_occupancy_hog(int kind, float* out, int blocks, double seconds, hipStream_t stream) {
  if (!out || blocks < 1 || blocks > (1 << 20) || !(seconds > 0) || seconds > 10 || (kind != 0 && kind != 1))
    return hipErrorInvalidValue;
  const uint64_t ticks = uint64_t(seconds * 1e8);
  if (kind == 0) hipLaunchKernelGGL(occupancy_hog_lds_kernel, dim3(blocks), dim3(64), 0, stream, out, ticks);
  else hipLaunchKernelGGL(occupancy_hog_waves_kernel, dim3(blocks), dim3(512), 0, stream, out, ticks);
  return hipGetLastError();
}

// Host checks (the kernel's loop relies on them): period > 0, on <= period, a bounded run.
hipError_t launch_mfma_duty(float* out, uint64_t* counts, int blocks, double duty, double period_s, double seconds,
                            uint32_t xcc_mask, hipStream_t stream) {
  if (!out || !counts || blocks < 1 || blocks > (1 << 16) || !(duty >= 0 && duty <= 1) || !(period_s >= 1e-5) ||
      period_s > 1.0 || !(seconds > 0) || seconds > 60)
    return hipErrorInvalidValue;
  const uint64_t period = uint64_t(period_s * 1e8 + 0.5);  // 100 MHz s_memrealtime ticks
  CalibMfmaArgs a{out, counts, period, uint64_t(double(period) * duty + 0.5), uint64_t(seconds * 1e8),
                  xcc_mask};
  if (a.on_ticks > a.period_ticks) a.on_ticks = a.period_ticks;
  hipLaunchKernelGGL(mfma_duty_kernel, dim3(blocks), dim3(kProbeBlock), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_stream_copy(const void* src, void* dst, size_t bytes, int blocks, hipStream_t stream) {
  if (bytes % 16) return hipErrorInvalidValue;
  CalibCopyArgs a{src, dst, bytes / 16, uint64_t(blocks)};
  hipLaunchKernelGGL(stream_copy_kernel, dim3(blocks), dim3(kProbeBlock), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_lds_probe(float* out, int blocks, int iters, int stride, hipStream_t stream) {
  CalibLdsArgs a{out, iters, stride};
  hipLaunchKernelGGL(lds_probe_kernel, dim3(blocks), dim3(kProbeBlock), 0, stream, a);
  return hipGetLastError();
}

}  // namespace gpuexp
