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

// vgpr:  1 wave per block claiming 400 of a lane's 512 registers (200 arch VGPRs + 200
//        AGPRs of the unified file; more would make the compiler spill): one wave per SIMD,
//        4 per CU, while 28 wave slots stay free and no LDS is used -> the limiter is VGPRs.
//        The clobbers size the kernel descriptor; no register holds a value across them.
__global__ __launch_bounds__(64) void occupancy_hog_vgpr_kernel(float* out, uint64_t ticks) {
  asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183", "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199", "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63", "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79", "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95", "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111", "a112", "a113", "a114", "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127", "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143", "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159", "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", "a172", "a173", "a174", "a175", "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191", "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199");
  hold_for(ticks);
  if (threadIdx.x == 0) out[blockIdx.x] = float(blockIdx.x);
}

// sgpr:  1 wave per block declaring 102 SGPRs (+ VCC): fewer such waves fit a SIMD's SGPR file
//        than it has wave slots -> the limiter is SGPRs (with wave slots close behind).
__global__ __launch_bounds__(64) void occupancy_hog_sgpr_kernel(float* out, uint64_t ticks) {
  asm volatile("" ::: "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "s8", "s9", "s10", "s11", "s12", "s13", "s14", "s15", "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s32", "s33", "s34", "s35", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "s98", "s99", "s100", "s101", "vcc");
  hold_for(ticks);
  if (threadIdx.x == 0) out[blockIdx.x] = float(blockIdx.x);
}

}  // namespace

hipError_t launch_occupancy_hog(int kind, float* out, int blocks, double seconds, hipStream_t stream) {
  if (!out || blocks < 1 || blocks > (1 << 20) || !(seconds > 0) || seconds > 10 || kind < 0 || kind > 3)
    return hipErrorInvalidValue;
  const uint64_t ticks = uint64_t(seconds * 1e8);
  if (kind == 0) hipLaunchKernelGGL(occupancy_hog_lds_kernel, dim3(blocks), dim3(64), 0, stream, out, ticks);
  else if (kind == 1) hipLaunchKernelGGL(occupancy_hog_waves_kernel, dim3(blocks), dim3(512), 0, stream, out, ticks);
  else if (kind == 2) hipLaunchKernelGGL(occupancy_hog_vgpr_kernel, dim3(blocks), dim3(64), 0, stream, out, ticks);
  else hipLaunchKernelGGL(occupancy_hog_sgpr_kernel, dim3(blocks), dim3(64), 0, stream, out, ticks);
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
