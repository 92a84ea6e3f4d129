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

}  // namespace gpuexp
