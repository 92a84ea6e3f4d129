// Counter set + derivations shared by the two device-counter plugins
// (_gpuexp_aqlpmc.so: direct aqlprofile PM4 on an exporter-owned queue;
//  _gpuexp_rocprof.so: rocprofiler-sdk device counting service).
//
// One pass within the gfx950 per-block slot limits (MI355X_MICROARCH.md "rocprofv3 PMC
// slots": SQ 8, TCC 4, GRBM 2):
//   SQ   SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT
//   GRBM GRBM_GUI_ACTIVE GRBM_COUNT
//   TCC  TCC_BUBBLE TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_EA0_WRREQ_64B
// Derived values follow the gfx950 formulas of /opt/rocm/share/rocprofiler-sdk/counter_defs.yaml
// (MfmaUtil, FETCH_SIZE, WRITE_SIZE, LDS utilisation / bank-conflict ratio).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>

namespace gpuexp_ctr {

enum Ctr {
  kMfma = 0,
  kSqBusy,
  kWaves,
  kLdsActive,
  kLdsConflict,
  kGuiActive,
  kGrbmCount,
  kTccBubble,
  kRdReq,
  kWrReq,
  kWrReq64,
  kNumCtr
};

inline const char* name(int c) {
  static const char* kNames[kNumCtr] = {"SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES",  "SQ_WAVES",
                                        "SQ_LDS_IDX_ACTIVE",        "SQ_LDS_BANK_CONFLICT",
                                        "GRBM_GUI_ACTIVE",          "GRBM_COUNT",      "TCC_BUBBLE",
                                        "TCC_EA0_RDREQ",            "TCC_EA0_WRREQ",   "TCC_EA0_WRREQ_64B"};
  return kNames[c];
}

// GRBM counters are per-XCC copies of one clock: reduce with max; everything else sums.
inline bool use_max(int c) { return c == kGuiActive || c == kGrbmCount; }

// Number of derived outputs (the CounterSource ABI: gpuexp_rp_sample fills 8 doubles).
constexpr int kNumOut = 8;

struct Derived {
  uint32_t simd = 0, cu = 0;
  int scope = -1;  // -1 unknown, 0 wave/EA counters VMID-filtered to this process, 1 device-wide
  double latest[kNumOut] = {};
  bool valid = false;
  uint64_t windows = 0;
};

// d: per-counter deltas over `wall` seconds; inst: instances that were reduced per counter.
inline void derive(Derived& a, const double* d, const int* inst, double wall) {
  const double nan = std::nan("");
  const double gui = d[kGuiActive];
  // Scope detection.  As a non-root client (perf_event_paranoid=3 on the test pool) the
  // wave-level SQ counters and the TCC EA requests are VMID-filtered to THIS process,
  // while SQ_VALU_MFMA_BUSY_CYCLES and GRBM are chip-global (measured against rocprofv3
  // dispatch counts: profiles/r01/pmc_gemm_dispatch.txt).  A busy GPU on which the
  // exporter sees almost no waves means the filtered set must not be exported as device
  // totals.
  if (d[kGrbmCount] > 0 && gui / d[kGrbmCount] > 0.5 && d[kMfma] > 0) a.scope = d[kWaves] / wall < 1000.0 ? 0 : 1;
  double* out = a.latest;
  out[0] = gui > 0 && a.simd ? 100.0 * d[kMfma] / (gui * a.simd) : nan;             // MfmaUtil
  const double se = inst[kSqBusy] > 0 ? inst[kSqBusy] : 1;                           // one per SE
  out[1] = gui > 0 ? std::min(100.0, 100.0 * d[kSqBusy] / (gui * se)) : nan;
  out[2] = d[kGrbmCount] > 0 ? 100.0 * gui / d[kGrbmCount] : nan;                    // GPU busy
  out[3] = d[kWaves] / wall;                                                         // waves/s
  out[4] = gui > 0 && a.cu ? 100.0 * d[kLdsActive] / (gui * a.cu) : nan;            // LDS util
  out[5] = d[kLdsActive] > 0 ? 100.0 * d[kLdsConflict] / d[kLdsActive] : 0.0;       // bank conflicts
  out[6] = (d[kTccBubble] * 128.0 + (d[kRdReq] - d[kTccBubble]) * 64.0) / wall;    // FETCH_SIZE B/s
  out[7] = ((d[kWrReq] - d[kWrReq64]) * 32.0 + d[kWrReq64] * 64.0) / wall;         // WRITE_SIZE B/s
  a.valid = true;
  a.windows += 1;
}

}  // namespace gpuexp_ctr
