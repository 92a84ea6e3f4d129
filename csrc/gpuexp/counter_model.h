// Counter set + derivations shared by the two device-counter plugins
// (_gpuexp_aqlpmc.so: direct aqlprofile PM4 on an exporter-owned queue;
//  _gpuexp_rocprof.so: rocprofiler-sdk device counting service).
//
// One pass within the gfx950 per-block slot limits (MI355X_MICROARCH.md "rocprofv3 PMC
// slots": SQ 8, TCC 4, GRBM 2):
//   SQ   SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT
//        SQ_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8
//   GRBM GRBM_GUI_ACTIVE GRBM_COUNT
//   TCC  TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B TCC_EA0_RDREQ_GMI_32B
//        TCC_EA0_WRREQ_WRITE_GMI_32B
//   SPI  SPI_RA_RES_STALL_CSN SPI_RA_LDS_CU_FULL_CSN SPI_RA_WAVE_SIMD_FULL_CSN
//        SPI_RA_VGPR_SIMD_FULL_CSN (the dispatcher's resource allocator: what keeps a compute
//        wave that is ready to launch from getting a CU -- LDS, wave slots, VGPRs)
// MFMA / LDS derivations follow the gfx950 formulas of
// /opt/rocm/share/rocprofiler-sdk/counter_defs.yaml (MfmaUtil, LDS utilisation /
// bank-conflict ratio).  HBM bytes do NOT use its gfx950 FETCH_SIZE: that formula weighs
// TCC_BUBBLE as the 128-byte read count, and on MI355X TCC_BUBBLE stays 0 while every
// TCC_EA0_RDREQ of a streaming copy is a 128-byte line (measured: FETCH_SIZE = 0.497x the
// bytes a copy moves, profiles/r02/pmc_calibration.txt).  The DRAM-sector counters count
// 32-byte sectors of requests that reach the memory controller (a 64-byte request counts 2),
// so x 32 B they are HBM bytes whatever the request sizes, with traffic to memory behind GMI
// (peer GPUs) and IO (host) in counters of their own.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace gpuexp_ctr {

enum Ctr {
  kMfma = 0,
  kSqBusy,
  kWaves,
  kLdsActive,
  kLdsConflict,
  kGuiActive,
  kGrbmCount,
  kDramRd32,
  kDramWr32,
  kGmiRd32,
  kGmiWr32,
  kSqCycles,
  kMopsBf16,  // MFMA work in units of 512 FLOPs (counter_defs.yaml: MFMA FLOPs = MOPS x 512)
  kMopsF8,
  kSpiResStall,  // arbiter cycles with a compute wave request that fits nowhere
  kSpiLdsFull,   // per such cycle: CUs whose free LDS cannot take the wave
  kSpiWaveFull,  // per such cycle: SIMDs with no free wave slot
  kSpiVgprFull,  // per such cycle: SIMDs with too few free VGPRs
  kSpiSgprFull,  // per such cycle: SIMDs with too few free SGPRs
  kNumCtr
};

inline const char* name(int c) {
  static const char* kNames[kNumCtr] = {"SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES",  "SQ_WAVES",
                                        "SQ_LDS_IDX_ACTIVE",        "SQ_LDS_BANK_CONFLICT",
                                        "GRBM_GUI_ACTIVE",          "GRBM_COUNT",
                                        "TCC_EA0_RDREQ_DRAM_32B",   "TCC_EA0_WRREQ_WRITE_DRAM_32B",
                                        "TCC_EA0_RDREQ_GMI_32B",    "TCC_EA0_WRREQ_WRITE_GMI_32B",
                                        "SQ_CYCLES",                "SQ_INSTS_VALU_MFMA_MOPS_BF16",
                                        "SQ_INSTS_VALU_MFMA_MOPS_F8", "SPI_RA_RES_STALL_CSN",
                                        "SPI_RA_LDS_CU_FULL_CSN",   "SPI_RA_WAVE_SIMD_FULL_CSN",
                                        "SPI_RA_VGPR_SIMD_FULL_CSN", "SPI_RA_SGPR_SIMD_FULL_CSN"};
  return kNames[c];
}

// GRBM counters are per-XCC copies of one clock: reduce with max; everything else sums.
inline bool use_max(int c) { return c == kGuiActive || c == kGrbmCount; }

// Number of derived outputs (the CounterSource ABI: gpuexp_rp_sample fills this many
// doubles; gpuexp::kCounterOutputs in sources.h).
constexpr int kNumOut = 18;

// Per-XCC MFMA busy (gpuexp_rp_sample_xcc): at most this many XCCs per GPU.
constexpr int kMaxXcc = 16;

// Wave-level SQ counters and TCC EA requests are VMID-filtered for unprivileged clients.
// The filter is on the HARDWARE VMID, which the scheduler hands out dynamically, so an
// unprivileged exporter sometimes sees another process's waves (a VMID collision) and
// sometimes only its own (measured: bench at 1 Hz looked device-wide, at 10 Hz filtered).
// No heuristic on the values can tell those apart, so scope comes from privilege:
// CAP_SYS_ADMIN or CAP_PERFMON in the effective set (what a privileged DaemonSet has).
inline bool process_has_pmc_privilege() {
  FILE* f = std::fopen("/proc/self/status", "r");
  if (!f) return false;
  char line[256];
  unsigned long long eff = 0;
  while (std::fgets(line, sizeof(line), f))
    if (std::sscanf(line, "CapEff: %llx", &eff) == 1) break;
  std::fclose(f);
  constexpr int kCapSysAdmin = 21, kCapPerfmon = 38;
  return (eff >> kCapSysAdmin & 1ull) || (eff >> kCapPerfmon & 1ull);
}

// Validation knob (tests/test_gpu.py::test_device_scope_pmc_*): GPUEXP_PMC_ASSUME_DEVICE_SCOPE=1
// treats the wave/LDS/EA counters as device-wide in an unprivileged process.  Only sound
// when every kernel on the GPU belongs to the counting process itself (the VMID filter
// then passes all of them), which is how the calibration tests run.
inline bool pmc_device_scope() {
  const char* f = std::getenv("GPUEXP_PMC_ASSUME_DEVICE_SCOPE");
  return process_has_pmc_privilege() || (f && f[0] == '1');
}

struct Derived {
  uint32_t simd = 0, cu = 0;
  bool privileged = false;  // set at init: process_has_pmc_privilege()
  int scope = -1;  // -1 unknown, 0 wave/EA counters VMID-filtered to this process, 1 device-wide
  double latest[kNumOut] = {};
  // Per-XCC MFMA busy of the latest window (NaN: that XCC's GRBM clock did not advance);
  // nxcc = 0 until the samples' XCC coordinates are known.
  double xcc_busy[kMaxXcc] = {};
  int nxcc = 0;
  bool valid = false;
  uint64_t windows = 0;
};

// d: per-counter deltas over `wall` seconds; inst: instances that were reduced per counter.
inline void derive(Derived& a, const double* d, const int* inst, double wall) {
  const double nan = std::nan("");
  const double gui = d[kGuiActive];
  // Scope.  SQ_VALU_MFMA_BUSY_CYCLES and GRBM are chip-global in every case (measured
  // against rocprofv3 dispatch counts: profiles/r01/pmc_gemm_dispatch.txt); the wave/LDS/EA
  // set is only device-wide for a privileged client (see process_has_pmc_privilege).
  // Privileged: device-wide unless a busy MFMA window shows no waves at all (sticky 0).
  if (!a.privileged) a.scope = 0;
  else if (a.scope != 0) a.scope = (d[kGrbmCount] > 0 && gui / d[kGrbmCount] > 0.5 && d[kMfma] > 0 &&
                                    d[kWaves] / wall < 1000.0) ? 0 : 1;
  double* out = a.latest;
  // MFMA busy over ELAPSED cycles (GRBM_COUNT, the free-running GRBM clock): the share of
  // the window's wall time the matrix cores of all SIMDs were issuing, so an idle GPU
  // reads 0 whatever it ran before (the DCGM tensor-active semantics).  out[10] is
  // counter_defs.yaml's MfmaUtil, over GUI-ACTIVE cycles only: a GEMM that runs for 1 % of
  // the window reads ~90 there and ~1 here.
  out[0] = d[kGrbmCount] > 0 && a.simd ? std::min(100.0, 100.0 * d[kMfma] / (d[kGrbmCount] * a.simd)) : nan;
  out[10] = gui > 0 && a.simd ? std::min(100.0, 100.0 * d[kMfma] / (gui * a.simd)) : nan;  // MfmaUtil
  const double se = inst[kSqBusy] > 0 ? inst[kSqBusy] : 1;                           // one per SE
  out[1] = gui > 0 ? std::min(100.0, 100.0 * d[kSqBusy] / (gui * se)) : nan;
  out[2] = d[kGrbmCount] > 0 ? 100.0 * gui / d[kGrbmCount] : nan;                    // GPU busy
  out[3] = d[kWaves] / wall;                                                         // waves/s
  out[4] = gui > 0 && a.cu ? 100.0 * d[kLdsActive] / (gui * a.cu) : nan;            // LDS util
  out[5] = d[kLdsActive] > 0 ? 100.0 * d[kLdsConflict] / d[kLdsActive] : 0.0;       // bank conflicts
  out[6] = d[kDramRd32] * 32.0 / wall;                                              // HBM read B/s
  out[7] = d[kDramWr32] * 32.0 / wall;                                              // HBM write B/s
  out[8] = d[kGmiRd32] * 32.0 / wall;                                               // remote (GMI) read B/s
  out[9] = d[kGmiWr32] * 32.0 / wall;                                               // remote (GMI) write B/s
  out[11] = d[kMopsBf16] * 512.0 / wall;                                            // bf16 MFMA FLOP/s
  out[12] = d[kMopsF8] * 512.0 / wall;                                              // fp8 MFMA FLOP/s
  // Occupancy limiters, from the SPI resource allocator (one instance per SE).  out[13]: the
  // share of the allocator's arbitration cycles in which an SE had a compute wave ready that
  // fit on none of its CUs; the allocator arbitrates every kSpiArbClocks clocks (measured on
  // MI355X: a permanently stalled queue reads 24.9-25.0 % of GRBM_COUNT, profiles/r04/
  // spi_scope.txt).  out[14..17]: over those stalled cycles, the share of the SE's CUs whose
  // LDS was too full for it / of its SIMDs without a free wave slot / without enough VGPRs /
  // without enough SGPRs, i.e. what capped residency.  0 when no wave waited.
  constexpr double kSpiArbClocks = 4.0;
  const double spi = inst[kSpiResStall] > 0 ? inst[kSpiResStall] : 0;
  const double stall = d[kSpiResStall];
  out[13] = spi > 0 && d[kGrbmCount] > 0
                ? std::min(100.0, 100.0 * kSpiArbClocks * stall / (spi * d[kGrbmCount]))
                : nan;
  const double cu_se = spi > 0 ? double(a.cu) / spi : 0, simd_se = spi > 0 ? double(a.simd) / spi : 0;
  auto share = [&](double full, double per_se) {
    if (spi <= 0 || per_se <= 0) return nan;
    return stall > 0 ? std::min(100.0, 100.0 * full / (stall * per_se)) : 0.0;
  };
  out[14] = share(d[kSpiLdsFull], cu_se);
  out[15] = share(d[kSpiWaveFull], simd_se);
  out[16] = share(d[kSpiVgprFull], simd_se);
  out[17] = share(d[kSpiSgprFull], simd_se);
  a.valid = true;
  a.windows += 1;
}

// Continuous cumulative counting: what to do with a window of deltas `d` (this read minus
// the previous one) that spans `wall` seconds.  Counters that went backwards were reset or
// re-programmed by someone else (another profiler's start packet); a GRBM_COUNT that did not
// advance over real time means counting was stopped under us (GRBM_COUNT always advances
// while counting runs) -- two such windows in a row, so one fluke never costs a re-arm.  Both
// re-arm counting with our own selects (aql_pmc.cc rearm).  The first window after (re)arming
// has no previous read to subtract: skipped.
enum WindowAction { kPublish = 0, kSkip = 1, kRearm = 2 };
inline WindowAction window_action(const double* d, bool first, double wall, int* zero_grbm) {
  bool backwards = false;
  for (int k = 0; k < kNumCtr; ++k) backwards = backwards || d[k] < 0;
  *zero_grbm = !first && !backwards && d[kGrbmCount] <= 0 && wall > 0.005 ? *zero_grbm + 1 : 0;
  if (!first && (backwards || *zero_grbm >= 2)) {
    *zero_grbm = 0;
    return kRearm;
  }
  return first ? kSkip : kPublish;
}

// Re-arming after a foreign reset (pmc_rounds.cc).  The PMC selects are chip state: another
// profiler on the GPU (rocprofv3, omniperf) that programs them also resets ours, and
// re-programming them at once would silently corrupt ITS session.  So the exporter does not
// fight: after a reset its windows are withheld (the counter families go absent, the health
// counter `reset` rises) and it re-arms only once the counters have been left alone for a
// back-off that doubles with every further reset it sees (another profiler resets them per
// dispatch or per session), up to max_ns.  Counters that merely stopped (GRBM_COUNT standing
// still: the other profiler finished) do not extend the back-off.  A reset soon after our own
// re-arm doubles it too; a re-arm calm_ns after the last one starts from base_ns again.
// GPUEXP_PMC_REARM: backoff (default) | off (never re-arm: withheld until restart) | now
// (re-arm at the first reset, the round-4 behaviour).
enum RearmMode { kRearmOff = 0, kRearmBackoff = 1, kRearmNow = 2 };
struct RearmConfig {
  RearmMode mode = kRearmBackoff;
  int64_t base_ns = 2000000000ll;     // first back-off (GPUEXP_PMC_REARM_BACKOFF_MS)
  int64_t max_ns = 64000000000ll;
  int64_t calm_ns = 300000000000ll;
};
struct RearmState {
  bool waiting = false;     // counters not ours since a reset: windows withheld, re-arm pending
  int64_t due_ns = 0;       // when to re-arm (while waiting)
  int64_t backoff_ns = 0;   // current back-off (0: not set yet = base)
  int64_t last_arm_ns = 0;  // when counting was last (re)armed by us (0: never)
  uint64_t conflicts = 0;   // resets that extended the back-off
};

// A window said the counters were reset (backwards) or stopped (!backwards) under us.
inline void rearm_on_reset(RearmState& s, const RearmConfig& c, int64_t now, bool backwards) {
  if (s.backoff_ns <= 0 || (!s.waiting && s.last_arm_ns && now - s.last_arm_ns > c.calm_ns)) s.backoff_ns = c.base_ns;
  if (!s.waiting) {
    s.waiting = true;
    if (backwards && s.last_arm_ns && now - s.last_arm_ns < 2 * s.backoff_ns) {  // right after our re-arm
      s.backoff_ns = std::min(2 * s.backoff_ns, c.max_ns);
      ++s.conflicts;
    }
    s.due_ns = c.mode == kRearmNow ? now : now + s.backoff_ns;
    return;
  }
  if (backwards) {  // reset again while we wait: someone is using the counters; wait longer
    ++s.conflicts;
    s.backoff_ns = std::min(2 * s.backoff_ns, c.max_ns);
    s.due_ns = c.mode == kRearmNow ? now : now + s.backoff_ns;
  }
}
inline bool rearm_due(const RearmState& s, const RearmConfig& c, int64_t now) {
  return s.waiting && c.mode != kRearmOff && now >= s.due_ns;
}
inline void rearm_done(RearmState& s, int64_t now) {
  s.waiting = false;
  s.last_arm_ns = now;
}

// Per-XCC MFMA busy: the chip formula with one XCC's share of the SIMDs.  mfma[x] sums that
// XCC's SQ instances (one per SE), grbm[x] is that XCC's own GRBM_COUNT.  Each XCD runs its
// own clock (DPM lowers a busy XCD's clock while idle ones stay high), so busy cycles are
// only comparable with the same XCD's elapsed cycles: the chip value becomes the mean of the
// per-XCC shares whenever they are known (the max-GRBM_COUNT formula of derive() read 10.3
// instead of 11.0 with one XCD 88 % busy: profiles/r03/xcc_mfma_calibration.txt).
inline void derive_xcc(Derived& a, const double* mfma, const double* grbm, int nxcc) {
  const double simd = nxcc > 0 ? double(a.simd) / nxcc : 0;
  double sum = 0;
  int n = 0;
  for (int x = 0; x < nxcc && x < kMaxXcc; ++x) {
    a.xcc_busy[x] = grbm[x] > 0 && simd > 0 ? std::min(100.0, 100.0 * mfma[x] / (grbm[x] * simd)) : std::nan("");
    if (!std::isnan(a.xcc_busy[x])) {
      sum += a.xcc_busy[x];
      ++n;
    }
  }
  a.nxcc = std::min(nxcc, kMaxXcc);
  if (n == a.nxcc && n > 0) a.latest[0] = sum / n;
}

}  // namespace gpuexp_ctr
