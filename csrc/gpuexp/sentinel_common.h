// Sentinel pieces shared by its two hosts: the HIP plugin (sentinel.hip, its own stream)
// and the aqlprofile plugin (aql_pmc.cc), which dispatches the same kernel as raw AQL on
// the HSA queue it already owns for the PMC counters, so sentinel + counters cost one GPU
// queue instead of two (each queue pins a ~173 MiB context save/restore area on MI355X;
// profiles/r01/exporter_rss.txt).  Ring layout, kernel arguments and the host-side
// drain of completed runs live here; the device code is in sentinel_device.h.
#pragma once

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "gpuexp/device.h"

namespace gpuexp {

constexpr int kSentinelMaxWaves = kMaxXcc;

struct alignas(64) SentinelSlot {
  uint64_t seq;          // written LAST by the wave (system-scope release)
  uint64_t rt0, rt1;     // s_memrealtime at start / end of the clock window (100 MHz)
  uint64_t mt0, mt1;     // s_memtime at start / end (shader clock)
  uint32_t xcc_id;
  uint32_t hw_id;
  uint64_t chase_rt;     // s_memrealtime ticks for `hops` dependent uncached HBM loads
  uint32_t hops;
  uint32_t chase_end;    // last index reached (keeps the chain live; must be 0)
};
static_assert(sizeof(SentinelSlot) == 64, "one cache line per wave: XCDs never share a line");

// Pointer chase for the memory-latency probe: `kChaseHops` 4-byte links 4 KiB apart in an
// uncached device buffer; each hop is a dependent volatile load, so the chain time is
// the memory path's load latency under the current traffic.  hop i -> i+1, last -> 0.
constexpr int kChaseHops = 16;
constexpr size_t kChaseStride = 4096 / sizeof(uint32_t);

// By-value kernel arguments of the HSACO entry points (gpuexp_sentinel / _init_chase).
struct SentinelArgs {
  SentinelSlot* ring;
  const uint32_t* chase;
  uint64_t seq;
  uint32_t slot;
  int32_t spin;
  int32_t hops;
  int32_t pad;
};
struct SentinelInitArgs {
  uint32_t* chase;
  int32_t hops;
  int32_t pad;
};

inline uint64_t sentinel_hsa_now() {
  uint64_t t = 0;
  hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
  return t;
}

// Per-GPU ring bookkeeping of one sentinel host.
struct SentinelRun {
  SentinelSlot* ring = nullptr;       // host view, nslots x kSentinelMaxWaves slots
  int waves = 1;                      // workgroups per run: one per XCD of this GPU / partition
  std::vector<uint64_t> host_launch;  // per run slot, HSA system time just before launch
  hsa_agent_t agent{};
  bool have_agent = false;
  uint64_t launched = 0, completed = 0, stalled = 0, errors = 0;
  // at the last drain (every tick's read, and each launch tick before its launch): age of the
  // oldest run still outstanding, 0 when every earlier launch had finished
  double pending_s = 0;
  // the run launched at this tick (0: none): it is not "waiting" when the same tick reads it
  // microseconds later (sentinel_read)
  uint64_t fresh_seq = 0;
  SentinelReading last;
};

// Host launch -> wave start (seconds), NaN when the clock domains disagree.
inline double sentinel_wave_latency(const SentinelRun& p, const SentinelSlot& w, uint64_t host_launch,
                                    double sys_ns_per_tick) {
  uint64_t sys = 0;
  if (!p.have_agent || hsa_amd_profiling_convert_tick_to_system_domain(p.agent, w.rt0, &sys) != HSA_STATUS_SUCCESS)
    return std::nan("");
  double lat = (double(sys) - double(host_launch)) * sys_ns_per_tick * 1e-9;
  // A negative value means the GPU tick and s_memrealtime domains disagree; keep the rest
  // of the reading and drop the latency rather than export garbage.
  if (lat > -1e-6 && lat < 10.0) return lat < 0 ? 0 : lat;
  return std::nan("");
}

// Folds every completed run (all its waves published their seq) into p.last.
inline void sentinel_drain(SentinelRun& p, int nslots, double sys_ns_per_tick) {
  while (p.completed < p.launched) {
    const uint64_t seq = p.completed + 1;
    const uint32_t slot = uint32_t(seq % uint64_t(nslots));
    const SentinelSlot* s = p.ring + size_t(slot) * kSentinelMaxWaves;
    bool done = true;
    for (int w = 0; w < p.waves && done; ++w) done = __atomic_load_n(&s[w].seq, __ATOMIC_ACQUIRE) == seq;
    if (!done) break;
    p.completed = seq;
    SentinelReading r = p.last;  // an XCD without a wave this run keeps its previous latency
    r.ok = true;
    r.xcc_id = double(s[0].xcc_id & 0xF);
    r.dispatch_latency_s = std::nan("");
    double sclk[kSentinelMaxWaves];
    int ns = 0;
    double mem_sum = 0;
    int mem_n = 0;
    for (int w = 0; w < p.waves; ++w) {
      const double drt = double(s[w].rt1 - s[w].rt0);
      const double dmt = double(s[w].mt1 - s[w].mt0);
      if (drt > 0) sclk[ns++] = dmt / drt * 100e6;
      if (s[w].hops > 0 && s[w].chase_end == 0) {  // 100 MHz ticks per hop -> seconds
        const double hl = double(s[w].chase_rt) * 10e-9 / double(s[w].hops);
        mem_sum += hl;
        ++mem_n;
        const uint32_t hx = s[w].xcc_id & 0xF;
        if (hx < uint32_t(kMaxXcc)) r.xcc_mem_latency_s[hx] = hl;
      }
      const double lat = sentinel_wave_latency(p, s[w], p.host_launch[slot], sys_ns_per_tick);
      if (std::isnan(lat)) continue;
      if (std::isnan(r.dispatch_latency_s) || lat < r.dispatch_latency_s) r.dispatch_latency_s = lat;
      const uint32_t x = s[w].xcc_id & 0xF;
      if (x < uint32_t(kMaxXcc)) r.xcc_latency_s[x] = lat;
    }
    std::nth_element(sclk, sclk + ns / 2, sclk + ns);
    r.sclk_hz = ns ? sclk[ns / 2] : std::nan("");
    r.mem_latency_s = mem_n ? mem_sum / mem_n : std::nan("");
    p.last = r;
  }
  p.pending_s = 0;
  if (p.completed < p.launched) {
    const uint64_t launch = p.host_launch[size_t((p.completed + 1) % uint64_t(nslots))];
    const uint64_t now = sentinel_hsa_now();
    p.pending_s = now > launch ? double(now - launch) * sys_ns_per_tick * 1e-9 : 1e-9;
  }
}

// The latest reading plus pending_s (as of the last drain); false until a run completed or
// one is found outstanding.  Before the first completion only pending_s is set.
inline bool sentinel_fill(const SentinelRun& p, SentinelReading* out) {
  if (!p.last.ok && !(p.pending_s > 0)) return false;
  *out = p.last;
  out->ok = true;
  out->runs = p.completed;
  out->pending_s = p.pending_s;
  return true;
}

// A sampler tick's read of GPU `p`: folds in completed runs and brings pending_s up to date
// (every tick, although launches run at most every sentinel_min_interval); a run launched by
// this same tick counts as not pending yet.
inline bool sentinel_read(SentinelRun& p, int nslots, double sys_ns_per_tick, SentinelReading* out) {
  sentinel_drain(p, nslots, sys_ns_per_tick);
  if (p.fresh_seq && p.completed + 1 == p.fresh_seq) p.pending_s = 0;
  p.fresh_seq = 0;
  return sentinel_fill(p, out);
}

// Marks run `seq`'s slots unpublished and returns the slot it uses.
inline uint32_t sentinel_prepare(SentinelRun& p, uint64_t seq, int nslots) {
  const uint32_t slot = uint32_t(seq % uint64_t(nslots));
  SentinelSlot* s = p.ring + size_t(slot) * kSentinelMaxWaves;
  for (int w = 0; w < p.waves; ++w) __atomic_store_n(&s[w].seq, 0ull, __ATOMIC_RELAXED);
  p.host_launch[slot] = sentinel_hsa_now();
  return slot;
}

}  // namespace gpuexp
