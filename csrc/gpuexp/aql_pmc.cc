// Device PMC plugin on an exporter-owned HSA queue (_gpuexp_aqlpmc.so), dlopen()ed by the
// core through the same gpuexp_rp_* ABI as the rocprofiler-sdk plugin (rocprof_plugin.cc).
//
// Why not rocprofiler-sdk's device counting service: registering that tool makes an HSA
// runtime thread spin one core at 100% for the life of the process (rocprof_plugin.cc
// header; measured 101% exporter CPU).  The counting itself is only three PM4 programs —
// select+reset+enable, and read+disable — which libhsa-amd-aqlprofile64 generates as AQL
// vendor packets (hsa_ven_amd_aqlprofile.h).  Here each GPU gets:
//   * one low-priority AQL queue of 64 slots (shared with the sentinel, see below),
//   * one interrupt-backed completion signal (waited on BLOCKED — no polling thread),
//   * a command buffer and a PMC output buffer in fine-grained system memory,
// and a background thread runs the counting in one of two modes:
//   continuous (default): one start packet at init, then one read packet per engine tick
//     (gpuexp_rp_kick at the tick's start; gpuexp_rp_sync before the tick exports), so
//     every tick exports the deltas over exactly its own interval and no wall time goes
//     uncounted.  What a read does to running counters (keep counting / reset / stop) is
//     probed on the GPU at init (read_semantics) rather than assumed.
//   duty: start packet -> wait -> sleep(window) -> read packet -> wait -> stop packet ->
//     wait -> iterate output, one window per interval (the round-1/2 behaviour).
// Measured on MI355X (profiles/r01/counters_aqlpmc.txt): same counter values as the
// rocprofiler-sdk path, exporter CPU 0.3-0.7% instead of 101%; continuous vs duty costs:
// profiles/r03/pmc_continuous_cost.txt.
// The engine's tick never blocks on the GPU beyond a bounded sync: gpuexp_rp_sample returns
// the latest completed window.
//
// Event ids are the gfx950 select values of /opt/rocm/share/rocprofiler-sdk/counter_defs.yaml
// (SQ 93/3/4/147/142, GRBM 2/0, TCC 112/115/113/117, SPI 91/120/103/109/115) and are checked with
// hsa_ven_amd_aqlprofile_validate_event at init.  TCC is programmed on every channel
// instance (16 per XCD); SQ and GRBM are broadcast and come back once per SE / XCC.
#include <execinfo.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_aqlprofile.h>

#include <algorithm>
#include <cctype>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>
#include <fcntl.h>
#include <sys/prctl.h>
#include <time.h>
#include <unistd.h>

#include "gpuexp/counter_model.h"
#include "gpuexp/pmc_agents.h"
#include "gpuexp/pmc_rounds.h"
#include "kernels/probe_args.h"
#include "gpuexp/sentinel_common.h"
#include "gpuexp/sources.h"

static_assert(gpuexp_ctr::kNumOut == gpuexp::kCounterOutputs, "counter plugin ABI");

namespace {

using namespace gpuexp_ctr;
using Clock = std::chrono::steady_clock;

struct EventDef {
  hsa_ven_amd_aqlprofile_block_name_t block;
  uint32_t id;
  int ctr;
};

// gfx950 select values (counter_defs.yaml, architectures: gfx950).
const EventDef kGfx950[] = {
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 93, kMfma},        {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 3, kSqBusy},
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 4, kWaves},        {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 147, kLdsActive},
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 142, kLdsConflict}, {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, 2, kGuiActive},
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_GRBM, 0, kGrbmCount},  {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TCC, 112, kDramRd32},
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TCC, 115, kDramWr32},  {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TCC, 113, kGmiRd32},
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TCC, 117, kGmiWr32},  {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 2, kSqCycles},
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 52, kMopsBf16},    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SQ, 56, kMopsF8},
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SPI, 91, kSpiResStall}, {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SPI, 120, kSpiLdsFull},
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SPI, 103, kSpiWaveFull}, {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SPI, 109, kSpiVgprFull},
    {HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SPI, 115, kSpiSgprFull},
};

// One GPU: its HSA queue(s), signals and aqlprofile programs.  The read machine
// (pmc_rounds.cc) drives it through the ReadPort interface; init, the duty-cycled windows and
// the sentinel / calibration dispatches use it directly.
// Its queue, signal and buffers (and the rescue queue's) are AgentResources (pmc_agents.h), created
// and released through HsaOps by the same code the stub-GPU lifecycle test runs.
struct Agent : public gpuexp_pmc::ReadPort, gpuexp_pmc::AgentResources<hsa_queue_t*, hsa_signal_t> {
  int dev = -1;
  hsa_agent_t gpu{};
  std::string bdf, gfx;
  std::vector<hsa_ven_amd_aqlprofile_event_t> events;
  std::vector<int> event_ctr;  // events[i] -> Ctr
  hsa_ven_amd_aqlprofile_profile_t profile{};
  hsa_ext_amd_aql_pm4_packet_t start_pkt{}, read_pkt{}, stop_pkt{};
  uint32_t out_size = 0, cmd_size = 0;
  bool ready = false;
  std::atomic<bool> queue_error{false};
  // The queue has two producers: the read machine / init (PM4 programs) and the sampler
  // thread (sentinel kernel dispatches, gpuexp_make_hsa_sentinel).
  std::mutex submit_mu;
  Clock::time_point t_submit{};  // run_packet (init, duty windows)
  Derived model;                 // SIMD / CU counts, privilege (the machine's derivations)
  // Read rescue (pmc_rounds.cc): a second queue that only ever carries read packets, with its
  // own profile, command and output buffers; exists between open_rescue and close_rescue.
  hsa_ven_amd_aqlprofile_profile_t rprofile{};
  hsa_ext_amd_aql_pm4_packet_t rstart_pkt{}, rread_pkt{};
  // debug (GPUEXP_AQLPMC_DEBUG): aqlprofile's coordinates of the first MFMA sample and the last
  // read's MFMA / GRBM samples
  std::mutex dbg_mu;
  std::string coord_names, last_xsamples;

  // ReadPort (pmc_rounds.h); defined below
  void post_read(int q) override;
  void post_arm(bool baseline_read) override;
  void post_start() override;
  void post_stop(int q) override;
  bool done(int q) override;
  bool failed() override { return queue_error.load(); }
  bool collect(int q, gpuexp_pmc::Sample* out) override;
  bool open_rescue() override;
  void close_rescue() override;
  std::string label() const override { return bdf; }
};

// aqlprofile entry points come from the runtime's extension table: the runtime loads
// libhsa-amd-aqlprofile64.so and hands it the HSA API table (calling the library's exports
// directly, without that hand-off, faults inside it).
hsa_ven_amd_aqlprofile_pfn_t g_aql{};
bool g_debug = false;

void crumb(const char* what, const std::string& detail = "") {
  if (g_debug) std::fprintf(stderr, "[aqlpmc] %s %s\n", what, detail.c_str());
}

void segv_backtrace(int sig) {
  void* frames[48];
  const int n = ::backtrace(frames, 48);
  ::backtrace_symbols_fd(frames, n, 2);
  ::signal(sig, SIG_DFL);
  ::raise(sig);
}

std::mutex g_mu;
std::vector<Agent*> g_agents;  // indexed by the engine's device index
std::string g_status = "not initialised";
bool g_hsa_up = false;
hsa_amd_memory_pool_t g_sys_pool{};
bool g_have_pool = false;
uint64_t g_ts_freq = 1000000000ull;
int g_window_ms = 20;
int g_interval_ms = 1000;
// Duty-cycled windows (gpuexp_rp_set_duty, or continuous counting unavailable): this
// thread's start -> sleep(window) -> read -> stop loop.
std::thread g_thread;
std::atomic<bool> g_quit{false};
std::condition_variable g_cv;
std::mutex g_cv_mu;
std::atomic<uint64_t> g_thread_cpu_ns{0};  // the duty thread's own CPU, published per window
// Continuous mode (gpuexp_rp_set_continuous): counting is started once and never stopped;
// the engine kicks one read round per tick, run by the read machine (pmc_rounds.h).
bool g_continuous = false;
// Inline rounds (continuous mode; gpuexp_rp_set_inline, which the engine calls when its
// sampler ticks periodically; GPUEXP_PMC_INLINE=0/1 overrides): the engine's sampler posts
// the round's read packets itself at gpuexp_rp_kick and collects them at gpuexp_rp_sync, after
// its device reads (~100-400 us later: the reads are done by then), so a tick costs the
// counting thread no wake-ups at all.
bool g_inline = false;
// The read machine: created at init (every mode: it also publishes duty windows), destroyed at
// shutdown after the engine's sampler has stopped kicking.
std::atomic<gpuexp_pmc::RoundMachine*> g_machine{nullptr};

uint64_t own_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}
using gpuexp_pmc::ReadMode;
using gpuexp_pmc::kReadUnknown;
using gpuexp_pmc::kCumulative;
using gpuexp_pmc::kResets;
using gpuexp_pmc::kStops;
using gpuexp_pmc::read_mode_name;
ReadMode g_read_mode = kReadUnknown;

std::string lower(std::string s) {
  for (auto& c : s) c = char(::tolower(c));
  return s;
}

void queue_error_cb(hsa_status_t, hsa_queue_t*, void* data) {
  static_cast<Agent*>(data)->queue_error.store(true);
}

hsa_status_t pick_sys_pool(hsa_amd_memory_pool_t pool, void*) {
  hsa_amd_segment_t seg{};
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  bool alloc = false;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  if (alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT)) {
    g_sys_pool = pool;
    g_have_pool = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

struct Found {
  std::vector<std::pair<hsa_agent_t, std::string>> gpus;  // (agent, bdf)
  std::vector<hsa_agent_t> cpus;
};

hsa_status_t collect_agent(hsa_agent_t a, void* ud) {
  auto* f = static_cast<Found*>(ud);
  hsa_device_type_t t{};
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU) {
    f->cpus.push_back(a);
  } else if (t == HSA_DEVICE_TYPE_GPU) {
    uint32_t bdfid = 0, domain = 0;
    hsa_agent_get_info(a, hsa_agent_info_t(HSA_AMD_AGENT_INFO_BDFID), &bdfid);
    hsa_agent_get_info(a, hsa_agent_info_t(HSA_AMD_AGENT_INFO_DOMAIN), &domain);
    char bdf[32];
    std::snprintf(bdf, sizeof(bdf), "%04x:%02x:%02x.%x", domain, (bdfid >> 8) & 0xFF, (bdfid >> 3) & 0x1F,
                  bdfid & 0x7);
    f->gpus.emplace_back(a, bdf);
  }
  return HSA_STATUS_SUCCESS;
}

void* sys_alloc(size_t bytes, hsa_agent_t gpu) {
  bytes = (bytes + 4095) & ~size_t(4095);
  void* p = nullptr;
  if (hsa_amd_memory_pool_allocate(g_sys_pool, bytes, 0, &p) != HSA_STATUS_SUCCESS) return nullptr;
  if (hsa_amd_agents_allow_access(1, &gpu, nullptr, p) != HSA_STATUS_SUCCESS) {
    hsa_amd_memory_pool_free(p);
    return nullptr;
  }
  std::memset(p, 0, bytes);
  return p;
}

// The HSA calls behind pmc_agents.h's lifecycle helpers, for one agent.
struct HsaOps {
  Agent* a;
  bool create_queue(hsa_queue_t** q) {
    if (hsa_queue_create(a->gpu, 64, HSA_QUEUE_TYPE_MULTI, queue_error_cb, a, UINT32_MAX, UINT32_MAX, q) !=
        HSA_STATUS_SUCCESS) {
      *q = nullptr;
      return false;
    }
    // experiment knob (profiles/r03/mfma_calibration.txt): low | normal | high
    const char* pr = std::getenv("GPUEXP_PMC_QUEUE_PRIORITY");
    const std::string p = pr ? pr : "low";
    hsa_amd_queue_set_priority(*q, p == "high"     ? HSA_AMD_QUEUE_PRIORITY_HIGH
                                   : p == "normal" ? HSA_AMD_QUEUE_PRIORITY_NORMAL
                                                   : HSA_AMD_QUEUE_PRIORITY_LOW);
    return true;
  }
  void destroy_queue(hsa_queue_t* q) { hsa_queue_destroy(q); }
  bool valid(hsa_queue_t* q) const { return q != nullptr; }
  bool create_signal(hsa_signal_t* s) { return hsa_signal_create(1, 0, nullptr, s) == HSA_STATUS_SUCCESS; }
  void destroy_signal(hsa_signal_t s) { hsa_signal_destroy(s); }
  bool valid(hsa_signal_t s) const { return s.handle != 0; }
  void* alloc(size_t bytes) { return sys_alloc(bytes, a->gpu); }
  void release(void* p) { hsa_amd_memory_pool_free(p); }
};

// Writes one vendor-specific AQL packet and rings the doorbell.  At most one PM4 packet and
// one sentinel dispatch are ever in flight on the 64-slot queue, so it never fills.
// barrier=false lets the packet processor run it without waiting for earlier packets to
// COMPLETE: the continuous read packets use that, so a sentinel dispatch that cannot get a
// SIMD (measured: next to waves issuing MFMAs back-to-back for seconds, even at wave
// priority 3) does not hold the counter reads behind it.
void submit_on(Agent& a, hsa_queue_t* q, hsa_signal_t sig, const hsa_ext_amd_aql_pm4_packet_t& pkt, bool barrier) {
  std::lock_guard<std::mutex> lk(a.submit_mu);
  const uint64_t idx = hsa_queue_add_write_index_screlease(q, 1);
  auto* slot = static_cast<hsa_ext_amd_aql_pm4_packet_t*>(q->base_address) + (idx & (q->size - 1));
  std::memcpy(slot->pm4_command, pkt.pm4_command, sizeof(pkt.pm4_command));
  slot->completion_signal = sig;
  const uint16_t header = uint16_t((HSA_PACKET_TYPE_VENDOR_SPECIFIC << HSA_PACKET_HEADER_TYPE) |
                                   ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                                   (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                   (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  __atomic_store_n(&slot->header, header, __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, hsa_signal_value_t(idx));
}

void submit(Agent& a, const hsa_ext_amd_aql_pm4_packet_t& pkt, bool barrier = true) {
  submit_on(a, a.queue, a.sig, pkt, barrier);
}

// Submits `pkt`, waits (interrupt-driven) up to 1 s; returns the midpoint of submit and
// completion (the packet's execution time estimate), or a default time_point on timeout.
// Split form, so one round can have a packet in flight on every GPU at once.
void post_packet(Agent& a, const hsa_ext_amd_aql_pm4_packet_t& pkt, bool barrier = true) {
  hsa_signal_store_relaxed(a.sig, 1);
  a.t_submit = Clock::now();
  submit(a, pkt, barrier);
}

// Waits for a completion signal by sleeping and looking, never by spinning: ROCr's own
// wait (hsa_signal_wait_*, even HSA_WAIT_STATE_BLOCKED) busy-polls ~200 us before it
// sleeps, and a PM4 read program takes about that long, so every read cost ~211 us of
// CPU per GPU (measured: tools/exporter_profile.py round_cpu_us_wait).  Sleeping 60 us,
// then 100 us slices, costs a few us per read and adds < 100 us of latency, which the
// tick absorbs (the read is kicked at the tick's start and needed only at its series stage).
bool wait_signal(hsa_signal_t sig, Clock::time_point deadline) {
  for (int i = 0;; ++i) {
    if (hsa_signal_load_scacquire(sig) < 1) return true;
    const auto now = Clock::now();
    if (now >= deadline) return false;
    const auto step = std::chrono::microseconds(i == 0 ? 60 : 100);
    std::this_thread::sleep_for(std::min<Clock::duration>(step, deadline - now));
  }
}

Clock::time_point wait_packet(Agent& a) {
  const bool done = wait_signal(a.sig, Clock::now() + std::chrono::seconds(1));
  const auto t1 = Clock::now();
  if (!done || a.queue_error.load()) return {};
  return a.t_submit + (t1 - a.t_submit) / 2;
}

Clock::time_point run_packet(Agent& a, const hsa_ext_amd_aql_pm4_packet_t& pkt) {
  post_packet(a, pkt);
  return wait_packet(a);
}

struct Accum {
  Agent* a;
  double v[kNumCtr];
  int inst[kNumCtr];
  uint64_t samples;
  double xm[kMaxXcc];  // SQ_VALU_MFMA_BUSY_CYCLES per XCC
  double xg[kMaxXcc];  // GRBM_COUNT per XCC
  int nxcc;            // XCCs seen in both counters (0: coordinates unavailable)
  int xm_n, xg_n;      // highest XCC + 1 seen per counter
  bool x_unmapped;     // a sample of either counter fell outside the XCC layout
  int x_seen[2];       // sample_id 0 seen so far, per counter (sample_xcc)
  int xm_cnt[kMaxXcc];  // MFMA samples per XCC (one per SE: equal on every XCC)
  // debug: the MFMA / GRBM_COUNT samples in callback order (sample_id, XCC, value)
  struct S {
    uint32_t id;
    int xcc;
    double v;
  } xs[2][64];
  int xs_n[2];
};

struct CoordProbe {
  std::string names;
};

hsa_status_t on_coord(int, int, int, int coordinate, const char* name, void* ud) {
  auto* p = static_cast<CoordProbe*>(ud);
  p->names += (p->names.empty() ? "" : ",") + std::string(name ? name : "?") + "=" + std::to_string(coordinate);
  return HSA_STATUS_SUCCESS;
}

// XCC of a sample of SQ_VALU_MFMA_BUSY_CYCLES (k = 0) or GRBM_COUNT (k = 1), from its place in
// the output: aqlprofile returns a counter's samples XCC by XCC, numbering them from 0 again
// in every XCC (SQ: sample_id = SE 0..3; GRBM: 0 once per XCC), so the XCC is the number of
// sample_id 0 seen before.  Its event coordinates do not say it (gfx950: "XCD=0,INSTANCE=0,
// SE=s" for all eight XCDs).  The order is ground-truthed against HW_REG_XCC_ID by an MFMA
// kernel confined to one XCC (profiles/r03/xcc_mfma_calibration.txt).
int sample_xcc(Accum* acc, int k, uint32_t sample_id) {
  if (sample_id == 0) acc->x_seen[k] += 1;
  const int xcc = acc->x_seen[k] - 1;
  return xcc >= 0 && xcc < kMaxXcc ? xcc : -1;
}

hsa_status_t on_data(hsa_ven_amd_aqlprofile_info_type_t type, hsa_ven_amd_aqlprofile_info_data_t* d, void* ud) {
  if (type != HSA_VEN_AMD_AQLPROFILE_INFO_PMC_DATA) return HSA_STATUS_SUCCESS;
  auto* acc = static_cast<Accum*>(ud);
  acc->samples += 1;
  const auto& ev = d->pmc_data.event;
  for (const auto& def : kGfx950) {
    if (def.block != ev.block_name || def.id != ev.counter_id) continue;
    const double x = double(d->pmc_data.result);
    acc->v[def.ctr] = use_max(def.ctr) ? std::max(acc->v[def.ctr], x) : acc->v[def.ctr] + x;
    acc->inst[def.ctr] += 1;
    if (def.ctr == kMfma || def.ctr == kGrbmCount) {
      const int k = def.ctr == kMfma ? 0 : 1;
      const int xcc = sample_xcc(acc, k, d->sample_id);
      if (g_debug && k == 0 && d->sample_id == 0 && acc->x_seen[0] == 1) {
        std::lock_guard<std::mutex> lk(acc->a->dbg_mu);
        if (acc->a->coord_names.empty()) {  // once, for the debug line
          CoordProbe p;
          if (g_aql.hsa_ven_amd_aqlprofile_iterate_event_coord)
            g_aql.hsa_ven_amd_aqlprofile_iterate_event_coord(acc->a->gpu, ev, 0, on_coord, &p);
          acc->a->coord_names = p.names.empty() ? "none" : p.names;
        }
      }
      if (acc->xs_n[k] < 64) acc->xs[k][acc->xs_n[k]++] = {d->sample_id, xcc, x};
      if (xcc < 0) {
        acc->x_unmapped = true;
      } else if (k == 0) {
        acc->xm[xcc] += x;
        acc->xm_cnt[xcc] += 1;
        acc->xm_n = std::max(acc->xm_n, xcc + 1);
      } else {
        acc->xg[xcc] = std::max(acc->xg[xcc], x);
        acc->xg_n = std::max(acc->xg_n, xcc + 1);
      }
    }
    break;
  }
  return HSA_STATUS_SUCCESS;
}

bool setup_agent(Agent& a, std::string* why) {
  char name[64] = {};
  hsa_agent_get_info(a.gpu, HSA_AGENT_INFO_NAME, name);
  a.gfx = name;
  crumb("agent", a.bdf + " " + a.gfx);
  if (a.gfx != "gfx950") {
    *why = "no PMC event table for " + a.gfx;
    return false;
  }
  uint32_t cu = 0, simd_per_cu = 0;
  hsa_agent_get_info(a.gpu, hsa_agent_info_t(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &cu);
  hsa_agent_get_info(a.gpu, hsa_agent_info_t(HSA_AMD_AGENT_INFO_NUM_SIMDS_PER_CU), &simd_per_cu);
  a.model.cu = cu;
  a.model.privileged = pmc_device_scope();
  a.model.simd = cu * simd_per_cu;

  hsa_ven_amd_aqlprofile_profile_t probe{};
  probe.agent = a.gpu;
  probe.type = HSA_VEN_AMD_AQLPROFILE_EVENT_TYPE_PMC;
  hsa_ven_amd_aqlprofile_id_query_t tcc{"TCC", 0, 0};
  if (g_aql.hsa_ven_amd_aqlprofile_get_info(&probe, HSA_VEN_AMD_AQLPROFILE_INFO_BLOCK_ID, &tcc) != HSA_STATUS_SUCCESS ||
      tcc.instance_count == 0)
    tcc.instance_count = 16;
  // GPUEXP_PMC_NO_SPI=1: without the SPI occupancy-limiter events (and the fallback below)
  const char* no_spi = std::getenv("GPUEXP_PMC_NO_SPI");
  const bool want_spi = !(no_spi && no_spi[0] == '1');
  for (const auto& def : kGfx950) {
    if (def.block == HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SPI && !want_spi) continue;
    const uint32_t n = def.block == HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_TCC ? tcc.instance_count : 1;
    for (uint32_t i = 0; i < n; ++i) {
      hsa_ven_amd_aqlprofile_event_t ev{def.block, i, def.id};
      bool ok = false;
      if (g_aql.hsa_ven_amd_aqlprofile_validate_event(a.gpu, &ev, &ok) != HSA_STATUS_SUCCESS || !ok) continue;
      a.events.push_back(ev);
      a.event_ctr.push_back(def.ctr);
    }
  }
  crumb("events", std::to_string(a.events.size()) + " (TCC instances " + std::to_string(tcc.instance_count) + ")");
  if (a.events.empty()) {
    *why = "aqlprofile rejected every event";
    return false;
  }
  a.profile.agent = a.gpu;
  a.profile.type = HSA_VEN_AMD_AQLPROFILE_EVENT_TYPE_PMC;
  a.profile.events = a.events.data();
  a.profile.event_count = uint32_t(a.events.size());
  uint32_t cmd_size = 0, out_size = 0;
  if (g_aql.hsa_ven_amd_aqlprofile_get_info(&a.profile, HSA_VEN_AMD_AQLPROFILE_INFO_COMMAND_BUFFER_SIZE, &cmd_size) !=
          HSA_STATUS_SUCCESS ||
      g_aql.hsa_ven_amd_aqlprofile_get_info(&a.profile, HSA_VEN_AMD_AQLPROFILE_INFO_PMC_DATA_SIZE, &out_size) !=
          HSA_STATUS_SUCCESS ||
      cmd_size == 0 || out_size == 0) {
    *why = "aqlprofile buffer size query failed";
    return false;
  }
  crumb("buffers", "cmd " + std::to_string(cmd_size) + " out " + std::to_string(out_size));
  // The legacy size query does not scale the PM4 program by the XCC count (gfx950: 8 XCCs
  // per agent; measured: a buffer of the reported 8 KiB is overrun inside
  // hsa_ven_amd_aqlprofile_start), so both buffers are over-provisioned.
  cmd_size = std::max<uint32_t>(cmd_size * 16, 256u << 10);
  out_size = std::max<uint32_t>(out_size * 16, 64u << 10);
  HsaOps ops{&a};
  a.cmd_buf = ops.alloc(cmd_size);
  a.out_buf = ops.alloc(out_size);
  if (!a.cmd_buf || !a.out_buf) {
    *why = "system memory pool allocation failed";
    return false;
  }
  a.profile.command_buffer = {a.cmd_buf, cmd_size};
  a.profile.output_buffer = {a.out_buf, out_size};
  if (g_aql.hsa_ven_amd_aqlprofile_start(&a.profile, &a.start_pkt) != HSA_STATUS_SUCCESS) {
    // the SPI block's counters are the newest addition: without them rather than nothing
    auto spi = [](const hsa_ven_amd_aqlprofile_event_t& e) { return e.block_name == HSA_VEN_AMD_AQLPROFILE_BLOCK_NAME_SPI; };
    if (std::any_of(a.events.begin(), a.events.end(), spi)) {
      std::vector<hsa_ven_amd_aqlprofile_event_t> ev;
      std::vector<int> ctr;
      for (size_t i = 0; i < a.events.size(); ++i)
        if (!spi(a.events[i])) {
          ev.push_back(a.events[i]);
          ctr.push_back(a.event_ctr[i]);
        }
      a.events.swap(ev);
      a.event_ctr.swap(ctr);
      a.profile.events = a.events.data();
      a.profile.event_count = uint32_t(a.events.size());
      std::fprintf(stderr, "[aqlpmc] gpu %s: aqlprofile refused the SPI events; counting without them\n",
                   a.bdf.c_str());
    }
    if (g_aql.hsa_ven_amd_aqlprofile_start(&a.profile, &a.start_pkt) != HSA_STATUS_SUCCESS) {
      *why = "aqlprofile start packet generation failed";
      return false;
    }
  }
  crumb("start packet ok");
  if (g_aql.hsa_ven_amd_aqlprofile_stop(&a.profile, &a.stop_pkt) != HSA_STATUS_SUCCESS) {
    *why = "aqlprofile stop packet generation failed";
    return false;
  }
  crumb("stop packet ok");
  if (g_aql.hsa_ven_amd_aqlprofile_read(&a.profile, &a.read_pkt) != HSA_STATUS_SUCCESS) {
    *why = "aqlprofile read packet generation failed";
    return false;
  }
  a.out_size = out_size;
  a.cmd_size = cmd_size;
  if (!ops.create_queue(&a.queue)) {
    *why = "hsa_queue_create failed";
    return false;
  }
  crumb("queue created");
  if (!ops.create_signal(&a.sig)) {
    *why = "hsa_signal_create failed";
    return false;
  }
  crumb("queue+signal ready; probing one window");
  // Probe one empty window: proves the queue executes the PM4 programs.
  if (run_packet(a, a.start_pkt) == Clock::time_point{} || run_packet(a, a.read_pkt) == Clock::time_point{} ||
      run_packet(a, a.stop_pkt) == Clock::time_point{}) {
    a.broken = true;
    *why = "PM4 start/stop packet did not complete (PMCs unavailable?)";
    return false;
  }
  a.ready = true;
  return true;
}

bool usable(const Agent* a) { return a && a->ready && !a->broken.load(); }

// Reads the output buffer the last read packet on queue q filled: reduced value + instances per
// counter.  The first queue's reads land in the agent's profile buffer, the rescue queue's in
// the rescue profile's.
bool collect(Agent& a, int q, Accum* acc) {
  *acc = Accum{};
  acc->a = &a;
  auto* prof = q == 1 ? &a.rprofile : &a.profile;
  const bool ok = g_aql.hsa_ven_amd_aqlprofile_iterate_data(prof, on_data, acc) == HSA_STATUS_SUCCESS;
  // per-XCC only when every sample of both counters has an XCC, both agree on the XCC count
  // and every XCC has as many SQ samples (SEs) as the first
  bool even = acc->xm_n > 0;
  for (int x = 1; x < acc->xm_n; ++x) even = even && acc->xm_cnt[x] == acc->xm_cnt[0];
  acc->nxcc = !acc->x_unmapped && even && acc->xm_n == acc->xg_n ? acc->xm_n : 0;
  if (g_debug) {
    std::string xs;
    for (int k = 0; k < 2; ++k) {
      xs += k ? ";grbm_samples=" : "mfma_samples=";
      for (int j = 0; j < acc->xs_n[k]; ++j) {
        char t[64];
        std::snprintf(t, sizeof(t), "%s%u@%d:%.0f", j ? "," : "", acc->xs[k][j].id, acc->xs[k][j].xcc,
                      acc->xs[k][j].v);
        xs += t;
      }
    }
    std::lock_guard<std::mutex> lk(a.dbg_mu);
    a.last_xsamples = std::move(xs);
  }
  return ok;
}

gpuexp_pmc::Sample to_sample(const Accum& acc) {
  gpuexp_pmc::Sample s;
  std::memcpy(s.v, acc.v, sizeof(s.v));
  std::memcpy(s.inst, acc.inst, sizeof(s.inst));
  s.samples = acc.samples;
  std::memcpy(s.xm, acc.xm, sizeof(s.xm));
  std::memcpy(s.xg, acc.xg, sizeof(s.xg));
  s.nxcc = acc.nxcc;
  return s;
}

// ---- ReadPort on HSA: every call comes from the read machine under its round lock ----
void Agent::post_read(int q) {
  if (q == 1) {
    hsa_signal_store_relaxed(rsig, 1);
    submit_on(*this, rq, rsig, rread_pkt, /*barrier=*/false);
  } else {
    hsa_signal_store_relaxed(sig, 1);
    submit_on(*this, queue, sig, read_pkt, /*barrier=*/false);
  }
}

// Start program, then (cumulative) the baseline read behind a barrier; one completion signal,
// on the last packet.  No wait: the machine looks at the signal in its rounds.
void Agent::post_arm(bool baseline_read) {
  hsa_signal_store_relaxed(sig, 1);
  if (baseline_read) {
    submit_on(*this, queue, hsa_signal_t{0}, start_pkt, /*barrier=*/true);
    submit_on(*this, queue, sig, read_pkt, /*barrier=*/true);
  } else {
    submit_on(*this, queue, sig, start_pkt, /*barrier=*/true);
  }
}

void Agent::post_start() { submit_on(*this, queue, hsa_signal_t{0}, start_pkt, /*barrier=*/true); }

void Agent::post_stop(int q) {
  hsa_signal_t s = q == 1 ? rsig : sig;
  hsa_signal_store_relaxed(s, 1);
  submit_on(*this, q == 1 ? rq : queue, s, stop_pkt, /*barrier=*/true);
}

bool Agent::done(int q) { return hsa_signal_load_scacquire(q == 1 ? rsig : sig) < 1; }

bool Agent::collect(int q, gpuexp_pmc::Sample* out) {
  Accum acc;
  if (!::collect(*this, q, &acc)) return false;
  *out = to_sample(acc);
  return true;
}

// Read rescue.  The sentinel shares the counters' queue (one ~173 MiB context-save area per
// GPU instead of two), and the packet processor does not look past a kernel dispatch whose
// waves cannot be placed: a workload holding every wave slot for seconds (measured: 8
// blocks x 4 waves per CU issuing MFMAs, tools/mfma_calibration.py --starve) holds every
// read behind the sentinel run, and the counters go stale exactly when the GPU is busiest.
// After rescue_rounds stuck rounds the read machine moves reads to a second queue of their own:
// the counters are chip state, so a read packet from any queue copies the same running totals
// (cumulative mode only: there a read changes nothing, and the abandoned read on the first
// queue, which still runs once the sentinel does, is harmless).  The second queue and its
// ~173 MiB context-save area exist only while a GPU needs them (measured: the first queue
// drains 0.8 s after a 6 s starvation, profiles/r03/sentinel_starvation.txt).
// GPUEXP_PMC_READ_RESCUE=0 disables.
bool Agent::open_rescue() {
  HsaOps ops{this};
  rprofile = profile;
  const bool ok = gpuexp_pmc::open_rescue(ops, *this, cmd_size, out_size, [this] {
    rprofile.command_buffer = {rcmd_buf, cmd_size};
    rprofile.output_buffer = {rout_buf, out_size};
    // the start program is generated (the read program is built after it) but never run:
    // it would re-program and reset the running counters
    return g_aql.hsa_ven_amd_aqlprofile_start(&rprofile, &rstart_pkt) == HSA_STATUS_SUCCESS &&
           g_aql.hsa_ven_amd_aqlprofile_read(&rprofile, &rread_pkt) == HSA_STATUS_SUCCESS;
  });
  return ok;
}

// Releases the rescue queue (its context-save area), its signal and buffers.
void Agent::close_rescue() {
  HsaOps ops{this};
  gpuexp_pmc::close_rescue(ops, *this);
}

// Duty-cycled windows: start, sleep(window), read, stop on every GPU, one window per interval.
void window_all(gpuexp_pmc::RoundMachine& m) {
  std::vector<Clock::time_point> t0(g_agents.size());
  for (size_t i = 0; i < g_agents.size(); ++i) {
    Agent* a = g_agents[i];
    if (!usable(a)) continue;
    if (g_debug) std::memset(a->out_buf, 0x5A, a->out_size);  // unwritten samples show as 0x5A5A..
    t0[i] = run_packet(*a, a->start_pkt);
    if (t0[i] == Clock::time_point{}) a->broken = true;
  }
  std::unique_lock<std::mutex> wl(g_cv_mu);
  g_cv.wait_for(wl, std::chrono::milliseconds(g_window_ms), [] { return g_quit.load(); });
  wl.unlock();
  for (size_t i = 0; i < g_agents.size(); ++i) {
    Agent* a = g_agents[i];
    if (!usable(a) || t0[i] == Clock::time_point{}) continue;
    // The read packet copies the counters to the output buffer (measured: the stop packet
    // alone leaves it untouched); stop then disables counting until the next window.
    const auto t1 = run_packet(*a, a->read_pkt);
    if (t1 == Clock::time_point{} || run_packet(*a, a->stop_pkt) == Clock::time_point{}) {
      a->broken = true;
      continue;
    }
    Accum acc;
    if (!collect(*a, 0, &acc)) continue;
    m.publish_window(int(i), acc.v, to_sample(acc), std::chrono::duration<double>(t1 - t0[i]).count());
  }
}

// What does a read packet do to running counters?  start, 20 ms, read (B), then at once a
// second read (C), on GRBM_COUNT (the GRBM clock count, which always advances while
// counting):
//   C == B exactly      -> the read stopped counting;
//   C >  B              -> cumulative (C = B + the few microseconds between the reads);
//   C <  B / 2          -> each read resets (C counts only those few microseconds).
// Only the ORDER of B and C decides, never a ratio to elapsed time: GRBM_COUNT runs at the
// current GFX clock, which DPM moves by 5x between idle and busy (a ratio test misread a
// GPU clocking down after a workload as "resets").  Anything else: unknown.
ReadMode read_semantics(Agent& a, std::string* why) {
  const auto ts = run_packet(a, a.start_pkt);
  double c[2] = {0, 0};
  for (int i = 0; i < 2; ++i) {
    if (i == 0) std::this_thread::sleep_for(std::chrono::milliseconds(20));
    const auto t = run_packet(a, a.read_pkt);
    Accum acc;
    if (ts == Clock::time_point{} || t == Clock::time_point{} || !collect(a, 0, &acc)) {
      *why = "PM4 read packet did not complete";
      return kReadUnknown;
    }
    c[i] = acc.v[kGrbmCount];
  }
  run_packet(a, a.stop_pkt);
  crumb("read semantics", "GRBM_COUNT B=" + std::to_string(c[0]) + " C=" + std::to_string(c[1]));
  if (c[0] <= 0) {
    *why = "GRBM_COUNT did not advance after the start packet";
    return kReadUnknown;
  }
  if (c[1] == c[0]) return gpuexp_pmc::kStops;
  if (c[1] > c[0]) return kCumulative;
  if (c[1] < 0.5 * c[0]) return kResets;
  *why = "read packet semantics unclear (GRBM_COUNT " + std::to_string(c[0]) + " then " + std::to_string(c[1]) + ")";
  return kReadUnknown;
}

void duty_loop(gpuexp_pmc::RoundMachine* m) {
  ::prctl(PR_SET_NAME, "gpuexp-pmc", 0, 0, 0);
  while (!g_quit.load()) {
    const auto begin = Clock::now();
    window_all(*m);
    g_thread_cpu_ns.store(own_cpu_ns());
    const auto spent = std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - begin).count();
    std::unique_lock<std::mutex> lk(g_cv_mu);
    g_cv.wait_for(lk, std::chrono::milliseconds(std::max<long long>(0, g_interval_ms - spent)),
                  [] { return g_quit.load(); });
  }
}

void teardown_locked() {
  for (Agent* a : g_agents) {
    if (!a) continue;
    // A timed-out (or still queued, or abandoned and never run) packet may still write the
    // buffers: the read machine marks such a GPU broken at its stop, and they are left.
    HsaOps ops{a};
    gpuexp_pmc::release_agent(ops, *a, a->broken.load());
    delete a;
  }
  g_agents.clear();
  if (g_hsa_up) hsa_shut_down();
  g_hsa_up = false;
}

// Read-machine settings from the environment (docs/CONFIG.md "PMC read machine").
gpuexp_pmc::MachineConfig machine_config(ReadMode mode) {
  gpuexp_pmc::MachineConfig c;
  c.mode = mode;
  c.interval_ms = g_interval_ms;
  c.inline_rounds = g_inline;
  const char* e = std::getenv("GPUEXP_PMC_READ_RESCUE");
  c.rescue = !(e && e[0] == '0');
  if (const char* r = std::getenv("GPUEXP_PMC_REARM")) {
    const std::string v = r;
    c.rearm.mode = v == "off" || v == "0" ? gpuexp_ctr::kRearmOff
                   : v == "now"           ? gpuexp_ctr::kRearmNow
                                          : gpuexp_ctr::kRearmBackoff;
  }
  if (const char* b = std::getenv("GPUEXP_PMC_REARM_BACKOFF_MS")) {
    const long ms = std::strtol(b, nullptr, 10);
    if (ms > 0) c.rearm.base_ns = int64_t(ms) * 1000000ll;
  }
  return c;
}

// ---------------------------------------------------------------------------------------
// Sentinel on the counters' queue.  Every GPU queue pins a context save/restore area sized
// for the whole GPU (~173 MiB on MI355X), so instead of the HIP plugin's own stream the
// sentinel kernel (gpuexp_sentinel.hsaco, same device code: sentinel_device.h) is
// dispatched here as raw AQL packets on the queue the PMC programs already use.
// ---------------------------------------------------------------------------------------
struct KernelSym {
  uint64_t object = 0;
  uint32_t kernarg = 0, group = 0, priv = 0;
};

std::string plugin_dir() {
  Dl_info info{};
  if (::dladdr(reinterpret_cast<void*>(&plugin_dir), &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    const size_t sl = p.rfind('/');
    return sl == std::string::npos ? std::string(".") : p.substr(0, sl);
  }
  return ".";
}

bool lookup(hsa_executable_t exe, hsa_agent_t gpu, const char* name, KernelSym* k) {
  hsa_executable_symbol_t sym{};
  if (hsa_executable_get_symbol_by_name(exe, name, &gpu, &sym) != HSA_STATUS_SUCCESS) return false;
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->object);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kernarg);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->group);
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->priv);
  return k->object != 0;
}

hsa_status_t pick_uncached_pool(hsa_amd_memory_pool_t pool, void* data) {
  hsa_amd_segment_t seg{};
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  bool alloc = false;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  if (seg == HSA_AMD_SEGMENT_GLOBAL && alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) {
    *static_cast<hsa_amd_memory_pool_t*>(data) = pool;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// One kernel dispatch packet (1-D grid of `groups` x `wg` lanes) on the agent's queue.
void dispatch(Agent& a, const KernelSym& k, void* kernarg, uint32_t groups, hsa_signal_t done, uint16_t wg = 64) {
  std::lock_guard<std::mutex> lk(a.submit_mu);
  hsa_queue_t* q = a.queue;
  const uint64_t idx = hsa_queue_add_write_index_screlease(q, 1);
  auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
  pkt->workgroup_size_x = wg;
  pkt->workgroup_size_y = 1;
  pkt->workgroup_size_z = 1;
  pkt->grid_size_x = groups * wg;
  pkt->grid_size_y = 1;
  pkt->grid_size_z = 1;
  pkt->private_segment_size = k.priv;
  pkt->group_segment_size = k.group;
  pkt->kernel_object = k.object;
  pkt->kernarg_address = kernarg;
  pkt->completion_signal = done;
  pkt->reserved0 = 0;
  pkt->reserved2 = 0;  // the slot may have held a PM4 packet with another layout
  const uint16_t header = uint16_t((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                   (1 << HSA_PACKET_HEADER_BARRIER) |
                                   (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                   (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  const uint16_t setup = uint16_t(1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS);
  __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), uint32_t(header) | (uint32_t(setup) << 16), __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, hsa_signal_value_t(idx));
}

class QueueSentinel : public gpuexp::SentinelSource {
  struct Per {
    Agent* a = nullptr;
    bool ready = false;
    hsa_executable_t exe{};
    bool have_exe = false;
    KernelSym run_k, init_k;
    char* kernargs = nullptr;  // one 64-byte slot per ring slot
    uint32_t* chase = nullptr;
    int hops = 0;
    gpuexp::SentinelRun run;
  };

 public:
  QueueSentinel(int ring, int spin) : nslots_(ring < 4 ? 4 : ring), spin_(spin < 16 ? 16 : spin) {}
  ~QueueSentinel() override { stop(); }

  bool start(const std::vector<gpuexp::DeviceInfo>& devs, std::string* err) override {
    const std::string path = plugin_dir() + "/gpuexp_sentinel.hsaco";
    uint64_t freq = 0;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &freq);
    sys_ns_per_tick_ = freq ? 1e9 / double(freq) : 1.0;
    std::vector<Agent*> agents;
    {
      std::lock_guard<std::mutex> lk(g_mu);
      agents = g_agents;
    }
    per_.resize(devs.size());
    int ok = 0, waves = 0;
    std::string why = "no GPU has a working PMC queue";
    for (size_t i = 0; i < devs.size() && i < agents.size(); ++i) {
      Agent* a = agents[i];
      if (!a || !a->ready || a->broken) continue;
      Per& p = per_[i];
      p.a = a;
      if (!setup(p, path, int(devs[i].num_xcc), &why)) {
        release(p);
        continue;
      }
      p.ready = true;
      ++ok;
      waves += p.run.waves;
    }
    if (!ok) {
      *err = why;
      return false;
    }
    status_ = "hsa sentinel on " + std::to_string(ok) + " GPU(s) (on the PMC queue: one GPU queue per GPU), " +
              std::to_string(waves) + " waves/tick (one per XCD), ring " + std::to_string(nslots_);
    return true;
  }

  void tick(uint64_t) override {
    for (Per& p : per_) {
      if (!p.ready || p.a->broken || p.a->queue_error.load()) continue;
      gpuexp::sentinel_drain(p.run, nslots_, sys_ns_per_tick_);
      // one run at a time: a run the workload leaves no SIMD for waits (and shows its wait as
      // dispatch latency once it runs) without a second one queued behind it
      if (p.run.launched - p.run.completed >= 1) {
        p.run.stalled += 1;
        continue;
      }
      const uint64_t seq = p.run.launched + 1;
      const uint32_t slot = gpuexp::sentinel_prepare(p.run, seq, nslots_);
      gpuexp::SentinelArgs args{p.run.ring, p.chase, seq, slot, spin_, p.hops, 0};
      char* ka = p.kernargs + size_t(slot) * 64;
      std::memcpy(ka, &args, sizeof(args));
      dispatch(*p.a, p.run_k, ka, uint32_t(p.run.waves), hsa_signal_t{0});
      p.run.launched = seq;
      p.run.fresh_seq = seq;
    }
  }

  bool read(int dev, gpuexp::SentinelReading* out) override {
    if (dev < 0 || size_t(dev) >= per_.size() || !per_[size_t(dev)].ready) return false;
    Per& p = per_[size_t(dev)];
    // every tick (the sampler's thread, like tick()): a completed run is folded in and the
    // outstanding one's pending time is current -- the launches alone run at most every
    // sentinel_min_interval, and a pending time sampled only then read in 0.5 s steps
    if (p.a->broken || p.a->queue_error.load()) return gpuexp::sentinel_fill(p.run, out);
    return gpuexp::sentinel_read(p.run, nslots_, sys_ns_per_tick_, out);
  }

  void stop() override {
    for (Per& p : per_) {
      if (p.ready) {
        // a run is microseconds long: wait (bounded) for the in-flight ones before freeing
        for (int i = 0; i < 200 && p.run.completed < p.run.launched; ++i) {
          gpuexp::sentinel_drain(p.run, nslots_, sys_ns_per_tick_);
          if (p.run.completed < p.run.launched) ::usleep(500);
        }
        if (p.run.completed < p.run.launched) continue;  // GPU may still write: leak, do not free
      }
      release(p);
    }
    per_.clear();
  }

  std::string status() const override { return status_; }

 private:
  bool setup(Per& p, const std::string& path, int num_xcc, std::string* why) {
    Agent& a = *p.a;
    const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      *why = "cannot open " + path;
      return false;
    }
    hsa_code_object_reader_t reader{};
    bool ok = hsa_code_object_reader_create_from_file(fd, &reader) == HSA_STATUS_SUCCESS;
    if (ok) {
      ok = hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &p.exe) ==
           HSA_STATUS_SUCCESS;
      p.have_exe = ok;
      ok = ok && hsa_executable_load_agent_code_object(p.exe, a.gpu, reader, nullptr, nullptr) == HSA_STATUS_SUCCESS;
      ok = ok && hsa_executable_freeze(p.exe, nullptr) == HSA_STATUS_SUCCESS;
      hsa_code_object_reader_destroy(reader);
    }
    ::close(fd);
    if (!ok || !lookup(p.exe, a.gpu, "gpuexp_sentinel.kd", &p.run_k) ||
        !lookup(p.exe, a.gpu, "gpuexp_sentinel_init_chase.kd", &p.init_k) ||
        p.run_k.kernarg > 64 || p.init_k.kernarg > 64) {
      *why = "cannot load the sentinel code object " + path;
      return false;
    }
    p.run.waves = num_xcc > 0 ? std::min(num_xcc, gpuexp::kSentinelMaxWaves) : gpuexp::kSentinelMaxWaves;
    p.run.ring = static_cast<gpuexp::SentinelSlot*>(
        sys_alloc(sizeof(gpuexp::SentinelSlot) * size_t(nslots_) * gpuexp::kSentinelMaxWaves, a.gpu));
    p.kernargs = static_cast<char*>(sys_alloc(size_t(nslots_ + 1) * 64, a.gpu));
    if (!p.run.ring || !p.kernargs) {
      *why = "sentinel ring allocation failed";
      return false;
    }
    p.run.host_launch.assign(size_t(nslots_), 0);
    p.run.agent = a.gpu;
    p.run.have_agent = true;
    // HBM latency chain in uncached device memory, written by a kernel (no copy queue)
    hsa_amd_memory_pool_t pool{};
    hsa_amd_agent_iterate_memory_pools(a.gpu, pick_uncached_pool, &pool);
    void* chase = nullptr;
    const size_t bytes = size_t(gpuexp::kChaseHops) * gpuexp::kChaseStride * sizeof(uint32_t);
    if (pool.handle &&
        hsa_amd_memory_pool_allocate(pool, bytes, HSA_AMD_MEMORY_POOL_UNCACHED_FLAG, &chase) == HSA_STATUS_SUCCESS) {
      hsa_signal_t done{};
      if (hsa_signal_create(1, 0, nullptr, &done) == HSA_STATUS_SUCCESS) {
        gpuexp::SentinelInitArgs ia{static_cast<uint32_t*>(chase), gpuexp::kChaseHops, 0};
        char* ka = p.kernargs + size_t(nslots_) * 64;  // the spare slot
        std::memcpy(ka, &ia, sizeof(ia));
        dispatch(a, p.init_k, ka, 1, done);
        if (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, g_ts_freq, HSA_WAIT_STATE_BLOCKED) < 1) {
          p.chase = static_cast<uint32_t*>(chase);
          p.hops = gpuexp::kChaseHops;
        }
        hsa_signal_destroy(done);
      }
      if (!p.chase) hsa_amd_memory_pool_free(chase);
    }
    return true;
  }

  void release(Per& p) {
    if (p.chase) hsa_amd_memory_pool_free(p.chase);
    if (p.kernargs) hsa_amd_memory_pool_free(p.kernargs);
    if (p.run.ring) hsa_amd_memory_pool_free(p.run.ring);
    if (p.have_exe) hsa_executable_destroy(p.exe);
    p = Per();
  }

  int nslots_;
  int spin_;
  double sys_ns_per_tick_ = 1.0;
  std::vector<Per> per_;
  std::string status_ = "not started";
};
}  // namespace

extern "C" __attribute__((visibility("default"))) void gpuexp_rp_set_duty(int window_ms, int interval_ms) {
  g_continuous = false;
  g_window_ms = std::max(1, window_ms);
  g_interval_ms = std::max(g_window_ms, interval_ms);
}

// Inline rounds (before gpuexp_rp_init): the caller of gpuexp_rp_kick / gpuexp_rp_sync runs
// each round itself.  Only for an engine that kicks every tick: with sparse manual ticks the
// counting thread's own rounds keep the windows short (thread mode).
extern "C" __attribute__((visibility("default"))) void gpuexp_rp_set_inline(int on) { g_inline = on != 0; }

// Continuous counting: started once, read once per gpuexp_rp_kick (one engine tick), or
// every `fallback_ms` when nothing kicks.
extern "C" __attribute__((visibility("default"))) void gpuexp_rp_set_continuous(int fallback_ms) {
  g_continuous = true;
  g_interval_ms = std::max(10, fallback_ms);
}

extern "C" __attribute__((visibility("default"))) void gpuexp_rp_kick() {
  if (auto* m = g_machine.load()) m->kick();
}

// CPU time the counting thread (continuous) or duty thread has used so far (charged to the
// engine's sampler account).
extern "C" __attribute__((visibility("default"))) uint64_t gpuexp_rp_cpu_ns() {
  auto* m = g_machine.load();
  return g_continuous && m ? m->thread_cpu_ns() : g_thread_cpu_ns.load();
}

// Waits up to `timeout_us` for the round of the last kick; 0 = done, 1 = timed out.
extern "C" __attribute__((visibility("default"))) int gpuexp_rp_sync(int timeout_us) {
  auto* m = g_machine.load();
  return m ? m->sync(timeout_us) : 0;
}

extern "C" __attribute__((visibility("default"))) int gpuexp_rp_init(int ndev, const char* const* bdfs, char* err,
                                                                     int errlen) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto fail = [&](const std::string& m) {
    std::snprintf(err, size_t(errlen), "%s", m.c_str());
    g_status = "unavailable: " + m;
    return 0;
  };
  if (g_hsa_up) return fail("already initialised");
  g_debug = std::getenv("GPUEXP_AQLPMC_DEBUG") != nullptr;
  if (g_debug) ::signal(SIGSEGV, segv_backtrace);

  if (hsa_init() != HSA_STATUS_SUCCESS) return fail("hsa_init failed");
  g_hsa_up = true;
  crumb("hsa_init ok");
  if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_AQLPROFILE, hsa_ven_amd_aqlprofile_VERSION_MAJOR,
                                           sizeof(g_aql), &g_aql) != HSA_STATUS_SUCCESS ||
      !g_aql.hsa_ven_amd_aqlprofile_start) {
    teardown_locked();
    return fail("HSA runtime did not provide the aqlprofile extension table");
  }
  crumb("aqlprofile table ok");
  hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &g_ts_freq);
  Found f;
  hsa_iterate_agents(collect_agent, &f);
  for (auto cpu : f.cpus) {
    hsa_amd_agent_iterate_memory_pools(cpu, pick_sys_pool, nullptr);
    if (g_have_pool) break;
  }
  if (!g_have_pool) {
    teardown_locked();
    return fail("no fine-grained system memory pool");
  }
  g_agents.assign(size_t(std::max(0, ndev)), nullptr);
  int ok = 0;
  std::string why;
  // Partitioned sockets (CPX/DPX/QPX) expose several agents with one BDF, in partition
  // order, as do the exporter's devices: the k-th device gets the k-th free agent
  // (pmc_agents.h match_agents).  A GPU whose setup fails keeps its slot, unusable.
  std::vector<std::string> gpu_bdfs;
  for (const auto& g : f.gpus) gpu_bdfs.push_back(g.second);
  const gpuexp_pmc::AgentMatch match = gpuexp_pmc::match_agents(ndev, bdfs, gpu_bdfs);
  const int disabled = match.n_reserved;
  for (int d = 0; d < ndev; ++d) {
    const int gi = match.gpu_of[size_t(d)];
    if (gi < 0) continue;
    auto* a = new Agent;
    a->dev = d;
    a->gpu = f.gpus[size_t(gi)].first;
    a->bdf = f.gpus[size_t(gi)].second;
    g_agents[size_t(d)] = a;
    if (setup_agent(*a, &why)) ++ok;
  }
  if (!ok) {
    teardown_locked();
    return fail(why.empty() ? (disabled ? "every GPU excluded by queue_devices"
                                        : "no HSA GPU agent matched the exporter's GPUs")
                            : why);
  }
  if (g_continuous) {
    // probe the read packet's effect once (first working GPU), then arm every GPU
    g_read_mode = kReadUnknown;
    for (Agent* a : g_agents) {
      if (!usable(a)) continue;
      g_read_mode = read_semantics(*a, &why);
      break;
    }
    if (g_read_mode == kReadUnknown) {
      // counting still works window by window: fall back to the duty cycle (status says so)
      std::fprintf(stderr, "[aqlpmc] continuous counting unavailable (%s): duty-cycled windows instead\n",
                   why.c_str());
      g_continuous = false;
      g_window_ms = std::max(1, std::min(20, g_interval_ms / 2));
    }
  }
  if (const char* e = std::getenv("GPUEXP_PMC_INLINE")) g_inline = e[0] != '0';
  auto* m = new gpuexp_pmc::RoundMachine(machine_config(g_continuous ? g_read_mode : kReadUnknown));
  for (Agent* a : g_agents) m->add(usable(a) ? a : nullptr, a ? a->model : Derived{});
  if (g_continuous) {
    ok = 0;
    for (int d = 0; d < ndev; ++d)
      if (usable(g_agents[size_t(d)]) && m->arm_sync(d)) ++ok;
    if (!ok) {
      delete m;
      teardown_locked();
      return fail("continuous counting: start/read packets did not complete");
    }
  }
  g_quit.store(false);
  g_machine.store(m);
  if (g_continuous) m->start();
  else g_thread = std::thread(duty_loop, m);
  g_status = "aqlprofile PMC on " + std::to_string(ok) + " GPU(s), " +
             (g_continuous ? std::string("continuous (one read per tick; read packets: ") +
                                 read_mode_name(g_read_mode) + (g_inline ? "; rounds run by the sampler" : "") + ")"
                           : std::to_string(g_window_ms) + " ms window every " + std::to_string(g_interval_ms) +
                                 " ms");
  return ok;
}

extern "C" __attribute__((visibility("default"))) int gpuexp_rp_sample(int dev, double, double* out) {
  auto* m = g_machine.load();
  return m ? m->sample(dev, out) : -1;
}

// Per-XCC MFMA busy of the window gpuexp_rp_sample returns: fills out[0..n) and returns n
// (the GPU's XCC count), or 0 when the samples' XCC coordinates are unknown / no window.
extern "C" __attribute__((visibility("default"))) int gpuexp_rp_sample_xcc(int dev, double* out, int max) {
  auto* m = g_machine.load();
  return m ? m->sample_xcc(dev, out, max) : 0;
}

extern "C" __attribute__((visibility("default"))) void gpuexp_rp_shutdown() {
  std::lock_guard<std::mutex> lk(g_mu);
  auto* m = g_machine.exchange(nullptr);
  if (m) m->stop();  // joins the counting thread, stops counting (bounded)
  g_quit.store(true);
  g_cv.notify_all();
  if (g_thread.joinable()) g_thread.join();
  delete m;
  teardown_locked();
  g_status = "shut down";
}

extern "C" __attribute__((visibility("default"))) const char* gpuexp_rp_status() { return g_status.c_str(); }

// Read health of one GPU (gpuexp::CounterHealth order): stalls, resets, rearms, rescues,
// rescue releases, rescue active.  0, or -1 for an unknown device.
extern "C" __attribute__((visibility("default"))) int gpuexp_rp_health(int dev, uint64_t* out, int n) {
  auto* m = g_machine.load();
  gpuexp_pmc::Health h;
  if (!m || n < 6 || !m->health(dev, &h)) return -1;
  out[0] = h.stalls;
  out[1] = h.resets;
  out[2] = h.rearms;
  out[3] = h.rescues;
  out[4] = h.releases;
  out[5] = h.rescue_active ? 1 : 0;
  return 0;
}

extern "C" __attribute__((visibility("default"))) int gpuexp_rp_scope(int dev) {
  auto* m = g_machine.load();
  return m ? m->scope(dev) : -1;
}

// Diagnostics: the reduced value and instance count of every counter in the last window,
// as "NAME=value/instances;..." (used by tools/gpu_features_check.py).
extern "C" __attribute__((visibility("default"))) int gpuexp_rp_debug(int dev, char* buf, int len) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto* m = g_machine.load();
  if (!m || dev < 0 || size_t(dev) >= g_agents.size() || !g_agents[size_t(dev)]) return -1;
  Agent& a = *g_agents[size_t(dev)];
  std::string s = "backend=aqlprofile;events=" + std::to_string(a.events.size()) + ";" + m->debug(dev);
  {
    std::lock_guard<std::mutex> dk(a.dbg_mu);
    s += "coords=" + a.coord_names + ";";
    if (!a.last_xsamples.empty()) s += a.last_xsamples + ";";
  }
  std::snprintf(buf, size_t(len), "%s", s.c_str());
  return 0;
}

// ---------------------------------------------------------------------------------------
// Calibration (tests/test_gpu.py::test_device_scope_pmc_calibration, tools/pmc_validate.py).
// An unprivileged process's agent-mode SQ/TCC counters count only the dispatches of the
// queue that programs them (profiles/r02/pmc_scope.txt), so known work is dispatched HERE,
// on the PMC queue, while the counting windows run:
//   kind 0: stream copy of 1 GiB (gpuexp_calib_copy): HBM read = write = 1 GiB per launch
//   kind 1: conflict-free LDS reads; kind 2: the same reads 32-way bank-conflicted
// 4096 blocks x 4 waves per launch, at most 4 launches queued so the windows' PM4 packets
// never wait long behind them.  out[0] = seconds, out[1] = waves per launch,
// out[2] = HBM bytes read per launch.  Returns 0, or -1 (see stderr).
// ---------------------------------------------------------------------------------------
extern "C" __attribute__((visibility("default"))) int gpuexp_rp_calibrate(int dev, int kind, int launches,
                                                                          double* out) {
  Agent* a = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (dev >= 0 && size_t(dev) < g_agents.size()) a = g_agents[size_t(dev)];
  }
  auto fail = [](const char* why) {
    std::fprintf(stderr, "[aqlpmc] calibrate: %s\n", why);
    return -1;
  };
  if (!a || !a->ready || a->broken) return fail("no working PMC queue for this device");
  if (kind < 0 || kind > 4 || launches < 1 || launches > 1000000) return fail("bad arguments");
  const std::string path = plugin_dir() + "/gpuexp_calib.hsaco";
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return fail("cannot open gpuexp_calib.hsaco");
  hsa_code_object_reader_t reader{};
  hsa_executable_t exe{};
  bool have_exe = false;
  bool ok = hsa_code_object_reader_create_from_file(fd, &reader) == HSA_STATUS_SUCCESS;
  if (ok) {
    have_exe = hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr,
                                         &exe) == HSA_STATUS_SUCCESS;
    ok = have_exe && hsa_executable_load_agent_code_object(exe, a->gpu, reader, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
         hsa_executable_freeze(exe, nullptr) == HSA_STATUS_SUCCESS;
    hsa_code_object_reader_destroy(reader);
  }
  ::close(fd);
  KernelSym k;
  // kinds: 0 stream copy, 1 / 2 LDS reads (conflict-free / 32-way), 3 / 4 fixed MFMA work (bf16 / fp8)
  const char* sym = kind == 0 ? "gpuexp_calib_copy.kd" : kind <= 2 ? "gpuexp_calib_lds.kd" : "gpuexp_calib_mfma.kd";
  ok = ok && lookup(exe, a->gpu, sym, &k) && k.kernarg <= 64;
  if (!ok) {
    if (have_exe) hsa_executable_destroy(exe);
    return fail("cannot load the calibration code object");
  }
  constexpr uint32_t kBlocks = 4096;
  constexpr size_t kCopyBytes = size_t(1) << 30;
  hsa_amd_memory_pool_t pool{};
  hsa_amd_agent_iterate_memory_pools(a->gpu, pick_uncached_pool, &pool);
  void* buf = nullptr;
  constexpr uint32_t kMfmaIters = 4096;  // ~3 ms per launch on MI355X at the bf16 rate
  const size_t bytes = kind == 0 ? 2 * kCopyBytes : kBlocks * (gpuexp::kProbeBlock / 64) * sizeof(float);
  char* ka = static_cast<char*>(sys_alloc(64, a->gpu));
  hsa_signal_t sig{};
  if (!pool.handle || hsa_amd_memory_pool_allocate(pool, bytes, 0, &buf) != HSA_STATUS_SUCCESS || !ka ||
      hsa_amd_agents_allow_access(1, &a->gpu, nullptr, buf) != HSA_STATUS_SUCCESS ||
      hsa_signal_create(launches, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) {
    if (buf) hsa_amd_memory_pool_free(buf);
    if (ka) hsa_amd_memory_pool_free(ka);
    hsa_executable_destroy(exe);
    return fail("allocation failed");
  }
  if (kind == 0) {
    gpuexp::CalibCopyArgs args{buf, static_cast<char*>(buf) + kCopyBytes, kCopyBytes / 16, uint64_t(kBlocks)};
    std::memcpy(ka, &args, sizeof(args));
  } else if (kind <= 2) {
    gpuexp::CalibLdsArgs args{static_cast<float*>(buf), 8192, kind == 2 ? 32 : 1};
    std::memcpy(ka, &args, sizeof(args));
  } else {
    gpuexp::CalibMfmaCountArgs args{static_cast<float*>(buf), kMfmaIters, uint32_t(kind - 3)};
    std::memcpy(ka, &args, sizeof(args));
  }
  const auto t0 = Clock::now();
  bool timed_out = false;
  for (int i = 0; i < launches && !timed_out; ++i) {
    // at most 4 in flight: wait until fewer than 4 of the i submitted are outstanding
    if (i >= 4)
      timed_out = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, hsa_signal_value_t(launches - i + 4),
                                            5 * g_ts_freq, HSA_WAIT_STATE_ACTIVE) >= launches - i + 4;
    if (!timed_out) dispatch(*a, k, ka, kBlocks, sig, uint16_t(gpuexp::kProbeBlock));
  }
  if (!timed_out)
    timed_out = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 30 * g_ts_freq,
                                          HSA_WAIT_STATE_BLOCKED) >= 1;
  const double secs = std::chrono::duration<double>(Clock::now() - t0).count();
  if (timed_out) {  // the GPU may still use the buffers: leak them
    a->broken = true;
    return fail("calibration dispatches did not complete");
  }
  hsa_signal_destroy(sig);
  hsa_amd_memory_pool_free(buf);
  hsa_amd_memory_pool_free(ka);
  hsa_executable_destroy(exe);
  out[0] = secs;
  out[1] = double(kBlocks) * (gpuexp::kProbeBlock / 64);
  // per launch: bytes copied (kind 0) or MFMA FLOPs issued (kinds 3, 4)
  out[2] = kind == 0 ? double(kCopyBytes)
           : kind >= 3 ? double(kBlocks) * (gpuexp::kProbeBlock / 64) * kMfmaIters * gpuexp::kMfmaCountChains *
                             gpuexp::kMfma32x32x16Flops
                       : 0.0;
  return 0;
}

// The sentinel on this plugin's PMC queues (see QueueSentinel); the engine asks for it after
// gpuexp_rp_init succeeded, and falls back to the HIP plugin's own stream otherwise.
extern "C" __attribute__((visibility("default"))) gpuexp::SentinelSource* gpuexp_make_hsa_sentinel(int ring_slots,
                                                                                                   int spin_iters) {
  return new QueueSentinel(ring_slots, spin_iters);
}
