// rocprofiler-sdk device-counting plugin (_gpuexp_rocprof.so), dlopen()ed by the core.
//
// BASELINE config 4 asks for MFMA / LDS counters per GPU at 10 Hz.  Shaders cannot read
// SQ/TCC performance counters (SURVEY.md §7.4 risk 2), so they come from the
// rocprofiler-sdk agent ("device") counting service: one context per GPU, one counter
// config that fits a single pass within the gfx950 per-block slot limits
// (MI355X_MICROARCH.md "rocprofv3 PMC slots": SQ 8, TCC 4, GRBM 2):
//   SQ   SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT
//   GRBM GRBM_GUI_ACTIVE GRBM_COUNT
//   TCC  TCC_BUBBLE TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_EA0_WRREQ_64B
// Derived per tick from deltas (formulas of counter_defs.yaml for gfx950: MfmaUtil,
// FETCH_SIZE, WRITE_SIZE, LDS util / bank-conflict ratio).  Counter values read by
// rocprofiler_sample_device_counting_service accumulate from context start; the plugin
// keeps the previous reading and treats a decrease as a restart.
//
// The tool registers with rocprofiler_force_configure() — it must run before the HSA
// runtime loads in this process, so the engine starts counters before the HIP sentinel.
// Any failure (non-root, PMCs owned by another profiler) leaves the engine without
// counter series; the other sources are unaffected.
//
// Measured cost (MI355X, ROCm 7.2): once this tool is registered and HSA is up, one HSA
// runtime thread (the async-signal loop: ioctl AMDKFD_IOC_WAIT_EVENTS returning at once,
// libhsa-runtime64 +0x13f7e7 <- +0x1357e4 <- +0x8b53a) spins a core at 100% whether or
// not a context is started — rocprofiler's agent completion handler waits on a signal with
// no interrupt event.  The default counter backend is therefore _gpuexp_aqlpmc.so
// (aql_pmc.cc), which submits the same PM4 packets on its own queue; this plugin stays
// selectable (counters_plugin=.../_gpuexp_rocprof.so) as the cross-check.
#include <hsa/hsa.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include "gpuexp/counter_model.h"
#include "gpuexp/sources.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

static_assert(gpuexp_ctr::kNumOut == gpuexp::kCounterOutputs, "counter plugin ABI");

namespace {

using namespace gpuexp_ctr;

struct Agent {
  rocprofiler_agent_id_t id{};
  int dev = -1;
  rocprofiler_context_id_t ctx{};
  rocprofiler_counter_config_id_t cfg{};
  bool have_cfg = false;
  bool started = false;
  std::map<uint64_t, int> counter_slot;  // counter id handle -> Ctr
  std::vector<rocprofiler_counter_record_t> recs;
  double last_raw[kNumCtr] = {};
  int last_inst[kNumCtr] = {};
  size_t last_nrec = 0;
  Derived m;
};

std::mutex g_mu;
std::vector<std::string> g_want_bdfs;
std::vector<Agent> g_agents;
std::string g_status = "not initialised";
std::string g_err;
bool g_configured = false;
rocprofiler_client_finalize_t g_fini = nullptr;
rocprofiler_client_id_t* g_client = nullptr;

std::string lower(std::string s) {
  for (auto& c : s) c = char(::tolower(c));
  return s;
}

void set_profile_cb(rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set_config,
                    void* user) {
  auto* a = static_cast<Agent*>(user);
  if (a && a->have_cfg) set_config(ctx, a->cfg);
}

int tool_init(rocprofiler_client_finalize_t fini, void*) {
  g_fini = fini;
  std::vector<rocprofiler_agent_v0_t> agents;
  auto cb = [](rocprofiler_agent_version_t ver, const void** arr, size_t n, void* ud) -> rocprofiler_status_t {
    if (ver != ROCPROFILER_AGENT_INFO_VERSION_0) return ROCPROFILER_STATUS_ERROR;
    auto* v = static_cast<std::vector<rocprofiler_agent_v0_t>*>(ud);
    for (size_t i = 0; i < n; ++i) {
      const auto* a = static_cast<const rocprofiler_agent_v0_t*>(arr[i]);
      if (a->type == ROCPROFILER_AGENT_TYPE_GPU) v->push_back(*a);
    }
    return ROCPROFILER_STATUS_SUCCESS;
  };
  if (rocprofiler_query_available_agents(ROCPROFILER_AGENT_INFO_VERSION_0, cb, sizeof(rocprofiler_agent_t),
                                         &agents) != ROCPROFILER_STATUS_SUCCESS) {
    g_err = "rocprofiler_query_available_agents failed";
    return -1;
  }
  g_agents.resize(g_want_bdfs.size());
  int matched = 0;
  for (const auto& a : agents) {
    char bdf[32];
    std::snprintf(bdf, sizeof(bdf), "%04x:%02x:%02x.%x", a.domain, (a.location_id >> 8) & 0xFF,
                  (a.location_id >> 3) & 0x1F, a.location_id & 0x7);
    for (size_t d = 0; d < g_want_bdfs.size(); ++d) {
      // several agents share a BDF on a partitioned socket: first free device slot wins
      const bool off = !g_want_bdfs[d].empty() && g_want_bdfs[d][0] == '-';  // queue_devices: reserve only
      if (lower(off ? g_want_bdfs[d].substr(1) : g_want_bdfs[d]) != bdf || g_agents[d].dev >= 0) continue;
      Agent& ag = g_agents[d];
      ag.id = a.id;
      ag.dev = int(d);
      if (off) break;
      ag.m.simd = a.simd_count;
      ag.m.privileged = pmc_device_scope();
      ag.m.cu = a.cu_count ? a.cu_count : (a.simd_per_cu ? a.simd_count / a.simd_per_cu : 0);
      // one agent per device slot (partitions of a socket share a BDF): stop at the first
      if (rocprofiler_create_context(&ag.ctx) != ROCPROFILER_STATUS_SUCCESS) break;
      rocprofiler_buffer_id_t nobuf{};  // values come back in the sample call itself
      if (rocprofiler_configure_device_counting_service(ag.ctx, nobuf, a.id, set_profile_cb, &ag) !=
          ROCPROFILER_STATUS_SUCCESS) {
        g_err = "configure_device_counting_service failed for " + std::string(bdf);
        break;
      }
      ++matched;
      break;
    }
  }
  g_configured = matched > 0;
  if (!matched && g_err.empty()) g_err = "no rocprofiler GPU agent matched the exporter's GPUs";
  return 0;
}

void tool_fini(void*) { g_configured = false; }

rocprofiler_tool_configure_result_t* configure(uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
  id->name = "gpuexp-device-counters";
  g_client = id;
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                 &tool_fini, nullptr};
  return &cfg;
}

// Builds the counter config for an agent, dropping counters the agent lacks.
bool build_config(Agent& a, std::string* why) {
  std::vector<rocprofiler_counter_id_t> all;
  rocprofiler_iterate_agent_supported_counters(
      a.id,
      [](rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) -> rocprofiler_status_t {
        auto* v = static_cast<std::vector<rocprofiler_counter_id_t>*>(ud);
        v->insert(v->end(), c, c + n);
        return ROCPROFILER_STATUS_SUCCESS;
      },
      &all);
  // The SPI occupancy-limiter counters are the newest addition: when the config cannot hold
  // them (or GPUEXP_PMC_NO_SPI=1), count without them rather than lose every counter -- the
  // same fallback as aql_pmc.cc's setup_agent.
  const char* no_spi = std::getenv("GPUEXP_PMC_NO_SPI");
  for (int attempt = (no_spi && no_spi[0] == '1') ? 1 : 0; attempt < 2; ++attempt) {
    std::vector<rocprofiler_counter_id_t> use;
    a.counter_slot.clear();
    for (auto& c : all) {
      rocprofiler_counter_info_v0_t info{};
      if (rocprofiler_query_counter_info(c, ROCPROFILER_COUNTER_INFO_VERSION_0, &info) != ROCPROFILER_STATUS_SUCCESS)
        continue;
      for (int k = 0; k < kNumCtr; ++k)
        if (info.name && std::strcmp(info.name, name(k)) == 0 && !(attempt == 1 && std::strncmp(info.name, "SPI_", 4) == 0)) {
          use.push_back(c);
          a.counter_slot[c.handle] = k;
        }
    }
    if (use.empty()) {
      *why = "agent supports none of the requested counters";
      return false;
    }
    size_t nrec = 0;
    for (auto& c : use) {
      rocprofiler_counter_info_v1_t info{};
      if (rocprofiler_query_counter_info(c, ROCPROFILER_COUNTER_INFO_VERSION_1, &info) == ROCPROFILER_STATUS_SUCCESS)
        nrec += info.dimensions_instances_count;
    }
    if (rocprofiler_create_counter_config(a.id, use.data(), use.size(), &a.cfg) == ROCPROFILER_STATUS_SUCCESS) {
      if (attempt == 1 && !(no_spi && no_spi[0] == '1'))
        std::fprintf(stderr, "[rocprof] the counter config cannot hold the SPI events; counting without them\n");
      a.have_cfg = true;
      a.recs.resize(nrec + 64);
      return true;
    }
  }
  *why = "create_counter_config failed (slot limits?)";
  return false;
}

}  // namespace

namespace {

// Duty cycle.  Measured on MI355X: while a device-counting context is STARTED a
// rocprofiler-sdk/HSA thread spins one core at 100% (even with no sample calls), so the
// context is only started for a short window per interval: start -> read (baseline) ->
// window -> read -> stop.  The window's deltas give the rates; the engine's tick never
// blocks on the GPU (it takes the latest completed window).
int g_window_ms = 20;
int g_interval_ms = 1000;
std::thread g_thread;
std::atomic<bool> g_quit{false};
std::condition_variable g_cv;
std::mutex g_cv_mu;

bool read_counts(Agent& a, double* v, int* inst) {
  size_t n = a.recs.size();
  if (rocprofiler_sample_device_counting_service(a.ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, a.recs.data(), &n) !=
      ROCPROFILER_STATUS_SUCCESS)
    return false;
  for (int k = 0; k < kNumCtr; ++k) {
    v[k] = 0;
    inst[k] = 0;
  }
  for (size_t i = 0; i < n; ++i) {
    rocprofiler_counter_id_t cid{};
    if (rocprofiler_query_record_counter_id(a.recs[i].id, &cid) != ROCPROFILER_STATUS_SUCCESS) continue;
    auto it = a.counter_slot.find(cid.handle);
    if (it == a.counter_slot.end()) continue;
    int k = it->second;
    double x = a.recs[i].counter_value;
    v[k] = use_max(k) ? std::max(v[k], x) : v[k] + x;
    inst[k] += 1;
  }
  a.last_nrec = n;
  return true;
}

void counting_loop() {
  while (!g_quit.load()) {
    double base[16][kNumCtr];
    std::chrono::steady_clock::time_point t0[16];
    bool ok[16] = {};
    {
      std::lock_guard<std::mutex> lk(g_mu);
      for (size_t i = 0; i < g_agents.size() && i < 16; ++i) {
        Agent& a = g_agents[i];
        if (!a.have_cfg || rocprofiler_start_context(a.ctx) != ROCPROFILER_STATUS_SUCCESS) continue;
        a.started = true;
        ok[i] = read_counts(a, base[i], a.last_inst);
        t0[i] = std::chrono::steady_clock::now();
      }
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(g_window_ms));
    {
      std::lock_guard<std::mutex> lk(g_mu);
      for (size_t i = 0; i < g_agents.size() && i < 16; ++i) {
        Agent& a = g_agents[i];
        if (!a.started) continue;
        double v[kNumCtr];
        if (ok[i] && read_counts(a, v, a.last_inst)) {
          double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0[i]).count();
          double d[kNumCtr];
          bool sane = wall > 0;
          for (int k = 0; k < kNumCtr; ++k) {
            d[k] = v[k] - base[i][k];
            if (d[k] < 0) sane = false;
          }
          std::memcpy(a.last_raw, d, sizeof(d));
          if (sane) derive(a.m, d, a.last_inst, wall);
        }
        rocprofiler_stop_context(a.ctx);
        a.started = false;
      }
    }
    std::unique_lock<std::mutex> lk(g_cv_mu);
    g_cv.wait_for(lk, std::chrono::milliseconds(std::max(0, g_interval_ms - g_window_ms)), [] { return g_quit.load(); });
  }
}

}  // namespace

extern "C" __attribute__((visibility("default"))) void gpuexp_rp_set_duty(int window_ms, int interval_ms) {
  g_window_ms = std::max(1, window_ms);
  g_interval_ms = std::max(g_window_ms, interval_ms);
}

extern "C" __attribute__((visibility("default"))) int gpuexp_rp_init(int ndev, const char* const* bdfs, char* err,
                                                                     int errlen) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto fail = [&](const std::string& m) {
    std::snprintf(err, size_t(errlen), "%s", m.c_str());
    g_status = "unavailable: " + m;
    return 0;
  };
  g_want_bdfs.assign(bdfs, bdfs + ndev);
  int inited = 0;
  rocprofiler_is_initialized(&inited);
  if (inited) return fail("rocprofiler already initialised in this process (HSA loaded before the plugin)");
  if (rocprofiler_force_configure(&configure) != ROCPROFILER_STATUS_SUCCESS)
    return fail("rocprofiler_force_configure failed");
  // Device counting needs the HSA runtime loaded; loading it now triggers tool_init.
  if (hsa_init() != HSA_STATUS_SUCCESS) return fail("hsa_init failed");
  if (!g_configured) return fail(g_err.empty() ? "tool_init did not configure any agent" : g_err);
  int ok = 0;
  std::string why;
  for (auto& a : g_agents) {
    if (a.dev < 0) continue;
    if (!build_config(a, &why)) continue;
    // Probe once that the context can start (PMC permission / exclusivity).
    if (rocprofiler_start_context(a.ctx) != ROCPROFILER_STATUS_SUCCESS) {
      why = "start_context failed (PMCs busy or insufficient permission?)";
      a.have_cfg = false;
      continue;
    }
    rocprofiler_stop_context(a.ctx);
    ++ok;
  }
  if (!ok) return fail(why.empty() ? "no agent started" : why);
  g_quit.store(false);
  g_thread = std::thread(counting_loop);
  g_status = "rocprofiler-sdk device counting on " + std::to_string(ok) + " GPU(s), " + std::to_string(g_window_ms) +
             " ms window every " + std::to_string(g_interval_ms) + " ms";
  return ok;
}

extern "C" __attribute__((visibility("default"))) int gpuexp_rp_sample(int dev, double dt_s, double* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (dev < 0 || size_t(dev) >= g_agents.size()) return -1;
  Agent& a = g_agents[size_t(dev)];
  if (!a.m.valid) return -1;
  std::memcpy(out, a.m.latest, sizeof(a.m.latest));
  (void)dt_s;
  return 0;
}

extern "C" __attribute__((visibility("default"))) void gpuexp_rp_shutdown() {
  g_quit.store(true);
  g_cv.notify_all();
  if (g_thread.joinable()) g_thread.join();
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& a : g_agents)
    if (a.started) {
      rocprofiler_stop_context(a.ctx);
      a.started = false;
    }
}

extern "C" __attribute__((visibility("default"))) const char* gpuexp_rp_status() { return g_status.c_str(); }

extern "C" __attribute__((visibility("default"))) int gpuexp_rp_scope(int dev) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (dev < 0 || size_t(dev) >= g_agents.size()) return -1;
  return g_agents[size_t(dev)].m.scope;
}

// Diagnostics: the raw (cumulative) reduced value and instance count of every counter in
// the last sample, as "NAME=value/instances;..." (used by tools/gpu_features_check.py).
extern "C" __attribute__((visibility("default"))) int gpuexp_rp_debug(int dev, char* buf, int len) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (dev < 0 || size_t(dev) >= g_agents.size()) return -1;
  const Agent& a = g_agents[size_t(dev)];
  std::string s = "records=" + std::to_string(a.last_nrec) + ";simd=" + std::to_string(a.m.simd) +
                  ";cu=" + std::to_string(a.m.cu) + ";";
  for (int k = 0; k < kNumCtr; ++k) {
    char t[128];
    std::snprintf(t, sizeof(t), "%s=%.0f/%d;", name(k), a.last_raw[k], a.last_inst[k]);
    s += t;
  }
  std::snprintf(buf, size_t(len), "%s", s.c_str());
  return 0;
}
