// HIP sentinel: one 64-lane wave per XCD per GPU per tick, on the lowest-priority stream,
// that stamps the shader clock (s_memtime), the 100 MHz reference clock (s_memrealtime)
// and the XCC/CU it landed on into a pinned, host-coherent ring.  The sampler never
// synchronizes: it drains completed runs (each wave writes its seq last, system-scope
// release) and launches the next run.  Nothing like it exists in the reference (NVML
// only, /root/reference/main.go:16); SURVEY.md §2.2 / §7.2 step 6.
//
// Grid = one workgroup per XCD: the dispatcher deals workgroups round-robin over the
// XCDs (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement"), so a run of 8 single-wave
// workgroups puts one wave on each XCD.  Placement is read back, not assumed.
//
// Measures, per tick:
//   sclk      = median over waves of d(s_memtime) / d(s_memrealtime) * 100 MHz over a
//               dependent ALU chain (the in-kernel clock recipe of MI355X_MICROARCH.md
//               "DVFS give-back" (6))
//   latency   = host launch -> wave start, both in the HSA system time domain (GPU ticks
//               converted with hsa_amd_profiling_convert_tick_to_system_domain); exported
//               for the first wave and per XCD (a saturated XCD starts its wave late)
//   xcc_id    = HW_REG_XCC_ID of workgroup 0
//   mem lat.  = 16 dependent loads through an uncached (hipDeviceMallocUncached) 64 KiB
//               chain, 4 KiB apart: load latency on the memory path as the running pods
//               leave it, per XCD and averaged.  Measured on MI355X (profiles/r01/
//               sentinel_memory_latency.txt): ~110 ns/hop idle, ~640 ns under an MFMA GEMM,
//               ~910 ns under a 5 TB/s HBM copy -- a contention probe, not a DRAM spec.
// Cost: one wave on one CU of each XCD for ~15 us + 16 loads per tick (<0.01% of the chip).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "gpuexp/sources.h"

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

// ring[run_slot * kSentinelMaxWaves + blockIdx.x]
// Writes the pointer-chase links in place (one lane per hop): initialising the chain with a
// kernel on the sentinel's stream instead of a copy keeps ROCr's blit/copy queues (each with
// its own ~173 MiB context save area on MI355X) from being created at all.
__global__ void __launch_bounds__(64) sentinel_init_chase(uint32_t* __restrict__ chase, int hops) {
  const int h = int(threadIdx.x);
  if (h < hops) chase[size_t(h) * kChaseStride] = uint32_t((h + 1) % hops);
}

__global__ void __launch_bounds__(64) sentinel_kernel(SentinelSlot* __restrict__ ring, uint32_t slot,
                                                      uint64_t seq, int spin, const uint32_t* chase, int hops) {
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

namespace {

struct HsaAgentMatch {
  uint32_t bdfid;
  uint32_t domain;
  hsa_agent_t agent;
  bool found;
};

hsa_status_t match_agent(hsa_agent_t a, void* data) {
  auto* m = static_cast<HsaAgentMatch*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdfid = 0, dom = 0;
  hsa_agent_get_info(a, hsa_agent_info_t(HSA_AMD_AGENT_INFO_BDFID), &bdfid);
  hsa_agent_get_info(a, hsa_agent_info_t(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
  if (bdfid == m->bdfid && dom == m->domain) {
    m->agent = a;
    m->found = true;
  }
  return HSA_STATUS_SUCCESS;
}

uint64_t hsa_now() {
  uint64_t t = 0;
  hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
  return t;
}

class HipSentinel : public SentinelSource {
  struct Reading {
    bool ok = false;
    double sclk_hz = 0, latency_s = 0, xcc = 0;
    double xcc_latency_s[kMaxXcc] = {kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN};
    double mem_latency_s = kNaN;
    double xcc_mem_latency_s[kMaxXcc] = {kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN};
  };
  struct Per {
    int hip = -1;
    bool ready = false;
    int waves = 1;  // workgroups per run: one per XCD of this GPU / partition
    hipStream_t stream = nullptr;
    SentinelSlot* ring = nullptr;
    SentinelSlot* dring = nullptr;
    uint32_t* chase = nullptr;  // uncached device buffer of the HBM latency probe
    int hops = 0;
    std::vector<uint64_t> host_launch;  // per run slot, HSA system time just before launch
    hsa_agent_t agent{};
    bool have_agent = false;
    uint64_t launched = 0, completed = 0, stalled = 0, errors = 0;
    Reading last;
  };

 public:
  HipSentinel(int ring, int spin) : nslots_(ring < 4 ? 4 : ring), spin_(spin < 16 ? 16 : spin) {}
  ~HipSentinel() override { stop(); }

  bool start(const std::vector<DeviceInfo>& devs, std::string* err) override {
    int nhip = 0;
    if (hipGetDeviceCount(&nhip) != hipSuccess || nhip == 0) {
      *err = "no HIP devices";
      return false;
    }
    // HIP device order can differ from the exporter's; match by PCI BDF.
    std::vector<std::string> hip_bdf(static_cast<size_t>(nhip));
    for (int h = 0; h < nhip; ++h) {
      char bus[64] = {0};
      if (hipDeviceGetPCIBusId(bus, sizeof(bus), h) == hipSuccess) {
        std::string b(bus);
        for (auto& c : b) c = char(::tolower(c));
        hip_bdf[size_t(h)] = b;
      }
    }
    hsa_init();  // refcounted; HIP already initialised it
    uint64_t freq = 0;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &freq);
    sys_ns_per_tick_ = freq ? 1e9 / double(freq) : 1.0;
    per_.resize(devs.size());
    int ok = 0, waves = 0;
    const size_t ring_bytes = sizeof(SentinelSlot) * size_t(nslots_) * kSentinelMaxWaves;
    // Partitioned sockets (CPX/DPX/QPX) expose several HIP devices with one BDF, in
    // partition order, as do the exporter's devices: the k-th takes the k-th free one.
    std::vector<bool> taken(size_t(nhip), false);
    for (size_t i = 0; i < devs.size(); ++i) {
      Per& p = per_[i];
      std::string want = devs[i].bdf;
      for (auto& c : want) c = char(::tolower(c));
      for (int h = 0; h < nhip && p.hip < 0; ++h)
        if (!taken[size_t(h)] && hip_bdf[size_t(h)] == want) {
          p.hip = h;
          taken[size_t(h)] = true;
        }
      if (p.hip < 0) continue;
      if (hipSetDevice(p.hip) != hipSuccess) continue;
      p.waves = devs[i].num_xcc ? std::min<int>(int(devs[i].num_xcc), kSentinelMaxWaves) : kSentinelMaxWaves;
      int least = 0, greatest = 0;
      (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
      if (hipStreamCreateWithPriority(&p.stream, hipStreamNonBlocking, least) != hipSuccess) continue;
      void* mem = nullptr;
      if (hipHostMalloc(&mem, ring_bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) continue;
      p.ring = static_cast<SentinelSlot*>(mem);
      std::memset(mem, 0, ring_bytes);
      p.host_launch.assign(size_t(nslots_), 0);
      // HBM latency probe chain (64 KiB, uncached); without it the kernel skips the probe.
      void* chase = nullptr;
      const size_t chase_words = size_t(kChaseHops) * kChaseStride;
      if (hipExtMallocWithFlags(&chase, chase_words * sizeof(uint32_t), hipDeviceMallocUncached) == hipSuccess) {
        // Initialised by a kernel on the sentinel's own stream, not by a copy: every hardware
        // queue the runtime creates (the stream's, the null stream's, the blit queues behind
        // hipMemcpy) costs a context save/restore area in GTT sized for the whole GPU
        // (~173 MiB on MI355X, KFD cwsr_size x XCCs; tools/probe_queue_rss.py).
        static_assert(kChaseHops <= 64, "one lane per hop");
        hipLaunchKernelGGL(sentinel_init_chase, dim3(1), dim3(64), 0, p.stream, static_cast<uint32_t*>(chase),
                           kChaseHops);
        if (hipGetLastError() == hipSuccess && hipStreamSynchronize(p.stream) == hipSuccess) {
          p.chase = static_cast<uint32_t*>(chase);
          p.hops = kChaseHops;
        } else {
          (void)hipFree(chase);
        }
      }
      void* dptr = nullptr;
      (void)hipHostGetDevicePointer(&dptr, mem, 0);
      p.dring = static_cast<SentinelSlot*>(dptr ? dptr : mem);
      // HSA agent for tick -> system-domain conversion.
      unsigned bus = 0, dev = 0, fn = 0, dom = 0;
      if (std::sscanf(want.c_str(), "%x:%x:%x.%x", &dom, &bus, &dev, &fn) == 4) {
        HsaAgentMatch m{(bus << 8) | (dev << 3) | fn, dom, {}, false};
        hsa_iterate_agents(match_agent, &m);
        p.agent = m.agent;
        p.have_agent = m.found;
      }
      p.ready = true;
      ++ok;
      waves += p.waves;
    }
    if (!ok) {
      *err = "no exporter GPU matched a HIP device";
      return false;
    }
    status_ = "hip sentinel on " + std::to_string(ok) + " GPU(s), " + std::to_string(waves) +
              " waves/tick (one per XCD), ring " + std::to_string(nslots_);
    return true;
  }

  void tick(uint64_t) override {
    for (size_t i = 0; i < per_.size(); ++i) {
      Per& p = per_[i];
      if (!p.ready) continue;
      drain(p);
      // Bound the in-flight window: a saturated queue shows up as latency, not as an
      // unbounded backlog of sentinel launches.
      if (p.launched - p.completed >= 4) {
        p.stalled += 1;
        continue;
      }
      uint64_t seq = p.launched + 1;
      uint32_t slot = uint32_t(seq % uint64_t(nslots_));
      SentinelSlot* s = p.ring + size_t(slot) * kSentinelMaxWaves;
      for (int w = 0; w < p.waves; ++w) __atomic_store_n(&s[w].seq, 0ull, __ATOMIC_RELAXED);
      (void)hipSetDevice(p.hip);
      p.host_launch[slot] = hsa_now();
      hipLaunchKernelGGL(sentinel_kernel, dim3(unsigned(p.waves)), dim3(64), 0, p.stream, p.dring, slot, seq,
                         spin_, p.chase, p.hops);
      if (hipGetLastError() != hipSuccess) {
        p.errors += 1;
        continue;
      }
      p.launched = seq;
    }
  }

  // Host launch -> wave start (seconds), NaN when the clock domains disagree.
  double wave_latency(const Per& p, const SentinelSlot& w, uint64_t host_launch) const {
    uint64_t sys = 0;
    if (!p.have_agent ||
        hsa_amd_profiling_convert_tick_to_system_domain(p.agent, w.rt0, &sys) != HSA_STATUS_SUCCESS)
      return std::nan("");
    double lat = (double(sys) - double(host_launch)) * sys_ns_per_tick_ * 1e-9;
    // A negative value means the GPU tick and s_memrealtime domains disagree; keep the
    // rest of the reading and drop the latency rather than export garbage.
    if (lat > -1e-6 && lat < 10.0) return lat < 0 ? 0 : lat;
    return std::nan("");
  }

  void drain(Per& p) {
    while (p.completed < p.launched) {
      uint64_t seq = p.completed + 1;
      uint32_t slot = uint32_t(seq % uint64_t(nslots_));
      const SentinelSlot* s = p.ring + size_t(slot) * kSentinelMaxWaves;
      bool done = true;
      for (int w = 0; w < p.waves && done; ++w) done = __atomic_load_n(&s[w].seq, __ATOMIC_ACQUIRE) == seq;
      if (!done) break;
      p.completed = seq;
      Reading r = p.last;  // an XCD without a wave this run keeps its previous latency
      r.ok = true;
      r.xcc = double(s[0].xcc_id & 0xF);
      r.latency_s = std::nan("");
      double sclk[kSentinelMaxWaves];
      int ns = 0;
      double mem_sum = 0;
      int mem_n = 0;
      for (int w = 0; w < p.waves; ++w) {
        double drt = double(s[w].rt1 - s[w].rt0);
        double dmt = double(s[w].mt1 - s[w].mt0);
        if (drt > 0) sclk[ns++] = dmt / drt * 100e6;
        if (s[w].hops > 0 && s[w].chase_end == 0) {  // 100 MHz ticks per hop -> seconds
          const double hl = double(s[w].chase_rt) * 10e-9 / double(s[w].hops);
          mem_sum += hl;
          ++mem_n;
          const uint32_t hx = s[w].xcc_id & 0xF;
          if (hx < uint32_t(kMaxXcc)) r.xcc_mem_latency_s[hx] = hl;
        }
        double lat = wave_latency(p, s[w], p.host_launch[slot]);
        if (std::isnan(lat)) continue;
        if (std::isnan(r.latency_s) || lat < r.latency_s) r.latency_s = lat;
        uint32_t x = s[w].xcc_id & 0xF;
        if (x < uint32_t(kMaxXcc)) r.xcc_latency_s[x] = lat;
      }
      std::nth_element(sclk, sclk + ns / 2, sclk + ns);
      r.sclk_hz = ns ? sclk[ns / 2] : std::nan("");
      r.mem_latency_s = mem_n ? mem_sum / mem_n : std::nan("");
      p.last = r;
    }
  }

  bool read(int dev, SentinelReading* out) override {
    if (dev < 0 || size_t(dev) >= per_.size() || !per_[size_t(dev)].ready) return false;
    Per& p = per_[size_t(dev)];
    if (!p.last.ok) return false;
    out->ok = true;
    out->sclk_hz = p.last.sclk_hz;
    out->dispatch_latency_s = p.last.latency_s;
    out->xcc_id = p.last.xcc;
    out->runs = p.completed;
    std::copy(std::begin(p.last.xcc_latency_s), std::end(p.last.xcc_latency_s), std::begin(out->xcc_latency_s));
    out->mem_latency_s = p.last.mem_latency_s;
    std::copy(std::begin(p.last.xcc_mem_latency_s), std::end(p.last.xcc_mem_latency_s),
              std::begin(out->xcc_mem_latency_s));
    return true;
  }

  void stop() override {
    for (auto& p : per_) {
      if (!p.ready) continue;
      (void)hipSetDevice(p.hip);
      (void)hipStreamSynchronize(p.stream);  // a sentinel run is microseconds long
      drain(p);
      (void)hipStreamDestroy(p.stream);
      (void)hipHostFree(p.ring);
      if (p.chase) (void)hipFree(p.chase);
      p.ready = false;
    }
    per_.clear();
  }

  std::string status() const override { return status_; }

 private:
  int nslots_;
  int spin_;
  double sys_ns_per_tick_ = 1.0;
  std::vector<Per> per_;
  std::string status_ = "not started";
};

}  // namespace

}  // namespace gpuexp

// Factory exported from libgpuexp_hip.so.  The telemetry core dlopen()s this library
// only when the sentinel is enabled, so the core itself never links a HIP runtime: a
// process that also imports torch (which bundles its own libamdhip64.so.7) must end up
// with ONE HIP runtime, not two (measured: two copies -> hipMalloc OOM + exit hang).
extern "C" __attribute__((visibility("default"))) gpuexp::SentinelSource* gpuexp_make_hip_sentinel(int ring_slots,
                                                                                                   int spin_iters) {
  return new gpuexp::HipSentinel(ring_slots, spin_iters);
}
