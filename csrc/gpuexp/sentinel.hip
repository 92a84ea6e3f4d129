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

#include "gpuexp/sentinel_device.h"
#include "gpuexp/sources.h"

namespace gpuexp {

__global__ void __launch_bounds__(64) sentinel_init_chase(uint32_t* __restrict__ chase, int hops) {
  sentinel_init_chase_body(chase, hops);
}

__global__ void __launch_bounds__(64) sentinel_kernel(SentinelSlot* __restrict__ ring, uint32_t slot,
                                                      uint64_t seq, int spin, const uint32_t* chase, int hops) {
  sentinel_body(ring, slot, seq, spin, chase, hops);
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

class HipSentinel : public SentinelSource {
  struct Per {
    int hip = -1;
    bool ready = false;
    hipStream_t stream = nullptr;
    SentinelSlot* dring = nullptr;
    uint32_t* chase = nullptr;  // uncached device buffer of the HBM latency probe
    int hops = 0;
    SentinelRun run;
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
      if (p.hip < 0 || !devs[i].queue_enabled) continue;  // disabled: its HIP device stays reserved
      if (hipSetDevice(p.hip) != hipSuccess) continue;
      p.run.waves = devs[i].num_xcc ? std::min<int>(int(devs[i].num_xcc), kSentinelMaxWaves) : kSentinelMaxWaves;
      int least = 0, greatest = 0;
      (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
      if (hipStreamCreateWithPriority(&p.stream, hipStreamNonBlocking, least) != hipSuccess) continue;
      void* mem = nullptr;
      if (hipHostMalloc(&mem, ring_bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) continue;
      p.run.ring = static_cast<SentinelSlot*>(mem);
      std::memset(mem, 0, ring_bytes);
      p.run.host_launch.assign(size_t(nslots_), 0);
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
        p.run.agent = m.agent;
        p.run.have_agent = m.found;
      }
      p.ready = true;
      ++ok;
      waves += p.run.waves;
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
      sentinel_drain(p.run, nslots_, sys_ns_per_tick_);
      // Bound the in-flight window: a saturated queue shows up as latency, not as an
      // unbounded backlog of sentinel launches.
      if (p.run.launched - p.run.completed >= 4) {
        p.run.stalled += 1;
        continue;
      }
      const uint64_t seq = p.run.launched + 1;
      (void)hipSetDevice(p.hip);
      const uint32_t slot = sentinel_prepare(p.run, seq, nslots_);
      hipLaunchKernelGGL(sentinel_kernel, dim3(unsigned(p.run.waves)), dim3(64), 0, p.stream, p.dring, slot, seq,
                         spin_, p.chase, p.hops);
      if (hipGetLastError() != hipSuccess) {
        p.run.errors += 1;
        continue;
      }
      p.run.launched = seq;
      p.run.fresh_seq = seq;
    }
  }

  bool read(int dev, SentinelReading* out) override {
    if (dev < 0 || size_t(dev) >= per_.size() || !per_[size_t(dev)].ready) return false;
    // every tick: completions folded in and the pending time current (launches run at most
    // every sentinel_min_interval)
    return sentinel_read(per_[size_t(dev)].run, nslots_, sys_ns_per_tick_, out);
  }

  void stop() override {
    for (auto& p : per_) {
      if (!p.ready) continue;
      (void)hipSetDevice(p.hip);
      (void)hipStreamSynchronize(p.stream);  // a sentinel run is microseconds long
      sentinel_drain(p.run, nslots_, sys_ns_per_tick_);
      (void)hipStreamDestroy(p.stream);
      (void)hipHostFree(p.run.ring);
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
