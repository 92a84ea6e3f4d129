// Optional per-GPU sources beyond the device backend: the HIP sentinel kernel, the
// rocprofiler-sdk device-counting plugin, and the RCCL API-trace shared-memory rings.
// None of these exist in the reference (it had NVML only, /root/reference/main.go:16).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "gpuexp/device.h"

namespace gpuexp {

class SentinelSource {
 public:
  virtual ~SentinelSource() = default;
  virtual bool start(const std::vector<DeviceInfo>& devs, std::string* err) = 0;
  // Called once per tick: drains completed runs, then launches the next one.
  virtual void tick(uint64_t now_ns) = 0;
  virtual bool read(int dev, SentinelReading* out) = 0;
  virtual void stop() = 0;
  virtual std::string status() const = 0;
};
// Implemented in sentinel.hip (1 wave, lowest-priority stream, pinned host ring), built
// as libgpuexp_hip.so and dlopen()ed from beside the core module; nullptr if unavailable.
std::unique_ptr<SentinelSource> make_hip_sentinel(int ring_slots, int spin_iters);
// The same sentinel kernel dispatched as raw AQL on the aqlprofile counters plugin's own
// HSA queue (one GPU queue for both); nullptr unless that plugin is loaded and exports it.
std::unique_ptr<SentinelSource> make_queue_sentinel(const std::string& counters_plugin, int ring_slots,
                                                   int spin_iters);
std::string default_rocprof_plugin();

// Derived values a counter plugin's gpuexp_rp_sample fills, in CounterReading order.
constexpr int kCounterOutputs = 18;
// CounterReading from those kCounterOutputs values (ok = true; nxcc left to the caller).
void fill_counter_reading(const double* v, CounterReading* out);

// Health of a GPU's counter reads (continuous mode), cumulative: reads found still queued,
// windows dropped because the counters went backwards, re-arms after another profiler reset
// or stopped them, moves to a rescue queue and its releases; rescue_active = reads are on the
// rescue queue now.
struct CounterHealth {
  uint64_t stalls = 0, resets = 0, rearms = 0, rescues = 0, releases = 0;
  bool rescue_active = false;
};

class CounterSource {
 public:
  virtual ~CounterSource() = default;
  virtual bool start(const std::vector<DeviceInfo>& devs, std::string* err) = 0;
  // Continuous mode: kick() at the start of a tick asks the plugin for one counter read per
  // GPU (non-blocking); sync() waits, at most `timeout_us`, for that round, so the values
  // sample() returns in the same tick cover exactly the last tick interval.  Duty-cycled
  // plugins ignore both.  sync() returns false when the round did not finish in time (the
  // previous window is exported again).
  virtual void kick() {}
  // Cumulative CPU time of the plugin's own thread(s), ns (0 if unknown).
  virtual uint64_t cpu_ns() { return 0; }
  virtual bool sync(int timeout_us) {
    (void)timeout_us;
    return true;
  }
  virtual bool sample(int dev, double dt_s, CounterReading* out) = 0;
  // -1 unknown, 0 = wave/LDS/EA counters only see this process (VMID-filtered), 1 = device-wide.
  virtual int scope(int dev) {
    (void)dev;
    return -1;
  }
  virtual bool health(int dev, CounterHealth* out) {
    (void)dev;
    (void)out;
    return false;
  }
  virtual void stop() = 0;
  virtual std::string status() const = 0;
};
// dlopen()s a counter plugin (_gpuexp_aqlpmc.so or _gpuexp_rocprof.so) next to the core.
// continuous (aqlprofile plugin only): counting runs without a break and is read once per
// engine tick; otherwise duty-cycled: a `window_ms` counting window every `interval_ms`.
// inline_rounds (continuous): the engine's sampler posts and collects each read round itself
// (no counting-thread wake-up per tick); for an engine that ticks periodically.
std::unique_ptr<CounterSource> make_rocprof_counters(const std::string& plugin_path, int window_ms,
                                                     int interval_ms, bool continuous = false,
                                                     bool inline_rounds = false);

// Tests / tools/project_cpu.py (fake_sources.cc): the real PMC read machine over scripted fake
// GPUs, and a sentinel, each burning `cost_us` of host CPU per GPU per read / run.
std::unique_ptr<CounterSource> make_fake_counters(uint64_t cost_us, int interval_ms, bool inline_rounds,
                                                  const std::vector<std::pair<int64_t, int64_t>>& stalls_us = {});
std::unique_ptr<SentinelSource> make_fake_sentinel(uint64_t cost_us);

// One collective call record written by the RCCL tracer tool into a per-process ring.
struct RcclTotals {
  int pid = 0;
  std::string op;     // allreduce, allgather, reducescatter, alltoall, send, recv, broadcast, ...
  uint64_t calls = 0;
  uint64_t bytes = 0;
  int rank = -1;      // communicator rank of the process (-1 unknown)
  int nranks = 0;     // communicator size (0 unknown)
};
class RcclSource {
 public:
  virtual ~RcclSource() = default;
  // Reads every tracer file under `dir` and returns cumulative per-(pid, op) totals of the
  // writers that could be identified and are still alive.
  virtual void poll(std::vector<RcclTotals>* out) = 0;
  // Files by state after the last poll: exported, writer not (yet) identified, writer gone.
  virtual void file_states(int* active, int* unverified, int* exited) const {
    *active = *unverified = *exited = 0;
  }
  // Directory entries the last listing skipped: not tracer files, not regular files, or
  // over the tracked-file cap.
  virtual int ignored() const { return 0; }
  virtual uint64_t scans() const { return 0; }  // directory listings so far
};
// verify_maps: a file is attributed only to a process that maps it (/proc/<pid>/maps).
// scan_interval_s: the directory is listed at most this often (and only when it changed).
std::unique_ptr<RcclSource> make_rccl_source(const std::string& dir, bool verify_maps = true,
                                             double scan_interval_s = 1.0);

}  // namespace gpuexp
