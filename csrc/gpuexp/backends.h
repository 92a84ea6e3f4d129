// Concrete device backends.
//   mock   — N scripted fake GPUs (BASELINE config 1; CPU-only tests, fault injection)
//   sysfs  — KFD topology + drm sysfs + raw gpu_metrics, all under an injectable host
//            root (fake-host integration tests; amdsmi-free fast path)
//   amdsmi — libamd_smi enumeration (UUID, BDF, KFD id, render node, xGMI peers) with
//            the raw gpu_metrics fast path validated against amdsmi's own decode.
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gpuexp/device.h"
#include "gpuexp/gpu_metrics.h"

namespace gpuexp {

// An fd kept open across ticks and pread() from offset 0 (sysfs regenerates the
// attribute on every read at offset 0): one syscall per value per tick.
class CachedFile {
 public:
  CachedFile() = default;
  ~CachedFile();
  CachedFile(const CachedFile&) = delete;
  CachedFile& operator=(const CachedFile&) = delete;
  CachedFile(CachedFile&& o) noexcept : fd_(o.fd_), path_(std::move(o.path_)) { o.fd_ = -1; }
  CachedFile& operator=(CachedFile&& o) noexcept;
  bool open(const std::string& path);
  bool is_open() const { return fd_ >= 0; }
  // Reads the whole (small) file. Returns bytes read, -1 on error.
  long read(char* buf, size_t cap);
  bool read_u64(uint64_t* v);
  void close();
  const std::string& path() const { return path_; }

 private:
  int fd_ = -1;
  std::string path_;
};

class MockBackend : public Backend {
 public:
  explicit MockBackend(int num_devices, uint32_t kfd_id_base = 1000);
  const char* name() const override { return "mock"; }
  bool init(std::vector<DeviceInfo>* devices, std::string* err) override;
  void sample(const DeviceInfo& dev, DeviceSample* out) override;
  bool processes(const DeviceInfo& dev, std::vector<ProcSample>* out) override;
  bool counters(const DeviceInfo& dev, double dt_s, CounterReading* out) override;
  bool sentinel(const DeviceInfo& dev, SentinelReading* out) override;

  // --- scripting (thread-safe; called from Python while the sampler runs) ---
  // Pins a field to a value ("gfx_activity", "umc_activity", "vram_used", "power_w",
  // "temp_hotspot", "temp_mem", "temp_vrsoc", "clk_gfx", "clk_mem", "clk_soc",
  // "xgmi_read_rate_kbps", "xgmi_write_rate_kbps", ...).  NaN clears the override.
  void set_value(int dev, const std::string& field, double v);
  // Scripted process list for a device; when any device has one, the mock is the
  // process source, otherwise the KFD sysfs reader is used (fake host root).
  void set_processes(int dev, const std::vector<ProcSample>& procs);
  void clear_processes();
  // Fault injection: "none", "error" (sample fails), "vanish" (device gone),
  // "counter_reset" (accumulators restart from 0 once), "wrap" (xGMI acc near 2^64).
  void set_fault(int dev, const std::string& fault);
  // Rehearsals of per-peer xGMI attribution on CPU ranks (bench.py --backend mock): `path` holds
  // an N x N little-endian uint64 matrix, bytes rank/GPU i sent to GPU j so far, written by the
  // traffic generators; each mock link's write (read) accumulator then carries exactly what its
  // GPU sent to (received from) the link's peer, and the synthetic per-link rates are off.
  void set_traffic_file(const std::string& path);

 private:
  struct Script {
    std::map<std::string, double> overrides;
    std::vector<ProcSample> procs;
    bool has_procs = false;
    std::string fault = "none";
    // integrated accumulators
    bool started = false;
    uint64_t last_ns = 0;
    double energy_units = 0;
    uint64_t xgmi_rd_kb[kMaxXgmiLinks] = {};  // unsigned: wraps like the hardware
    uint64_t xgmi_wr_kb[kMaxXgmiLinks] = {};
    double xgmi_frac[2][kMaxXgmiLinks] = {};
    double busy_acc[kMaxXcc] = {};
    double accum = 0;
    double res_ppt = 0;
    double pcie_acc = 0;
  };
  double get(const Script& s, const char* field, double dflt) const;
  int n_;
  uint32_t kfd_base_;
  std::string traffic_path_;
  bool read_traffic(std::vector<uint64_t>* m) const;  // the N x N matrix (false: unreadable)
  mutable std::mutex mu_;
  std::vector<Script> scripts_;
};

class SysfsBackend : public Backend {
 public:
  explicit SysfsBackend(std::string host_root);
  const char* name() const override { return "sysfs"; }
  bool init(std::vector<DeviceInfo>* devices, std::string* err) override;
  void sample(const DeviceInfo& dev, DeviceSample* out) override;
  std::string describe(const DeviceInfo& dev) override {
    return devs_.at(size_t(dev.index))->gm_ok ? "raw gpu_metrics v1.8 (sysfs)" : "drm sysfs + hwmon";
  }
  double metrics_period_s(const DeviceInfo& dev) override {
    return double(devs_.at(size_t(dev.index))->gm.period_ns()) * 1e-9;
  }
  void update_metrics_min_interval(const DeviceInfo& dev, uint64_t ns, uint64_t not_before_ns = 0) override {
    devs_.at(size_t(dev.index))->gm.set_min_fresh_interval(ns);
    devs_.at(size_t(dev.index))->gm.defer_fresh_until(not_before_ns);
  }

  // amdsmi-compatible UUID from the KFD unique_id + PCI device id.
  static std::string uuid_from_unique_id(uint64_t unique_id, uint32_t device_id);

 protected:
  struct Dev {
    std::string dev_dir;   // .../drm/renderD<minor>/device
    GpuMetricsReader gm;
    bool gm_ok = false;
    CachedFile vram_used, busy, mem_busy, power, temp_hot, temp_mem, temp_edge;
    double power_cap_w = kNaN;
    int xcp = 0, nxcc = 0;  // compute partition of this logical GPU (see DeviceInfo)
  };
  void open_dev_files(Dev* d);
  void sample_fallback(Dev& d, DeviceSample* out);
  std::string root_;
  std::vector<std::unique_ptr<Dev>> devs_;
};

std::unique_ptr<Backend> make_amdsmi_backend(const std::string& host_root, bool amdsmi_procs,
                                             bool force_amdsmi_metrics);

}  // namespace gpuexp
