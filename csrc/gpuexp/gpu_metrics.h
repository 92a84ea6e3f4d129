// Direct decoder for the amdgpu `gpu_metrics` sysfs blob (format 1, content 8 — the
// layout MI355X/gfx950 PMFW publishes; 3872 bytes, measured on the box:
// profiles/probe_amdsmi.txt).
//
// Why: amdsmi_get_gpu_metrics_info() costs ~150 us per call on MI355X (same probe),
// i.e. 12% of a core at 100 Hz x 8 GPUs.  The blob itself is one pread() on a cached
// fd.  The layout is validated at start-up against amdsmi's decode of the same device
// (GpuMetricsReader::validate); on any mismatch the backend falls back to amdsmi.
//
// Replaces NVML Device.GetMemoryInfo()/per-device reads (/root/reference/main.go:129-132)
// with every device-level signal the north star asks for (util, HBM, power, temps,
// clocks, xGMI accumulators, throttle residencies) from ONE read.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "gpuexp/device.h"

namespace gpuexp {

#pragma pack(push, 1)
struct GpuMetricsHeader {
  uint16_t structure_size;
  uint8_t format_revision;
  uint8_t content_revision;
};
#pragma pack(pop)

// Natural alignment (the kernel struct is not packed).
struct XcpMetricsV1_8 {
  uint32_t gfx_busy_inst[8];
  uint16_t jpeg_busy[40];
  uint16_t vcn_busy[4];
  uint64_t gfx_busy_acc[8];
  uint64_t gfx_below_host_limit_ppt_acc[8];
  uint64_t gfx_below_host_limit_thm_acc[8];
  uint64_t gfx_low_utilization_acc[8];
  uint64_t gfx_below_host_limit_total_acc[8];
};

struct GpuMetricsV1_8 {
  GpuMetricsHeader header;
  uint16_t temperature_hotspot;
  uint16_t temperature_mem;
  uint16_t temperature_vrsoc;
  uint16_t curr_socket_power;
  uint16_t average_gfx_activity;
  uint16_t average_umc_activity;
  uint64_t mem_max_bandwidth;
  uint64_t energy_accumulator;
  uint64_t system_clock_counter;
  uint32_t accumulation_counter;
  uint32_t prochot_residency_acc;
  uint32_t ppt_residency_acc;
  uint32_t socket_thm_residency_acc;
  uint32_t vr_thm_residency_acc;
  uint32_t hbm_thm_residency_acc;
  uint32_t gfxclk_lock_status;
  uint16_t pcie_link_width;
  uint16_t pcie_link_speed;
  uint16_t xgmi_link_width;
  uint16_t xgmi_link_speed;
  uint32_t gfx_activity_acc;
  uint32_t mem_activity_acc;
  uint64_t pcie_bandwidth_acc;
  uint64_t pcie_bandwidth_inst;
  uint64_t pcie_l0_to_recov_count_acc;
  uint64_t pcie_replay_count_acc;
  uint64_t pcie_replay_rover_count_acc;
  uint32_t pcie_nak_sent_count_acc;
  uint32_t pcie_nak_rcvd_count_acc;
  uint64_t xgmi_read_data_acc[8];
  uint64_t xgmi_write_data_acc[8];
  uint16_t xgmi_link_status[8];
  uint16_t padding;
  uint64_t firmware_timestamp;
  uint16_t current_gfxclk[8];
  uint16_t current_socclk[4];
  uint16_t current_vclk0[4];
  uint16_t current_dclk0[4];
  uint16_t current_uclk;
  uint16_t num_partition;
  XcpMetricsV1_8 xcp_stats[8];
  uint32_t pcie_lc_perf_other_end_recovery;
};

static_assert(sizeof(XcpMetricsV1_8) == 440, "xcp v1.8 layout");
static_assert(offsetof(GpuMetricsV1_8, xgmi_read_data_acc) == 136, "v1.8 layout");
static_assert(offsetof(GpuMetricsV1_8, firmware_timestamp) == 288, "v1.8 layout");
static_assert(offsetof(GpuMetricsV1_8, xcp_stats) == 344, "v1.8 layout");
static_assert(sizeof(GpuMetricsV1_8) == 3872, "v1.8 size (measured blob size)");

// Decodes a v1.8 blob into `out`.  Returns false if the header does not match.
// `xcp` / `nxcc` select the compute partition a logical GPU is (SPX: xcp 0 with all 8
// XCDs; CPX: xcp k owns XCD k): its per-XCD busy accumulators come from xcp_stats[xcp]
// and its gfx clocks from current_gfxclk[xcp*nxcc, (xcp+1)*nxcc).  nxcc 0 = every XCD.
bool decode_gpu_metrics_v1_8(const void* blob, size_t len, DeviceSample* out, int xcp = 0, int nxcc = 0);

// Reader for one device's gpu_metrics file: keeps the fd open and pread()s from 0.
// Reads <dev>/gpu_metrics.  Each fresh read makes the driver fetch the table from the SMU
// (120-420 us of CPU in the kernel, measured), but the PMFW refreshes the table only every
// ~20 ms on MI355X (profiles/r01/pmfw_rate.txt: firmware_timestamp steps of 20.0 ms; at
// 100 Hz half the reads, at 1 kHz 95%, return an identical table).  With coalescing on,
// the reader learns the refresh period from firmware_timestamp steps and, until the next
// expected refresh, decodes its cached copy instead of re-reading — no information is
// lost, the kernel-side cost drops to the PMFW rate.
// One fetched table, shared by the readers of the compute partitions of one socket (CPX:
// eight logical GPUs, one SMU): the first partition to read fresh at a tick fetches, the others
// decode the same blob for their own XCDs at that tick instead of asking the SMU again.
struct GpuMetricsShared {
  uint64_t tick_ns = 0;  // the tick (now_ns) it was fetched at (0 = never)
  long n = 0;
  alignas(8) unsigned char buf[8192];
};

class GpuMetricsReader {
 public:
  GpuMetricsReader() = default;
  ~GpuMetricsReader();
  // Owns its fd: move-only (a copy would close the fd under the other copy's feet).
  GpuMetricsReader(const GpuMetricsReader&) = delete;
  GpuMetricsReader& operator=(const GpuMetricsReader&) = delete;
  GpuMetricsReader(GpuMetricsReader&& o) noexcept;
  GpuMetricsReader& operator=(GpuMetricsReader&& o) noexcept;
  bool open(const std::string& path, std::string* err);
  // Reads (or re-decodes the cached table, see above) at host time `now_ns` (0 = always
  // read).  Returns false (and sets out->error) on I/O or format error.
  bool read(DeviceSample* out, uint64_t now_ns = 0);
  bool is_open() const { return fd_ >= 0; }
  uint8_t format() const { return fmt_; }
  uint8_t content() const { return content_; }
  const std::string& path() const { return path_; }
  void set_coalesce(bool on) { coalesce_ = on; }
  // Fresh reads at most every `ns` (0 = as often as the PMFW refreshes): caps the kernel
  // CPU of the SMU fetches (120-420 us each) when many GPUs are sampled at a high rate.
  void set_min_fresh_interval(uint64_t ns) { min_fresh_ns_ = ns; }
  // No fresh read before `ns` (0 = none): the engine gives each GPU's fetch its own phase of the
  // cap, so a node's GPUs do not all fetch on the same tick.
  void defer_fresh_until(uint64_t ns) { not_before_ns_ = ns; }
  uint64_t min_fresh_interval() const { return min_fresh_ns_; }
  // Tests only: thread CPU burnt per fresh read (models the SMU round trip on a fake host).
  void set_fake_cost(uint64_t ns) { fake_cost_ns_ = ns; }
  void set_partition(int xcp, int nxcc) {
    xcp_ = xcp;
    nxcc_ = nxcc;
  }
  // Partitions of one socket share their fetches (see GpuMetricsShared; nullptr = own fetches).
  void set_shared(std::shared_ptr<GpuMetricsShared> s) { shared_ = std::move(s); }
  // Never reuse a table for longer than this, whatever the learnt period.
  static constexpr uint64_t kMaxCoalesceNs = 50000000;
  uint64_t period_ns() const { return period_ns_; }
  uint64_t fresh_reads() const { return fresh_reads_; }
  uint64_t coalesced_reads() const { return coalesced_reads_; }

 private:
  int fd_ = -1;
  std::string path_;
  uint8_t fmt_ = 0, content_ = 0;
  bool coalesce_ = true;
  uint64_t min_fresh_ns_ = 0;
  uint64_t not_before_ns_ = 0;
  uint64_t fake_cost_ns_ = 0;
  int xcp_ = 0, nxcc_ = 0;
  long last_n_ = 0;
  uint64_t last_fw_ts_ = 0;      // firmware_timestamp of the cached table (10 ns units)
  uint64_t t_change_ns_ = 0;     // estimated host time the cached table appeared
  uint64_t last_read_ns_ = 0;    // host time of the last fresh read
  bool last_was_fresh_ = false;  // no coalesced read since the previous fresh one
  uint64_t period_ns_ = 0;       // learnt PMFW refresh period (0 = unknown)
  // Table-to-table steps seen by back-to-back fresh reads; the period is their median
  // (a startup gap or a missed table is an outlier, not the estimate).
  static constexpr int kSteps = 16;
  uint64_t steps_[kSteps] = {};
  int nsteps_ = 0;
  uint64_t fresh_reads_ = 0, coalesced_reads_ = 0;
  std::shared_ptr<GpuMetricsShared> shared_;
  alignas(8) unsigned char buf_[8192];
};

// Gives the logical GPUs of each partitioned socket one GpuMetricsShared, so one SMU fetch per
// tick serves all of them, and a common DeviceInfo::socket_group (the engine phases the fetch
// cap per socket).  The socket of device i is `socket(i)` (default: its PCI BDF, which KFD
// gives every partition of a socket; amdsmi: its socket handle).  `reader(i)` is device i's
// reader (nullptr: none).  Whole GPUs (alone on their socket) are left alone.
void share_socket_fetches(std::vector<DeviceInfo>* devs, const std::function<GpuMetricsReader*(size_t)>& reader,
                          const std::function<std::string(size_t)>& socket = nullptr);

}  // namespace gpuexp
