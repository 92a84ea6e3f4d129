// Device identity + per-tick sample model and the backend interface.
//
// Reference: NVML DeviceGetCount / DeviceGetHandleByIndex / GetMemoryInfo /
// GetComputeRunningProcesses, re-queried every cycle and fatal on any error
// (/root/reference/main.go:116-138).  Here devices are enumerated ONCE (stable identity:
// BDF, UUID, KFD gpu_id, render minor), and each tick fills a DeviceSample per GPU;
// a failing GPU only marks itself down (amd_gpu_up=0) — no other GPU is affected.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "gpuexp/common.h"

namespace gpuexp {

constexpr int kMaxXgmiLinks = 8;   // AMDSMI_MAX_NUM_XGMI_LINKS (amdsmi.h:118)
constexpr int kMaxHbm = 4;         // AMDSMI_NUM_HBM_INSTANCES (amdsmi.h:97)
constexpr int kMaxXcc = 8;         // AMDSMI_MAX_NUM_XCC (amdsmi.h:167)

struct DeviceInfo {
  int index = 0;              // exporter GPU index == `gpu` label
  std::string uuid;
  std::string bdf;            // "0000:72:00.0"
  std::string name;           // marketing/asic name
  uint32_t kfd_gpu_id = 0;    // /sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>
  int render_minor = -1;      // /dev/dri/renderD<minor>
  int card = -1;
  int hip_id = -1;
  uint64_t vram_total = 0;    // bytes (static)
  uint32_t num_xcc = 0;        // XCDs of this (logical) GPU: 8 in SPX, 1 in CPX
  uint32_t num_cu = 0;
  // Compute / memory partitioning of the socket (amdgpu current_compute_partition /
  // current_memory_partition): SPX|DPX|QPX|CPX and NPS1|NPS2|NPS4.  In a partitioned mode
  // each partition is its own logical GPU (own KFD node + render node, same PCI BDF);
  // socket-level telemetry (power, temperatures, xGMI, PCIe) is shared by all of them.
  std::string compute_partition, memory_partition;
  int partition_id = 0;        // XCP index of this logical GPU within its socket
  // Logical GPUs of one partitioned socket (same BDF) share one gpu_metrics fetch per tick and
  // one phase of the fetch cap (share_socket_fetches); -1 = a whole GPU, its own fetches.
  int socket_group = -1;
  // The sysfs device behind the render node: the PCI BDF for a whole GPU and for partition
  // 0 of a partitioned socket, "amdgpu_xcp.<n>" for its other partitions (platform
  // devices).  What device plugins name a logical GPU by; unique per logical GPU where the
  // BDF is not (see device_owner_keys).
  std::string dev_node;
  std::string xgmi_peer_bdf[kMaxXgmiLinks];  // from amdsmi_get_link_metrics (once)
  // Board identity and firmware (amdgpu sysfs on the PCI function, read once; "" = n/a)
  std::string vbios_version, product_name, product_number, serial_number;
  std::vector<std::pair<std::string, std::string>> firmware;  // (component, version), fw_version/*_fw_version
  // false: no exporter-owned GPU queue on this device (no sentinel, no PMC counters); each
  // queue pins ~346 MiB of host memory on MI355X (profiles/r02/queue_memory.txt)
  bool queue_enabled = true;
};

// Basename of realpath(<root>/sys/class/drm/renderD<minor>/device): the BDF or
// "amdgpu_xcp.<n>"; `bdf` when the node cannot be resolved (or is not a device link).
std::string render_dev_node(const std::string& root, int render_minor, const std::string& bdf);

// Keys under which a device owner (device plugin allocation) may name this logical GPU,
// lower-case, most specific first: the sysfs device node (and its "amdgpu_xcp_<n>"
// spelling), "<bdf>/<partition>", the render node, "kfd:<gpu_id>", the UUID, and the bare
// BDF only when the BDF is this GPU's own device node (a whole GPU, or partition 0) — a
// bare BDF never names the other partitions of a socket.
std::vector<std::string> device_owner_keys(const DeviceInfo& d);

// xGMI link index -> peer GPU PCI BDF for the GPU at `bdf`, from amdgpu's per-device
// xgmi_port_num listings under <root>/sys/bus/pci/devices ("<node>:<port> ->  <peer
// node>:<peer port>" per link; node ids shared across the hive).  gpu_metrics's
// xgmi_*_data_acc[l] is source port l (checked against amdsmi_get_link_metrics on MI355X).
// Fills peers[port]; returns how many links resolved.
int xgmi_peers_from_sysfs(const std::string& root, const std::string& bdf, std::string peers[kMaxXgmiLinks]);

// Fills d->vbios_version / product_* / serial_number / firmware from <root>/sys/bus/pci/
// devices/<bdf> (vbios_version, product_name, product_number, serial_number and
// fw_version/<component>_fw_version).  Missing or unreadable files stay empty.
void read_board_info(const std::string& root, DeviceInfo* d);

// One tick of device telemetry.  NaN = unsupported/unavailable; raw accumulators are
// kept as integers so deltas are exact across wraps.
struct DeviceSample {
  bool ok = false;
  std::string error;
  uint64_t host_ns = 0;        // CLOCK_MONOTONIC at read
  uint64_t fw_ts_10ns = 0;     // PMFW timestamp (10 ns units), 0 = n/a
  bool metrics_coalesced = false;  // decoded from the cached gpu_metrics table (no SMU fetch)
  bool metrics_shared = false;     // a fresh table another partition of the socket fetched this tick
  // What this sample's reads cost (filled by the backend; the engine's devices-stage split,
  // gpuexp_device_read_seconds_total): gpu_metrics wall + thread CPU (a fresh read is an
  // SMU round trip the kernel busy-waits on; ~0 when coalesced), the VRAM-used file, wall.
  uint64_t metrics_wall_ns = 0, metrics_cpu_ns = 0, vram_wall_ns = 0;
  bool time_parts = true;  // set by the engine: time the VRAM read (vram_wall_ns) on this tick
  bool read_memory = true;  // set by the engine: read VRAM used on this tick (else left NaN)

  double gfx_activity = kNaN;  // %
  double umc_activity = kNaN;  // %
  double mm_activity = kNaN;   // %
  double vram_used = kNaN;     // bytes
  double vram_total = kNaN;    // bytes
  double power_w = kNaN;       // current socket power
  double power_cap_w = kNaN;
  uint64_t energy_acc = 0;     // raw accumulator
  double energy_unit_j = 15.259e-6;  // J per unit (amdsmi: 15.259 uJ)
  bool energy_valid = false;

  // temperatures (C)
  double temp_hotspot = kNaN, temp_mem = kNaN, temp_edge = kNaN;
  double temp_vrgfx = kNaN, temp_vrsoc = kNaN, temp_vrmem = kNaN;
  double temp_hbm[kMaxHbm] = {kNaN, kNaN, kNaN, kNaN};

  // clocks (MHz); clk_gfx is the mean over the XCDs' own gfx clocks
  double clk_gfx = kNaN, clk_soc = kNaN, clk_mem = kNaN;
  double clk_gfx_xcc[kMaxXcc] = {kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN};  // this GPU's XCDs
  int num_partition = 0;       // gpu_metrics num_partition (0 = n/a)

  // xGMI accumulators (KB) per link; link_up: 1/0, NaN unsupported
  int num_xgmi_links = 0;
  uint64_t xgmi_read_kb[kMaxXgmiLinks] = {};
  uint64_t xgmi_write_kb[kMaxXgmiLinks] = {};
  double xgmi_link_up[kMaxXgmiLinks] = {kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN};
  bool xgmi_valid = false;

  // PMFW PCIe link traffic, Mb/s (megabits; amdsmi's documented unit — the kernel header's
  // "GB/sec" is wrong: a 57.6 GB/s host-to-device copy reads 560550, i.e. 70.1 GB/s of link
  // traffic incl. protocol overhead, tools/probe_pcie_units.py)
  double pcie_bw_inst = kNaN;
  uint64_t pcie_bw_acc = 0;         // sum of the PMFW's 1 ms pcie_bw_inst samples
  double pcie_replay = kNaN;        // count
  double pcie_width = kNaN, pcie_speed_gts = kNaN;
  // link reliability (gpu_metrics v1.8 accumulators; NaN unsupported)
  double pcie_nak_sent = kNaN, pcie_nak_rcvd = kNaN, pcie_l0_recov = kNaN;
  double xgmi_width = kNaN, xgmi_speed = kNaN;  // lanes, Gb/s per lane (PMFW units)

  // RAS / AER error totals (sysfs ras/*_err_count and aer_dev_*; refreshed at a low rate)
  double ecc_ce = kNaN, ecc_ue = kNaN, ecc_de = kNaN;
  double aer_cor = kNaN, aer_nonfatal = kNaN, aer_fatal = kNaN;
  // HBM pages in the RAS bad-page table (refreshed with the RAS totals)
  double pages_retired = kNaN, pages_pending = kNaN, pages_unreservable = kNaN;
  // GTT: system memory mapped into the GPU's address space (mem_info_gtt_*, bytes)
  double gtt_used = kNaN, gtt_total = kNaN;

  // throttle residency accumulators (same units as accumulation_counter)
  bool residency_valid = false;
  uint64_t accumulation_counter = 0;
  uint64_t res_ppt = 0, res_socket_thm = 0, res_vr_thm = 0, res_hbm_thm = 0, res_prochot = 0;

  // per-XCC busy accumulators (for gfx util from counters)
  uint64_t gfx_busy_acc[kMaxXcc] = {};
  double vram_max_bw_gbs = kNaN;
};

// One GPU process observed on one device.
struct ProcSample {
  int pid = 0;
  int device = 0;              // DeviceInfo::index
  double vram_bytes = 0;
  double cu_occupancy = kNaN;  // CUs (KFD stats_<id>/cu_occupancy)
  double sdma_us = kNaN;       // accumulated SDMA usage (us)
  double evicted_ms = kNaN;    // accumulated time the process's queues were evicted (KFD stats)
  double gfx_ns = kNaN;        // engine time (amdsmi)
  std::string name;            // comm
  // The KFD reader's identity of this process: one id per KFD proc entry, never reused, so two
  // samples with the same id are the same process (0: the sample did not come from KFD)
  uint64_t kfd_id = 0;
};

// rocprofiler-sdk device-counting derived values for one GPU over one tick.
struct CounterReading {
  bool ok = false;
  double mfma_busy_pct = kNaN;      // SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_COUNT * SIMDs): share of wall time
  double mfma_util_pct = kNaN;      // SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * SIMDs): MfmaUtil
  double sq_busy_pct = kNaN;        // SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE
  double gui_active_pct = kNaN;     // GRBM_GUI_ACTIVE / GRBM_COUNT
  double waves_per_s = kNaN;        // SQ_WAVES / dt
  double lds_active_pct = kNaN;     // SQ_LDS_IDX_ACTIVE / (GUI_ACTIVE * CUs)
  double lds_bank_conflict_pct = kNaN;  // SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  double hbm_read_bps = kNaN;       // TCC_EA0_RDREQ_DRAM_32B * 32 B / dt
  double hbm_write_bps = kNaN;      // TCC_EA0_WRREQ_WRITE_DRAM_32B * 32 B / dt
  double remote_read_bps = kNaN;    // TCC_EA0_RDREQ_GMI_32B * 32 B / dt (memory behind GMI: peers)
  double remote_write_bps = kNaN;   // TCC_EA0_WRREQ_WRITE_GMI_32B * 32 B / dt
  double mfma_bf16_flops = kNaN;    // SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 / dt
  double mfma_fp8_flops = kNaN;     // SQ_INSTS_VALU_MFMA_MOPS_F8 * 512 / dt
  // occupancy limiters (SPI resource allocator, counter_model.h): share of cycles a ready
  // compute wave fit nowhere; over those cycles, share of CUs LDS-full / SIMDs wave-slot-full /
  // SIMDs VGPR-full
  double dispatch_stall_pct = kNaN, lds_limited_pct = kNaN, wave_limited_pct = kNaN, vgpr_limited_pct = kNaN,
         sgpr_limited_pct = kNaN;
  // mfma_busy_pct of each XCC (its SQ instances over its own GRBM_COUNT x its SIMDs);
  // nxcc = 0 when the counter source cannot attribute samples to XCCs
  int nxcc = 0;
  double xcc_mfma_busy_pct[kMaxXcc] = {kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN};
};

// HIP sentinel kernel stamps for one GPU (latest completed run).  A run is one wave per
// XCD (the dispatcher deals workgroups round-robin over the 8 XCDs), so the chip-level
// values below aggregate per-XCD stamps.
struct SentinelReading {
  bool ok = false;
  double sclk_hz = kNaN;              // median over waves of d(s_memtime)/d(s_memrealtime) * 100 MHz
  double dispatch_latency_s = kNaN;   // host launch -> first wave running
  double xcc_id = kNaN;               // XCC workgroup 0 landed on
  uint64_t runs = 0;                  // completed sentinel runs
  // host launch -> wave start on each XCD (indexed by HW_REG_XCC_ID; NaN = no wave there yet)
  double xcc_latency_s[kMaxXcc] = {kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN};
  // dependent uncached device-memory load latency (mean over waves; per XCD by XCC_ID)
  double mem_latency_s = kNaN;
  double xcc_mem_latency_s[kMaxXcc] = {kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN};
  // how long the oldest launched run has been waiting to finish (0: none outstanding): grows
  // while the GPU gives a one-wave kernel no slot (compute starvation) or stops (hang)
  double pending_s = kNaN;
};

class Backend {
 public:
  virtual ~Backend() = default;
  // gpu_metrics read coalescing (GpuMetricsReader); set before init().
  void set_metrics_coalescing(bool on) { coalesce_metrics_ = on; }
  void set_metrics_min_interval(uint64_t ns) { metrics_min_ns_ = ns; }
  // Tests only: burn this much thread CPU per fresh gpu_metrics read, so a fake host root
  // carries the SMU fetch's measured cost (a real fetch is kernel busy-wait); set before init().
  void set_fake_metrics_cost(uint64_t ns) { fake_metrics_cost_ns_ = ns; }
  // Per-GPU cap on fresh gpu_metrics reads, changed while running (the engine's "auto"
  // policy, EngineConfig::metrics_min_interval_s < 0).  Sampler thread only.
  // not_before_ns: no fresh read before then (0 = none): the GPU's phase within the cap.
  virtual void update_metrics_min_interval(const DeviceInfo& dev, uint64_t ns, uint64_t not_before_ns = 0) {
    (void)dev;
    (void)ns;
    (void)not_before_ns;
  }
  virtual const char* name() const = 0;
  // Enumerates devices once.  Returns false (with *err) if the backend cannot run.
  virtual bool init(std::vector<DeviceInfo>* devices, std::string* err) = 0;
  virtual void sample(const DeviceInfo& dev, DeviceSample* out) = 0;
  // Optional process listing owned by the backend (mock, amdsmi).  Returns false if the
  // backend has no process source (the engine then uses the KFD sysfs reader).
  virtual bool processes(const DeviceInfo& dev, std::vector<ProcSample>* out) {
    (void)dev;
    (void)out;
    return false;
  }
  // Optional synthetic counter/sentinel sources (the mock backend simulates both so the
  // CPU-only plumbing config exports the full 64-series/GPU profile).
  virtual bool counters(const DeviceInfo& dev, double dt_s, CounterReading* out) {
    (void)dev;
    (void)dt_s;
    (void)out;
    return false;
  }
  virtual bool sentinel(const DeviceInfo& dev, SentinelReading* out) {
    (void)dev;
    (void)out;
    return false;
  }
  // Human-readable per-device source description (e.g. which metrics path is in use).
  // Learnt PMFW gpu_metrics refresh period (GpuMetricsReader); 0 = unknown / n/a.
  virtual double metrics_period_s(const DeviceInfo& dev) {
    (void)dev;
    return 0;
  }
  virtual std::string describe(const DeviceInfo& dev) {
    (void)dev;
    return name();
  }
  virtual void shutdown() {}
 protected:
  bool coalesce_metrics_ = true;
  uint64_t metrics_min_ns_ = 0;
  uint64_t fake_metrics_cost_ns_ = 0;
};

}  // namespace gpuexp
