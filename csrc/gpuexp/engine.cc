#include "gpuexp/engine.h"

#include <fcntl.h>
#include <sys/eventfd.h>
#include <sys/poll.h>
#include <sys/prctl.h>
#include <sys/timerfd.h>
#include <sys/utsname.h>
#include <unistd.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <set>

namespace gpuexp {

namespace {

const std::vector<std::string> kDevLabels = {"gpu", "bdf", "namespace", "pod", "container"};

std::vector<std::string> with(const std::vector<std::string>& base, std::initializer_list<const char*> extra) {
  std::vector<std::string> v = base;
  for (auto e : extra) v.emplace_back(e);
  return v;
}

std::string lower(std::string s) {
  std::transform(s.begin(), s.end(), s.begin(), ::tolower);
  return s;
}

// Delta of a monotonically increasing hardware accumulator.  Unsigned wrap is accepted
// when the wrapped delta is plausible; a large backwards jump is a reset (returns false).
bool acc_delta(uint64_t cur, uint64_t prev, double* d) {
  uint64_t diff = cur - prev;  // modular
  if (cur >= prev || diff < (1ull << 62)) {
    *d = double(diff);
    return true;
  }
  return false;
}

const std::vector<double>& stage_bounds() {
  // 9 bounds: the per-stage histograms are re-rendered and re-compressed every tick (at 14
  // bounds they were a third of a 1-GPU exposition), so keep them coarse.
  static const std::vector<double> b = {5e-6, 25e-6, 100e-6, 250e-6, 500e-6, 1e-3, 2.5e-3, 10e-3, 100e-3};
  return b;
}

// "0".."63" without a std::to_string per series per tick (label values of links / XCDs)
const char* idx_str(int i) {
  static const char* k[64] = {"0",  "1",  "2",  "3",  "4",  "5",  "6",  "7",  "8",  "9",  "10", "11", "12",
                              "13", "14", "15", "16", "17", "18", "19", "20", "21", "22", "23", "24", "25",
                              "26", "27", "28", "29", "30", "31", "32", "33", "34", "35", "36", "37", "38",
                              "39", "40", "41", "42", "43", "44", "45", "46", "47", "48", "49", "50", "51",
                              "52", "53", "54", "55", "56", "57", "58", "59", "60", "61", "62", "63"};
  return i >= 0 && i < 64 ? k[i] : "?";
}

// True on an engine's own sampler thread (set in run_sampler): that thread charges its
// whole clock to the sampler account, a manual tick_now() caller only the tick itself.
thread_local bool tl_sampler_thread = false;

const char* kTempNames[9] = {"hotspot", "mem", "vrsoc", "edge", "vrgfx", "vrmem", "hbm0", "hbm1", "hbm2"};
const char* kClkNames[3] = {"gfx", "soc", "mem"};
const char* kThrNames[5] = {"ppt", "socket_thermal", "vr_thermal", "hbm_thermal", "prochot"};

}  // namespace

ForkJoinPool::ForkJoinPool(int threads) {
  const size_t n = threads > 1 ? size_t(threads - 1) : 0;
  wcpu_.reset(new std::atomic<uint64_t>[n > 0 ? n : 1]);
  for (size_t t = 0; t < n; ++t) wcpu_[t].store(0);
  for (size_t t = 0; t < n; ++t) workers_.emplace_back([this, t] { worker(t); });
}

uint64_t ForkJoinPool::cpu_ns_total() const {
  uint64_t s = 0;
  for (size_t t = 0; t < workers_.size(); ++t) s += wcpu_[t].load();
  return s;
}

ForkJoinPool::~ForkJoinPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    quit_ = true;
  }
  cv_.notify_all();
  for (auto& w : workers_) w.join();
}

void ForkJoinPool::worker(size_t idx) {
  set_thread_name("gpuexp-dev");
  uint64_t seen = 0;
  for (;;) {
    const std::function<void(int)>* fn;
    int n;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return quit_ || epoch_ != seen; });
      if (quit_) return;
      seen = epoch_;
      fn = fn_;
      n = n_;
    }
    for (int i; (i = next_.fetch_add(1)) < n;) (*fn)(i);
    wcpu_[idx].store(thread_cpu_ns());  // before pending_ drops: run() sees it
    std::lock_guard<std::mutex> lk(mu_);
    pending_ -= 1;
    if (pending_ == 0) done_cv_.notify_all();
  }
}

void ForkJoinPool::run(int n, const std::function<void(int)>& fn) {
  if (workers_.empty() || n <= 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    fn_ = &fn;
    n_ = n;
    next_.store(0);
    pending_ = int(workers_.size());
    ++epoch_;
  }
  cv_.notify_all();
  for (int i; (i = next_.fetch_add(1)) < n;) fn(i);
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return pending_ == 0; });
}

const char* Engine::stage_name(int i) {
  static const char* n[kStages] = {"devices", "processes", "attribution", "sentinel",
                                   "counters", "series", "render", "publish"};
  return n[i];
}

const char* Engine::dev_part_name(int i) {
  static const char* n[kDevParts] = {"counters_kick", "control", "gpu_metrics", "vram", "ras", "gtt"};
  return n[i];
}

Engine::Engine(const EngineConfig& cfg) : cfg_(cfg) { self_pid_ = int(::getpid()); }

Engine::~Engine() { stop(); }

void Engine::define_families() {
  auto G = MetricType::kGauge;
  auto C = MetricType::kCounter;
  auto H = MetricType::kHistogram;
  auto add = [this](const char* n, const char* h, MetricType t, std::vector<std::string> l) {
    return table_.add_family(FamilyDef{n, h, t, std::move(l)});
  };
  const auto& D = kDevLabels;
  // --- per-GPU device families (standard profile: 64 series per GPU) ---
  f_info_ = add("amd_gpu_info", "MI355X device identity (value is always 1)", G,
                {"gpu", "bdf", "uuid", "name", "kfd_gpu_id", "render_node", "hip_id", "partition",
                 "compute_partition", "memory_partition", "device_node"});
  f_up_ = add("amd_gpu_up", "1 if the last telemetry read of this GPU succeeded", G, D);
  f_gfx_ = add("amd_gpu_gfx_activity_percent", "Average graphics/compute engine activity (PMFW)", G, D);
  f_umc_ = add("amd_gpu_umc_activity_percent", "Average memory-controller (HBM3E) activity", G, D);
  f_xcc_ = add("amd_gpu_xcc_busy_percent", "Per-XCD compute busy over the last tick (gfx_busy_acc deltas)", G,
               with(D, {"xcc"}));
  f_vram_used_ = add("amd_gpu_vram_used_bytes", "HBM3E VRAM in use", G, D);
  f_vram_total_ = add("amd_gpu_vram_total_bytes", "HBM3E VRAM capacity", G, D);
  f_hbm_bw_ = add("amd_gpu_hbm_bandwidth_bytes_per_second",
                  "HBM bandwidth estimate: UMC activity x max VRAM bandwidth", G, D);
  f_power_ = add("amd_gpu_power_watts", "Current socket power", G, D);
  f_power_cap_ = add("amd_gpu_power_cap_watts", "Socket power cap", G, D);
  f_energy_ = add("amd_gpu_energy_joules_total", "Energy consumed (hardware accumulator)", C, D);
  f_temp_ = add("amd_gpu_temperature_celsius", "Temperature by sensor", G, with(D, {"sensor"}));
  f_clk_ = add("amd_gpu_clock_hz", "Current clock frequency by domain", G, with(D, {"clock"}));
  f_xrd_ = add("amd_gpu_xgmi_read_bytes_total", "xGMI bytes received on a link (hardware accumulator)", C,
               with(D, {"link", "peer_bdf"}));
  f_xwr_ = add("amd_gpu_xgmi_write_bytes_total", "xGMI bytes sent on a link (hardware accumulator)", C,
               with(D, {"link", "peer_bdf"}));
  f_xrd_rate_ = add("amd_gpu_xgmi_read_bytes_per_second", "xGMI receive rate summed over links", G, D);
  f_xwr_rate_ = add("amd_gpu_xgmi_write_bytes_per_second", "xGMI transmit rate summed over links", G, D);
  f_links_up_ = add("amd_gpu_xgmi_links_up", "Number of xGMI links reporting up", G, D);
  f_pcie_bw_ = add("amd_gpu_pcie_bandwidth_bytes_per_second",
                   "PCIe link traffic, both directions incl. protocol overhead (PMFW instantaneous, Mb/s / 8)", G, D);
  f_pcie_replay_ = add("amd_gpu_pcie_replay_total", "PCIe replay count", C, D);
  f_pcie_speed_ = add("amd_gpu_pcie_link_speed_gts", "PCIe link speed (GT/s)", G, D);
  f_pcie_width_ = add("amd_gpu_pcie_link_width", "PCIe link width (lanes)", G, D);
  f_thr_ = add("amd_gpu_throttle_residency_percent", "Share of the last tick spent throttled, by reason", G,
               with(D, {"reason"}));
  f_nprocs_ = add("amd_gpu_processes", "Processes with a KFD context on this GPU", G, D);
  f_cu_occ_ = add("amd_gpu_cu_occupancy",
                  "Resident waves of all processes on this GPU in CU-equivalents (KFD: waves / max waves per CU; "
                  "the bench's saturating 256x256 GEMM reads 64 on MI355X)", G, D);
  // --- full profile: link / memory reliability (error totals; not part of the 64-series load) ---
  f_ecc_ = add("amd_gpu_ecc_errors_total", "RAS ECC error count summed over IP blocks (sysfs ras/*_err_count)", C,
               with(D, {"type"}));
  f_aer_ = add("amd_gpu_pcie_aer_errors_total", "PCIe AER errors reported for the GPU function", C,
               with(D, {"severity"}));
  f_pcie_nak_ = add("amd_gpu_pcie_nak_total", "PCIe NAKs (PMFW accumulator)", C, with(D, {"direction"}));
  f_pcie_recov_ = add("amd_gpu_pcie_recovery_total", "PCIe L0 -> recovery transitions (PMFW accumulator)", C, D);
  f_xgmi_width_ = add("amd_gpu_xgmi_link_width", "xGMI link width (PMFW)", G, D);
  f_xgmi_speed_ = add("amd_gpu_xgmi_link_speed", "xGMI link speed (PMFW units)", G, D);
  f_mfma_ = add("amd_gpu_mfma_busy_percent",
                "MFMA (matrix core) busy: share of the last tick's wall time the matrix cores of all SIMDs were "
                "issuing (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_COUNT x SIMDs), per XCD over its own clock, averaged)", G, D);
  f_mfma_util_ = add("amd_gpu_mfma_util_percent",
                     "MFMA utilisation while the GPU was active (rocprof MfmaUtil: SQ_VALU_MFMA_BUSY_CYCLES / "
                     "(GRBM_GUI_ACTIVE x SIMDs))", G, D);
  f_mfma_flops_ = add("amd_gpu_mfma_flops_per_second",
                      "Matrix-core work done, by operand type: FLOP/s over the last tick "
                      "(SQ_INSTS_VALU_MFMA_MOPS_<type> x 512)", G, with(D, {"dtype"}));
  f_disp_stall_ = add("amd_gpu_dispatch_stall_percent",
                      "Share of the time a compute wave ready to launch fitted on no CU of its shader engine "
                      "(SPI resource allocator; every process's waves, full profile)",
                      G, D);
  f_occ_lim_ = add("amd_gpu_occupancy_limiter_percent",
                   "While compute waves waited for a CU: the share of CUs whose free LDS could not take the "
                   "wave (resource=lds: LDS occupancy), of SIMDs without a free wave slot (wave_slots), "
                   "without enough free VGPRs (vgpr) or SGPRs (sgpr); 0 when no wave waited (every process's "
                   "waves, full profile)",
                   G, with(D, {"resource"}));
  f_sq_busy_ = add("amd_gpu_sq_busy_percent", "Shader sequencer busy (SQ_BUSY_CYCLES)", G, D);
  f_gui_ = add("amd_gpu_gui_active_percent", "Graphics pipe active (GRBM_GUI_ACTIVE / GRBM_COUNT)", G, D);
  f_waves_ = add("amd_gpu_waves_per_second", "Waves dispatched per second (SQ_WAVES)", G, D);
  f_lds_ = add("amd_gpu_lds_active_percent",
               "LDS ACTIVITY: cycles per CU in which the LDS served an instruction (SQ_LDS_IDX_ACTIVE); how much "
               "LDS space waves hold (LDS OCCUPANCY) is amd_gpu_occupancy_limiter_percent{resource=\"lds\"}",
               G, D);
  f_lds_conf_ = add("amd_gpu_lds_bank_conflict_percent", "LDS bank-conflict cycles / LDS active cycles", G, D);
  f_hbm_rd_ = add("amd_gpu_hbm_read_bytes_per_second",
                  "HBM read bandwidth: L2 read sectors from the memory controller (TCC_EA0_RDREQ_DRAM_32B x 32 B)", G, D);
  f_hbm_wr_ = add("amd_gpu_hbm_write_bytes_per_second",
                  "HBM write bandwidth: L2 write sectors to the memory controller (TCC_EA0_WRREQ_WRITE_DRAM_32B x 32 B)", G,
                  D);
  f_remote_rd_ = add("amd_gpu_remote_read_bytes_per_second",
                     "L2 reads of memory behind GMI, e.g. a peer GPU's HBM over xGMI (TCC_EA0_RDREQ_GMI_32B x 32 B)", G, D);
  f_remote_wr_ = add("amd_gpu_remote_write_bytes_per_second",
                     "L2 writes to memory behind GMI, e.g. a peer GPU's HBM over xGMI (TCC_EA0_WRREQ_WRITE_GMI_32B x 32 B)",
                     G, D);
  f_sen_sclk_ = add("amd_gpu_sentinel_sclk_hz", "Effective shader clock measured by the sentinel kernel", G, D);
  f_sen_lat_ = add("amd_gpu_sentinel_dispatch_latency_seconds",
                   "Host launch to first-wave start of the sentinel kernel (queue contention)", G, D);
  f_sen_xcc_ = add("amd_gpu_sentinel_xcc_id", "XCC that workgroup 0 of the last sentinel run landed on", G, D);
  f_sen_runs_ = add("amd_gpu_sentinel_runs_total", "Completed sentinel kernel runs", C, D);
  f_sen_pend_ = add("amd_gpu_sentinel_pending_seconds",
                    "How long the sentinel's outstanding run has waited to finish (0: none outstanding). Grows "
                    "while the workload leaves a one-wave kernel no CU slot, or without bound on a hung GPU", G, D);
  f_sen_mem_ = add("amd_gpu_sentinel_memory_latency_seconds",
                   "Dependent-load latency of the sentinel's uncached device-memory chain: memory-path contention probe", G, D);
  // --- full profile: per-XCD detail (8 XCDs on an SPX-mode MI355X) ---
  f_xcc_clk_ = add("amd_gpu_xcc_clock_hz", "Per-XCD gfx clock (PMFW current_gfxclk of each XCC)", G,
                   with(D, {"xcc"}));
  f_sen_xlat_ = add("amd_gpu_sentinel_xcc_dispatch_latency_seconds",
                    "Host launch to sentinel wave start on each XCD (per-XCD CU contention)", G, with(D, {"xcc"}));
  f_xcc_mfma_ = add("amd_gpu_xcc_mfma_busy_percent",
                    "MFMA busy of each XCD: its SQ_VALU_MFMA_BUSY_CYCLES / (its GRBM_COUNT x its SIMDs); "
                    "amd_gpu_mfma_busy_percent is their mean", G, with(D, {"xcc"}));
  f_sen_xmem_ = add("amd_gpu_sentinel_xcc_memory_latency_seconds",
                    "Sentinel memory-chain load latency seen from each XCD (memory-path contention probe)", G,
                    with(D, {"xcc"}));

  // --- per-process / per-pod families ---
  const std::vector<std::string> P = {"gpu", "pid", "comm", "namespace", "pod", "container"};
  f_proc_vram_ = add("amd_gpu_process_vram_bytes", "VRAM held by a process on a GPU (KFD)", G, P);
  f_proc_cu_ = add("amd_gpu_process_cu_occupancy",
                   "Resident waves of a process on a GPU in CU-equivalents (KFD stats_<id>/cu_occupancy)", G, P);
  f_proc_sdma_ = add("amd_gpu_process_sdma_seconds_total",
                     "KFD's per-process SDMA activity (sdma_<gpu_id>, read as microseconds); only with "
                     "kfd_sdma_activity: on MI355X the file is not SDMA time (one jump at the first copy, "
                     "then flat under 55 GB/s of copies)",
                     C, P);
  f_proc_evicted_ = add("amd_gpu_process_evicted_seconds_total",
                        "Time the process's GPU queues were evicted (memory pressure / preemption; KFD stats)", C, P);
  f_proc_gfx_ = add("amd_gpu_process_gfx_activity_percent",
                    "GPU gfx activity attributed to a process: the GPU's activity split by the processes' "
                    "occupied CUs (estimate on shared GPUs; exact for a sole process)", G, P);
  if (cfg_.legacy_families) {
    // Byte-compatible with the reference (/root/reference/main.go:22-35): names, HELP,
    // label names and order {pid, pod}.  `pid` is the host PID (the reference's intended
    // meaning; it accidentally exported a slice index, main.go:144).
    f_legacy_mem_ = add("pod_gpu_memory_usage", "GPU memory used by Kubernetes Pod", G, {"pid", "pod"});
    f_legacy_perc_ = add("docker_gpu_memory_perc_usage", "GPU memory in percentage used by pod", G,
                         {"pid", "pod"});
  }
  const std::vector<std::string> PO = {"namespace", "pod"};
  f_pod_vram_ = add("amd_pod_gpu_vram_bytes", "VRAM held by all GPU processes of a pod", G, PO);
  f_pod_procs_ = add("amd_pod_gpu_processes", "GPU processes of a pod", G, PO);
  f_pod_gpus_ = add("amd_pod_gpus", "GPUs attributed to a pod", G, PO);
  f_pod_xrd_ = add("amd_pod_xgmi_read_bytes_per_second", "xGMI receive rate of the pod's GPUs", G, PO);
  f_pod_xwr_ = add("amd_pod_xgmi_write_bytes_per_second", "xGMI transmit rate of the pod's GPUs", G, PO);
  f_pod_xrd_total_ = add("amd_pod_xgmi_read_bytes_total",
                         "xGMI bytes received by the pod's GPUs (per-tick link accumulator deltas; on a shared GPU "
                         "the pod's CU-occupancy share)", C, PO);
  f_pod_xwr_total_ = add("amd_pod_xgmi_write_bytes_total",
                         "xGMI bytes sent by the pod's GPUs (per-tick link accumulator deltas; on a shared GPU the "
                         "pod's CU-occupancy share)", C, PO);
  f_pod_mfma_ = add("amd_pod_gpu_mfma_busy_percent",
                    "Mean MFMA busy of the pod's GPUs (amd_gpu_mfma_busy_percent of each GPU it owns)", G, PO);
  f_pod_flops_ = add("amd_pod_gpu_mfma_flops_per_second",
                     "MFMA FLOP/s of the pod's GPUs by operand type (sum of amd_gpu_mfma_flops_per_second over "
                     "the GPUs it owns)", G, with(PO, {"dtype"}));
  f_pod_hbm_ = add("amd_pod_gpu_hbm_bandwidth_bytes_per_second",
                   "HBM bandwidth of the pod's GPUs (sum of amd_gpu_hbm_bandwidth_bytes_per_second over the GPUs it owns)",
                   G, PO);
  f_pod_power_ = add("amd_pod_gpu_power_watts", "Socket power of the pod's GPUs", G, PO);
  f_pod_alloc_s_ = add("amd_pod_gpu_allocated_seconds_total",
                       "GPU-seconds the pod has held GPUs (device-plugin allocation; one GPU for one second = 1)", C, PO);
  f_pod_busy_s_ = add("amd_pod_gpu_busy_seconds_total",
                      "GPU-seconds the pod's GPUs were busy (per-XCD gfx_busy accumulators; a shared GPU's busy time "
                      "split by the pod's CU-occupancy share)", C, PO);
  f_pod_energy_ = add("amd_pod_gpu_energy_joules_total",
                      "GPU energy used by the pod: its GPUs' hardware energy counters, and on a shared GPU the "
                      "pod's CU-occupancy share of it (chargeback)", C, PO);
  f_pod_gfx_ = add("amd_pod_gpu_gfx_activity_percent", "Mean gfx activity of the pod's GPUs", G, PO);
  f_pod_gfx_share_ = add("amd_pod_gfx_activity_share_percent",
                         "GPU gfx activity of the pod's processes summed over GPUs, in percent of one GPU "
                         "(per-process CU-occupancy split; covers shared GPUs)", G, PO);
  f_rccl_calls_ = add("amd_rccl_collective_calls_total", "RCCL collective/p2p calls by op (rocprofiler-sdk tracer)",
                      C, {"namespace", "pod", "pid", "op"});
  f_rccl_bytes_ = add("amd_rccl_collective_bytes_total", "RCCL payload bytes by op (rocprofiler-sdk tracer)", C,
                      {"namespace", "pod", "pid", "op"});
  f_rccl_comm_ = add("amd_rccl_communicator_info",
                     "Rank and size of the largest RCCL communicator of a process (value is always 1)", G,
                     {"namespace", "pod", "pid", "rank", "nranks"});
  f_board_ = add("amd_gpu_board_info", "Board identity: product, serial number, VBIOS (value is always 1; full profile)",
                 G, {"gpu", "bdf", "product_name", "product_number", "serial_number", "vbios_version"});
  f_fw_ = add("amd_gpu_firmware_info",
              "Loaded firmware versions by component, from amdgpu fw_version/ (value is always 1; full profile)", G,
              {"gpu", "bdf", "component", "version"});
  f_driver_ = add("amd_driver_info", "amdgpu driver and kernel release of the node (value is always 1; full profile)", G,
                  {"version", "kernel"});
  f_pages_ = add("amd_gpu_retired_pages",
                 "HBM pages in the RAS bad-page table by state: retired (never handed out again), pending, "
                 "unreservable (ras/gpu_vram_bad_pages; full profile)",
                 G, with(D, {"state"}));
  f_gtt_used_ = add("amd_gpu_gtt_used_bytes", "System memory mapped into the GPU's address space (GTT, full profile)",
                    G, D);
  f_gtt_total_ = add("amd_gpu_gtt_total_bytes", "GTT size (full profile)", G, D);
  f_kfd_ev_ = add("amd_gpu_kfd_events_total",
                  "KFD SMI events on this GPU: vm_fault (a process's GPU page fault), thermal_throttle, "
                  "gpu_pre_reset / gpu_post_reset, queue_eviction / queue_restore (full profile)",
                  C, with(D, {"event"}));
  f_pod_kfd_ev_ = add("amd_pod_gpu_kfd_events_total",
                      "Per-process KFD SMI events (vm_fault, queue_eviction, queue_restore) of a pod's processes, "
                      "over all GPUs", C, {"namespace", "pod", "event"});

  // --- exporter self-metrics (own prefix; the reference registry had none, main.go:40) ---
  f_self_build_ = add("gpuexp_build_info", "Exporter build and backend", G, {"version", "backend"});
  f_self_ticks_ = add("gpuexp_ticks_total", "Sampler ticks completed", C, {});
  f_self_pods_complete_ = add("gpuexp_pod_list_complete",
                              "1 if the applied pod list came from a refresh in which every metadata source "
                              "answered (per-pod totals of pods missing from it are dropped at once); 0: a source "
                              "failed, and totals of missing pods are kept for pod_totals_ttl (1 h)",
                              G, {});
  f_self_kfd_scans_ = add("gpuexp_kfd_proc_scans_total",
                          "KFD process scans by kind: list (the /sys/class/kfd/kfd/proc directory was listed: "
                          "its mtime moved, a tracked process left, or kfd_rescan_interval passed) or tracked "
                          "(only the known processes' files were read)",
                          C, {"kind"});
  f_self_kfd_tracked_ = add("gpuexp_kfd_procs_tracked",
                            "Processes in the KFD proc directory the exporter tracks (any GPU of the node)", G, {});
  f_self_startup_ = add("gpuexp_startup_seconds",
                        "Engine start to its first sample: backend init (amdsmi + raw-path validation), one "
                        "HSA queue per GPU with PMC programs and sentinel, plugin probes",
                        G, {});
  f_self_last_ = add("gpuexp_last_sample_timestamp_seconds",
                     "Unix time of the tick that produced this exposition (alert on time() - this: a stuck "
                     "sampler keeps serving its last snapshot)", G, {});
  f_self_stage_ = add("gpuexp_sample_stage_duration_seconds", "Sampler stage duration", H, {"stage"});
  // counters, not histograms: 6 parts x 11 bucket lines would be re-rendered and re-gzipped
  // every tick for a split whose means (rate / rate(gpuexp_ticks_total)) are what matters
  f_self_dev_part_ = add("gpuexp_device_read_seconds_total",
                         "The devices stage split: time in each part (counters_kick: PMC read submitted; "
                         "control: control-plane apply; gpu_metrics: SMU fetch or cached decode; vram; ras; "
                         "gtt; these three timed on one tick in four and scaled), summed over GPUs", C, {"part"});
  f_self_fetch_cpu_ = add("gpuexp_gpu_metrics_fetch_cpu_seconds_total",
                          "Thread CPU of fresh gpu_metrics reads (each one an SMU round trip the kernel "
                          "busy-waits on)", C, {"gpu"});
  f_self_fetch_cap_ = add("gpuexp_gpu_metrics_min_interval_seconds",
                          "Current cap on fresh gpu_metrics reads per GPU (metrics_min_interval; auto: the "
                          "measured fetch CPU x GPUs / metrics_cpu_budget)", G, {"gpu"});
  f_self_metrics_age_ = add("gpuexp_gpu_metrics_age_seconds",
                            "Age of the GPU's gpu_metrics table at this tick: seconds since it was last fetched "
                            "fresh from the SMU (0 on a fresh tick).  The families it feeds (power, temperatures, "
                            "clocks, activity, throttle residency, xGMI/PCIe bytes) are this old; under the auto "
                            "fetch policy it cycles up to about the min interval", G, {"gpu"});
  f_self_scrape_ = add("gpuexp_scrape_duration_seconds", "Server-side /metrics latency (request parsed -> last byte written)",
                       H, {});
  f_self_scrapes_ = add("gpuexp_scrapes_total", "Scrapes of the metrics path", C, {});
  f_self_http_bytes_ = add("gpuexp_http_response_bytes_total", "HTTP response bytes written", C, {});
  f_self_prewake_ = add("gpuexp_http_prewake_wakeups_total",
                        "Timer wake-ups of the HTTP worker ahead of expected scrapes (scrape-phase pre-wake)", C, {});
  f_self_prewake_hits_ = add("gpuexp_http_prewake_hits_total",
                             "Scrapes of the metrics path that arrived while their HTTP worker was pre-woken "
                             "(its pre-wake timer fired within the lead + one slice before the request)",
                             C, {});
  f_self_prewake_hits_narrow_ = add("gpuexp_http_prewake_hits_narrow_total",
                                    "Pre-woken scrapes under round 3's narrower window (timer fired within the "
                                    "minimum lead + one slice before the request)", C, {});
  f_self_prewake_spins_ = add("gpuexp_http_prewake_spins_total",
                              "Spin pre-wake windows the HTTP worker polled in, by how they ended: a /metrics "
                              "request arrived (hit) or the window ran out (timeout)", C, {"outcome"});
  f_self_prewake_spin_s_ = add("gpuexp_http_prewake_spin_seconds_total",
                               "Wall time the HTTP worker spent polling in spin pre-wake windows (the CPU the "
                               "spin mode costs)", C, {});
  f_self_rx_moves_ = add("gpuexp_http_rx_cpu_moves_total",
                         "Times an HTTP worker moved to the CPU a steady scraper's requests arrive on "
                         "(http follow_rx_cpu; 0 when off)",
                         C, {});
  f_self_gzip_ = add("gpuexp_gzip_compressions_total",
                     "gzip compressions of the exposition: by the sampler (a gzip scrape was expected before "
                     "the next tick) or per request (off schedule)",
                     C, {"where"});
  f_self_render_bytes_ = add("gpuexp_render_bytes", "Size of the last rendered exposition", G, {});
  f_self_expo_ = add("gpuexp_exposition_events_total",
                     "Compiled exposition: families laid out again (a series appeared or went, a value outgrew "
                     "its field), segments parsed on their own while their layout settled, and Huffman code "
                     "builds (0 per tick in steady state)", C, {"event"});
  f_self_series_ = add("gpuexp_series", "Series in the last rendered exposition", G, {});
  f_self_dev_errors_ = add("gpuexp_device_errors_total", "Failed telemetry reads per GPU", C, {"gpu"});
  f_self_overruns_ = add("gpuexp_tick_overruns_total", "Ticks skipped because a tick ran past its deadline", C, {});
  f_self_cpu_ = add("gpuexp_sampler_cpu_seconds_total",
                    "CPU time of the sampling work: the sampler thread, its per-GPU read threads and the PMC "
                    "counter thread (not the HTTP server)", C, {});
  f_self_source_up_ = add("gpuexp_source_up", "1 if an optional source is active", G, {"source"});
  f_self_metrics_reads_ = add("gpuexp_gpu_metrics_reads_total",
                              "gpu_metrics reads by kind: fresh (SMU table fetch) or coalesced (cached table, "
                              "PMFW had not refreshed yet)",
                              C, {"gpu", "kind"});
  f_self_metrics_period_ = add("gpuexp_gpu_metrics_refresh_period_seconds",
                               "PMFW gpu_metrics refresh period learnt from firmware timestamps (0 = learning)",
                               G, {"gpu"});
  f_self_unresolved_ = add("gpuexp_pods_unresolved",
                           "Pod UIDs found in GPU processes' cgroups that the control plane has not named "
                           "yet (their series carry pod=\"\" and no legacy series until it does)",
                           G, {});
  f_self_rccl_files_ = add("gpuexp_rccl_files",
                           "RCCL tracer directory entries by state: active (writer identified, exported), "
                           "unverified (no live process maps it as claimed), exited (writer gone, file left "
                           "behind), ignored (not a tracer file, not a regular file, or over the 1024-file cap)",
                           G, {"state"});
  f_self_rccl_scans_ = add("gpuexp_rccl_dir_scans_total",
                           "Listings of the RCCL tracer directory (only when it changed, at most once per "
                           "rccl_scan_interval_s)", C, {});
  f_self_ctr_late_ = add("gpuexp_counters_late_ticks_total",
                         "Ticks that exported the previous counter window because this tick's PMC read had not "
                         "completed within counters_sync_us (continuous counters)",
                         C, {});
  f_self_ctr_events_ = add("gpuexp_counters_events_total",
                           "PMC read health per GPU: read_stall (a read still queued at the round's end), "
                           "reset (a window dropped: counters went backwards), rearm (counting restarted after "
                           "another profiler reset or stopped it), rescue / rescue_release (reads moved to a "
                           "queue of their own behind a starved sentinel run, and back)",
                           C, {"gpu", "event"});
  f_self_ctr_rescue_ = add("gpuexp_counters_rescue_active",
                           "1 while a GPU's PMC reads run on a rescue queue (+173 MiB pinned while it lasts)", G,
                           {"gpu"});
  f_self_ctr_scope_ = add("gpuexp_counters_device_scope",
                          "1 if wave/LDS/HBM PMC counters see every process on the GPU, 0 if they are "
                          "VMID-filtered to the exporter (not exported then)",
                          G, {"gpu"});
}

namespace {
// Runtime libraries started here (amdsmi, ROCr/HSA, HIP) create threads of their own, which
// inherit the creating thread's name: named "gpuexp-rt" they show apart from the host
// process's threads in per-thread CPU accounting (bench.py exporter_cpu_us_per_step_by_thread).
struct RuntimeThreadsName {
  char saved[17] = {};
  RuntimeThreadsName() {
    ::prctl(PR_GET_NAME, saved, 0, 0, 0);
    set_thread_name("gpuexp-rt");
  }
  ~RuntimeThreadsName() { set_thread_name(saved); }
};
}  // namespace

bool Engine::start(std::string* err) {
  if (running_.load()) return true;
  RuntimeThreadsName rt_name;
  start_mono_ns_ = mono_ns();
  compiled_ = cfg_.exposition != "classic";
  counters_kick_mode_ = cfg_.counters_kick != "auto" ? cfg_.counters_kick
                        : (cfg_.interval_s > 0 && cfg_.interval_s < 0.05 ? "end" : "start");
  define_families();
  // Listen first: a port conflict fails before any GPU-side source (amdsmi, HSA queues,
  // sentinel runs) exists.  Every later failure tears down what was already started.
  if (cfg_.serve_http) {
    HttpConfig hc = cfg_.http;
    hc.gzip_level = cfg_.gzip_level;
    if (const char* e = std::getenv("GPUEXP_HTTP_FOLLOW_RX_CPU")) hc.follow_rx_cpu = e[0] != '0';
    // experiment knobs (A/B on a box): pre-wake slice and minimum lead, microseconds
    if (const char* e = std::getenv("GPUEXP_HTTP_PREWAKE_STEP_US")) hc.prewake_step_ns = uint64_t(std::atoll(e)) * 1000;
    if (const char* e = std::getenv("GPUEXP_HTTP_PREWAKE_LEAD_US")) hc.prewake_lead_ns = uint64_t(std::atoll(e)) * 1000;
    if (const char* e = std::getenv("GPUEXP_HTTP_PREWAKE_SPIN_MAX_US"))
      hc.prewake_spin_max_ns = uint64_t(std::atoll(e)) * 1000;
    http_ = std::make_unique<HttpServer>(&store_, hc);
    if (!http_->start(err)) {
      http_.reset();
      return false;
    }
  }
  bool ok = false;
  struct Undo {
    Engine* e;
    bool* ok;
    ~Undo() {
      if (*ok) return;
      if (e->http_) e->http_->stop();
      e->http_.reset();
      if (e->backend_) e->backend_->shutdown();
      e->backend_.reset();
      e->mock_ = nullptr;
      e->devices_.clear();
    }
  } undo{this, &ok};
  if (cfg_.backend == "mock") {
    auto m = std::make_unique<MockBackend>(cfg_.mock_devices);
    mock_ = m.get();
    backend_ = std::move(m);
  } else if (cfg_.backend == "sysfs") {
    backend_ = std::make_unique<SysfsBackend>(cfg_.host_root);
  } else if (cfg_.backend == "amdsmi") {
    backend_ = make_amdsmi_backend(cfg_.host_root, cfg_.process_source == "amdsmi", cfg_.force_amdsmi_metrics);
  } else {
    *err = "unknown backend: " + cfg_.backend;
    return false;
  }
  backend_->set_metrics_coalescing(cfg_.metrics_coalesce);
  backend_->set_metrics_min_interval(uint64_t(std::max(0.0, cfg_.metrics_min_interval_s) * 1e9));
  backend_->set_fake_metrics_cost(cfg_.fake_metrics_cost_us * 1000ull);
  std::vector<DeviceInfo> all;
  if (!backend_->init(&all, err)) return false;
  if (!cfg_.device_filter.empty() || !cfg_.device_filter_bdf.empty()) {
    auto lower = [](std::string x) {
      for (auto& ch : x) ch = char(::tolower(static_cast<unsigned char>(ch)));
      return x;
    };
    for (auto& d : all) {
      bool want = std::find(cfg_.device_filter.begin(), cfg_.device_filter.end(), d.index) != cfg_.device_filter.end();
      for (const auto& b : cfg_.device_filter_bdf) want = want || lower(b) == lower(d.bdf);
      if (want) devices_.push_back(d);
    }
    // keep backend indices: DeviceInfo::index addresses the backend's own table
  } else {
    devices_ = all;
  }
  if (!cfg_.queue_devices.empty() || !cfg_.queue_devices_bdf.empty()) {
    for (auto& d : devices_) {
      bool on = std::find(cfg_.queue_devices.begin(), cfg_.queue_devices.end(), d.index) != cfg_.queue_devices.end();
      for (const auto& b : cfg_.queue_devices_bdf) on = on || lower(b) == lower(d.bdf);
      d.queue_enabled = on;
    }
  }
  const bool any_queue = std::any_of(devices_.begin(), devices_.end(), [](const DeviceInfo& d) {
    return d.queue_enabled;
  });
  dstate_.assign(devices_.size(), DevState());
  owner_keys_.clear();
  for (const DeviceInfo& d : devices_) owner_keys_.push_back(device_owner_keys(d));
  metrics_fresh_.assign(devices_.size(), 0);
  metrics_coalesced_.assign(devices_.size(), 0);
  if (cfg_.series_profile == "full" && cfg_.backend != "mock") {
    const std::string root = cfg_.host_root.empty() ? "" : cfg_.host_root;
    ras_.resize(devices_.size());
    for (size_t i = 0; i < devices_.size(); ++i) {
      const DeviceInfo& di = devices_[i];
      if (di.render_minor >= 0)
        ras_[i].open(root + "/sys/class/drm/renderD" + std::to_string(di.render_minor) + "/device");
      else if (!di.bdf.empty())
        ras_[i].open(root + "/sys/bus/pci/devices/" + di.bdf);
    }
    ras_cache_.assign(devices_.size(), RasTotals());
    ras_next_ns_.assign(devices_.size(), 0);
    // GTT lives on the PCI function (a partition's amdgpu_xcp node has no mem_info_*)
    gtt_used_f_.resize(devices_.size());
    gtt_total_.assign(devices_.size(), kNaN);
    for (size_t i = 0; i < devices_.size(); ++i) {
      const DeviceInfo& di = devices_[i];
      for (const std::string& dir : {root + "/sys/class/drm/renderD" + std::to_string(di.render_minor) + "/device",
                                     root + "/sys/bus/pci/devices/" + di.bdf}) {
        if (!gtt_used_f_[i].open(dir + "/mem_info_gtt_used")) continue;
        std::string body;
        uint64_t v = 0;
        if (read_small_file(dir + "/mem_info_gtt_total", &body) && parse_u64(body.data(), body.size(), &v))
          gtt_total_[i] = double(v);
        break;
      }
    }
  }
  // auto = serial: a fresh gpu_metrics read is kernel busy-wait (its CPU is the same on any
  // thread) and waking a pool costs more CPU than the parallel reads save wall time
  // (8 fake GPUs at 100 Hz: 9.8 % vs 6.3 % of a core, profiles/r04/devices_split.txt); a
  // pool only shortens the tick's wall time (8 x 0.45 ms at most), so it stays opt-in.
  int nthreads = cfg_.device_threads;
  if (nthreads <= 0) nthreads = 1;
  if (nthreads > 1) pool_ = std::make_unique<ForkJoinPool>(nthreads);
  kfd_ = std::make_unique<KfdProcReader>(cfg_.host_root, cfg_.exclude_self ? self_pid_ : -1, cfg_.kfd_cu_occupancy,
                                         uint64_t(cfg_.kfd_detail_interval_s * 1e9),
                                         uint64_t(cfg_.kfd_rescan_interval_s * 1e9), cfg_.kfd_sdma);
  resolver_ = std::make_unique<PidResolver>(cfg_.host_root);

  // Counters first: the rocprofiler tool must register before the HSA runtime loads,
  // which the sentinel's first HIP call does.
  if (cfg_.enable_counters && cfg_.backend != "mock" && !any_queue) {
    counters_status_ = "disabled: no GPU in queue_devices";
  } else if (cfg_.enable_counters && cfg_.backend != "mock") {
    const bool continuous = cfg_.counters_mode == "continuous";
    // continuous: every tick kicks a read; the plugin's own timer (2 ticks) only covers
    // engines without a sampler thread
    const int interval_ms = continuous && cfg_.interval_s > 0 ? std::max(10, int(cfg_.interval_s * 2000))
                                                              : cfg_.counters_interval_ms;
    // a periodic sampler runs each tick's read round itself (kick / sync): no wake-ups of the
    // plugin's counting thread per tick (~30-55 us of CPU per tick on MI355X, profiles/r04)
    const bool inline_rounds = continuous && cfg_.interval_s > 0 && cfg_.counters_inline;
    counters_ = make_rocprof_counters(cfg_.counters_plugin, cfg_.counters_window_ms, interval_ms, continuous,
                                      inline_rounds);
    std::string e;
    if (!counters_ || !counters_->start(devices_, &e)) {
      counters_status_ = "unavailable: " + e;
      GPUEXP_LOG(LogLevel::kWarn, "counters", counters_status_);
      counters_.reset();
    } else {
      counters_status_ = counters_->status();
    }
  } else if (cfg_.enable_counters) {
    counters_status_ = "mock";
  }
  if (cfg_.enable_sentinel && cfg_.backend != "mock" && !any_queue) {
    sentinel_status_ = "disabled: no GPU in queue_devices";
  } else if (cfg_.enable_sentinel && cfg_.backend != "mock") {
    std::string e;
    // Prefer the counters plugin's queue (one GPU queue, and its ~173 MiB context save
    // area, per GPU instead of two); the HIP plugin's own stream otherwise.
    if (cfg_.sentinel_impl != "hip" && counters_) {
      sentinel_ = make_queue_sentinel(cfg_.counters_plugin, cfg_.sentinel_ring, cfg_.sentinel_spin);
      if (sentinel_ && !sentinel_->start(devices_, &e)) {
        GPUEXP_LOG(LogLevel::kInfo, "sentinel", "queue sentinel unavailable (" + e + "), using HIP");
        sentinel_.reset();
      }
    }
    if (!sentinel_ && cfg_.sentinel_impl != "queue") {
      sentinel_ = make_hip_sentinel(cfg_.sentinel_ring, cfg_.sentinel_spin);
      e = "libgpuexp_hip.so not loadable";
      if (sentinel_ && !sentinel_->start(devices_, &e)) sentinel_.reset();
    }
    if (!sentinel_) {
      sentinel_status_ = "unavailable: " + e;
      GPUEXP_LOG(LogLevel::kWarn, "sentinel", sentinel_status_);
      sentinel_.reset();
    } else {
      sentinel_status_ = sentinel_->status();
    }
  } else if (cfg_.enable_sentinel) {
    sentinel_status_ = "mock";
  }
  if (cfg_.enable_rccl) rccl_ = make_rccl_source(cfg_.rccl_dir, cfg_.rccl_verify, cfg_.rccl_scan_interval_s);
  {
    std::string v;
    driver_version_ = read_small_file((cfg_.host_root.empty() ? "" : cfg_.host_root) + "/sys/module/amdgpu/version", &v, 128)
                          ? trim(v)
                          : (mock_ ? "mock" : "in-kernel");  // DKMS builds carry a version file
    struct utsname u{};
    kernel_release_ = ::uname(&u) == 0 ? u.release : "";
  }
  if (!cfg_.state_file.empty()) load_state();
  if (cfg_.enable_kfd_events && cfg_.series_profile == "full") {
    kfd_events_ = std::make_unique<KfdEventSource>();
    if (mock_) {
      kfd_events_->set_devices(devices_.size());  // events arrive through inject_kfd_events only
      kfd_events_status_ = "mock (injected events)";
    } else {
      std::string e;
      const int n = kfd_events_->open(devices_, cfg_.kfd_path, &e);
      if (n == 0) {
        kfd_events_status_ = "unavailable: " + e;
        GPUEXP_LOG(LogLevel::kWarn, "kfd_events", kfd_events_status_);
        kfd_events_.reset();
      } else {
        kfd_events_status_ = "on " + std::to_string(n) + " GPU(s), " +
                             (kfd_events_->all_processes() ? "every process's events"
                                                           : "device-wide events + own process (no CAP_SYS_ADMIN)");
      }
    }
  }

  if (!cfg_.trace_path.empty()) {
    trace_ = std::fopen(cfg_.trace_path.c_str(), "w");
    if (trace_) {
      std::fputs("[\n", trace_);
      trace_t0_ = mono_ns();
    }
  }
  ok = true;
  running_.store(true);
  if (cfg_.interval_s > 0) {
    stop_fd_ = ::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
    sampler_ = std::thread([this] { run_sampler(); });
  }
  return true;
}

void Engine::stop() {
  if (!running_.exchange(false)) return;
  if (stop_fd_ >= 0) {
    uint64_t one = 1;
    ssize_t r = ::write(stop_fd_, &one, sizeof(one));
    (void)r;
  }
  if (sampler_.joinable()) sampler_.join();
  if (stop_fd_ >= 0) ::close(stop_fd_);
  stop_fd_ = -1;
  if (!cfg_.state_file.empty()) {
    std::lock_guard<std::mutex> lk(tick_mu_);
    save_state();
  }
  if (http_) http_->stop();
  if (sentinel_) sentinel_->stop();
  if (counters_) counters_->stop();
  if (backend_) backend_->shutdown();
  if (trace_) {
    std::fputs("{}]\n", trace_);
    std::fclose(trace_);
    trace_ = nullptr;
  }
}

void Engine::run_sampler() {
  set_thread_name("gpuexp-sampler");
  tl_sampler_thread = true;
  int tfd = ::timerfd_create(CLOCK_MONOTONIC, TFD_CLOEXEC);
  uint64_t period = uint64_t(cfg_.interval_s * 1e9);
  if (period < 1000000) period = 1000000;  // 1 kHz cap
  itimerspec its{};
  its.it_interval.tv_sec = time_t(period / 1000000000ull);
  its.it_interval.tv_nsec = long(period % 1000000000ull);
  its.it_value.tv_nsec = 1;  // first tick immediately
  ::timerfd_settime(tfd, 0, &its, nullptr);
  pollfd fds[2] = {{tfd, POLLIN, 0}, {stop_fd_, POLLIN, 0}};
  while (running_.load()) {
    int n = ::poll(fds, 2, -1);
    if (n < 0) continue;
    if (fds[1].revents & POLLIN) break;
    if (fds[0].revents & POLLIN) {
      uint64_t expirations = 0;
      ssize_t r = ::read(tfd, &expirations, sizeof(expirations));
      if (r != sizeof(expirations)) continue;
      if (expirations > 1) {
        std::lock_guard<std::mutex> lk(stats_mu_);
        stats_.overruns += expirations - 1;
      }
      std::lock_guard<std::mutex> lk(tick_mu_);
      tick_locked(mono_ns());
    }
  }
  ::close(tfd);
}

void Engine::tick_now(uint64_t now_ns) {
  std::lock_guard<std::mutex> lk(tick_mu_);
  tick_locked(now_ns);
}

void Engine::set_pods(std::vector<PodMeta> pods, bool complete) {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_pods_ = std::move(pods);
  ctl_dirty_ = true;
  pending_complete_ = complete;
}

void Engine::set_device_owners(std::vector<std::pair<std::string, DeviceOwner>> owners) {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_owners_ = std::move(owners);
  ctl_dirty_ = true;
}

void Engine::inject_kfd_events(int dev, const std::string& bytes) {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_kfd_bytes_.emplace_back(dev, bytes);
}

// Drains the KFD event fds (and injected bytes) into per-GPU counts and, for events that
// name a process, per-pod counts (PID -> cgroup -> pod, cached by the resolver, so a
// process killed by its own VM fault is still attributed if it was seen before).
void Engine::count_kfd_events() {
  std::vector<KfdEvent> evs;
  kfd_events_->drain(&evs);
  {
    std::lock_guard<std::mutex> lk(ctl_mu_);
    for (auto& b : pending_kfd_bytes_) kfd_events_->feed(b.first, b.second.data(), b.second.size(), &evs);
    pending_kfd_bytes_.clear();
  }
  for (const KfdEvent& e : evs) {
    if (e.dev < 0 || size_t(e.dev) >= dstate_.size() || e.event <= 0 || e.event >= kKfdEventIds) continue;
    dstate_[size_t(e.dev)].kfd_events[e.event] += 1;
    if (e.pid <= 0) continue;
    const CgroupInfo* ci = cfg_.pod_attribution ? resolver_->resolve(e.pid) : nullptr;
    auto pit = ci && ci->kube ? pods_by_uid_.find(ci->pod_uid) : pods_by_uid_.end();
    if (pit == pods_by_uid_.end()) {
      ++kfd_events_unattributed_;
      continue;
    }
    pod_kfd_events_[std::make_tuple(pit->second.ns, pit->second.name, e.event)] += 1;
  }
}

void Engine::emit_kfd_events(uint64_t gen) {
  // a pod's counts live as long as the control plane knows the pod
  std::set<std::pair<std::string, std::string>> live;
  for (auto& kv : pods_by_uid_) live.emplace(kv.second.ns, kv.second.name);
  for (auto it = pod_kfd_events_.begin(); it != pod_kfd_events_.end();) {
    const auto& k = it->first;
    // restored from the state file while the pod list is not here yet: keep (and export);
    // gone from a complete list, or from every partial one for the TTL: drop
    const std::pair<std::string, std::string> pk{std::get<0>(k), std::get<1>(k)};
    auto lk = pod_last_known_ns_.find(pk);
    if (lk == pod_last_known_ns_.end() && !live.count(pk))  // never listed yet: the TTL starts now
      lk = pod_last_known_ns_.emplace(pk, mono_ns()).first;
    const bool expired = lk != pod_last_known_ns_.end() && mono_ns() - lk->second > uint64_t(cfg_.pod_totals_ttl_s * 1e9);
    if (!live.count(pk) && (pods_complete_ || expired)) {
      it = pod_kfd_events_.erase(it);
      continue;
    }
    table_.put(f_pod_kfd_ev_, {std::get<0>(k), std::get<1>(k), kfd_event_name(std::get<2>(k))}, double(it->second),
               gen);
    ++it;
  }
}

std::string Engine::device_key(size_t i) const {
  return lower(devices_[i].bdf) + "/" + std::to_string(devices_[i].partition_id);
}

// State file: one record per line, tab-separated (Kubernetes names carry no tabs):
//   gpuexp-state 1
//   pod_energy <ns> <pod> <joules>
//   pod_event  <ns> <pod> <event id> <count>
//   pod_xgmi   <ns> <pod> <read bytes> <write bytes>
//   dev_event  <bdf>/<partition> <event id> <count>
void Engine::load_state() {
  std::string body;
  if (!read_small_file(cfg_.state_file, &body, 16u << 20)) {
    set_state_status("no state yet (" + cfg_.state_file + ")");
    return;
  }
  if (body.compare(0, 14, "gpuexp-state 1") != 0) {
    set_state_status("ignored: unknown format in " + cfg_.state_file);
    GPUEXP_LOG(LogLevel::kWarn, "state", "ignored: unknown format in " + cfg_.state_file);
    return;
  }
  std::unordered_map<std::string, size_t> dev_by_key;
  for (size_t i = 0; i < devices_.size(); ++i) dev_by_key[device_key(i)] = i;
  size_t n = 0, pos = body.find('\n');
  while (pos != std::string::npos && pos + 1 < body.size()) {
    size_t eol = body.find('\n', pos + 1);
    const std::string line = body.substr(pos + 1, (eol == std::string::npos ? body.size() : eol) - pos - 1);
    pos = eol;
    std::vector<std::string> f;
    for (size_t a = 0, b; a <= line.size(); a = b + 1) {
      b = line.find('\t', a);
      if (b == std::string::npos) b = line.size();
      f.push_back(line.substr(a, b - a));
    }
    if (f[0] == "pod_energy" && f.size() == 4) {
      pod_energy_j_[{f[1], f[2]}] = std::strtod(f[3].c_str(), nullptr);
      ++n;
    } else if (f[0] == "pod_xgmi" && f.size() == 5) {
      pod_xgmi_[{f[1], f[2]}] = {std::strtod(f[3].c_str(), nullptr), std::strtod(f[4].c_str(), nullptr)};
      ++n;
    } else if (f[0] == "pod_gpu_seconds" && f.size() == 5) {
      pod_gpu_s_[{f[1], f[2]}] = {std::strtod(f[3].c_str(), nullptr), std::strtod(f[4].c_str(), nullptr)};
      ++n;
    } else if (f[0] == "pod_event" && f.size() == 5) {
      const int ev = std::atoi(f[3].c_str());
      if (ev > 0 && ev < kKfdEventIds) pod_kfd_events_[std::make_tuple(f[1], f[2], ev)] = std::strtoull(f[4].c_str(), nullptr, 10);
      ++n;
    } else if (f[0] == "dev_event" && f.size() == 4) {
      auto it = dev_by_key.find(f[1]);
      const int ev = std::atoi(f[2].c_str());
      if (it != dev_by_key.end() && ev > 0 && ev < kKfdEventIds)
        dstate_[it->second].kfd_events[ev] = std::strtoull(f[3].c_str(), nullptr, 10);
      ++n;
    }
  }
  set_state_status("restored " + std::to_string(n) + " records from " + cfg_.state_file);
  GPUEXP_LOG(LogLevel::kInfo, "state", "restored " + std::to_string(n) + " records from " + cfg_.state_file);
}

bool Engine::save_state() {
  state_saved_ns_ = mono_ns();
  std::string out = "gpuexp-state 1\n";
  char num[64];
  for (auto& kv : pod_energy_j_) {
    std::snprintf(num, sizeof(num), "%.17g", kv.second);
    out += "pod_energy\t" + kv.first.first + "\t" + kv.first.second + "\t" + num + "\n";
  }
  for (auto& kv : pod_xgmi_) {
    char rd[64], wr[64];
    std::snprintf(rd, sizeof(rd), "%.17g", kv.second.first);
    std::snprintf(wr, sizeof(wr), "%.17g", kv.second.second);
    out += "pod_xgmi\t" + kv.first.first + "\t" + kv.first.second + "\t" + rd + "\t" + wr + "\n";
  }
  for (auto& kv : pod_gpu_s_) {
    char al[64], bu[64];
    std::snprintf(al, sizeof(al), "%.17g", kv.second.first);
    std::snprintf(bu, sizeof(bu), "%.17g", kv.second.second);
    out += "pod_gpu_seconds\t" + kv.first.first + "\t" + kv.first.second + "\t" + al + "\t" + bu + "\n";
  }
  for (auto& kv : pod_kfd_events_)
    out += "pod_event\t" + std::get<0>(kv.first) + "\t" + std::get<1>(kv.first) + "\t" +
           std::to_string(std::get<2>(kv.first)) + "\t" + std::to_string(kv.second) + "\n";
  for (size_t i = 0; i < dstate_.size() && i < devices_.size(); ++i)
    for (int ev = 1; ev < kKfdEventIds; ++ev)
      if (dstate_[i].kfd_events[ev])
        out += "dev_event\t" + device_key(i) + "\t" + std::to_string(ev) + "\t" +
               std::to_string(dstate_[i].kfd_events[ev]) + "\n";
  // write + fsync + rename + fsync(dir): after a node crash the file is the old state or
  // the new one, never a renamed-but-empty one (the point of a hostPath checkpoint)
  const std::string tmp = cfg_.state_file + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "w");
  bool ok = f && std::fwrite(out.data(), 1, out.size(), f) == out.size();
  if (f) ok = std::fflush(f) == 0 && ::fsync(::fileno(f)) == 0 && ok;
  if (f) ok = (std::fclose(f) == 0) && ok;
  ok = ok && std::rename(tmp.c_str(), cfg_.state_file.c_str()) == 0;
  if (ok) {
    const size_t sl = cfg_.state_file.rfind('/');
    const std::string dir = sl == std::string::npos ? "." : (sl == 0 ? "/" : cfg_.state_file.substr(0, sl));
    const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    if (dfd >= 0) {
      ::fsync(dfd);
      ::close(dfd);
    }
  }
  if (!ok) {
    set_state_status("save failed: " + cfg_.state_file);
    GPUEXP_LOG(LogLevel::kWarn, "state", "save failed: " + cfg_.state_file);
  }
  return ok;
}

void Engine::set_pid_cgroup(int pid, const std::string& cgroup_path) {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_overrides_.emplace_back(pid, cgroup_path);
}

void Engine::clear_pid_cgroups() {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_overrides_.clear();
  clear_overrides_ = true;
}

void Engine::trace_event(const char* name, uint64_t start_ns, uint64_t dur_ns) {
  if (!trace_ || trace_events_ >= cfg_.trace_max_events) return;
  ++trace_events_;
  std::fprintf(trace_, "{\"name\":\"%s\",\"ph\":\"X\",\"ts\":%.3f,\"dur\":%.3f,\"pid\":%d,\"tid\":1},\n", name,
               double(start_ns - trace_t0_) * 1e-3, double(dur_ns) * 1e-3, self_pid_);
}

void Engine::dput(DevState& st, int dev, SeriesRef& r, int fid, std::initializer_list<const char*> extra,
                  double v, uint64_t gen) {
  if (std::isnan(v)) return;
  if (table_.set(r, v, gen)) return;  // the per-tick path: no allocation, no hashing
  const DeviceInfo& d = devices_[size_t(dev)];
  std::vector<std::string> labels = {std::to_string(d.index), d.bdf, st.owner.ns, st.owner.pod,
                                     st.owner.container};
  for (const char* e : extra) labels.emplace_back(e);
  r = table_.upsert(fid, labels);
  table_.set(r, v, gen);
}

void Engine::collect_device(int i, uint64_t gen, double dt_s) {
  DevState& st = dstate_[size_t(i)];
  const DeviceInfo& d = devices_[size_t(i)];
  const DeviceSample& c = st.cur;
  // Owner change -> rebuild every cached handle with the new pod labels.
  if (!st.owner_built_set || st.owner.ns != st.owner_built.ns || st.owner.pod != st.owner_built.pod ||
      st.owner.container != st.owner_built.container) {
    DeviceOwner keep = st.owner;
    DevState fresh;
    fresh.cur = st.cur;
    fresh.prev = st.prev;
    fresh.have_prev = st.have_prev;
    std::copy(std::begin(st.xgmi_rd_rate), std::end(st.xgmi_rd_rate), std::begin(fresh.xgmi_rd_rate));
    std::copy(std::begin(st.xgmi_wr_rate), std::end(st.xgmi_wr_rate), std::begin(fresh.xgmi_wr_rate));
    fresh.rates_valid = st.rates_valid;
    std::copy(std::begin(st.thr_last), std::end(st.thr_last), std::begin(fresh.thr_last));
    std::copy(std::begin(st.xcc_last), std::end(st.xcc_last), std::begin(fresh.xcc_last));
    fresh.errors = st.errors;
    fresh.err_ref = st.err_ref;
    fresh.fetch_cost_ns = st.fetch_cost_ns;  // the fetch policy's state is the GPU's, not the owner's
    fresh.fetch_cpu_s = st.fetch_cpu_s;
    fresh.fetch_cap_ns = st.fetch_cap_ns;
    fresh.metrics_fresh_ns = st.metrics_fresh_ns;
    std::copy(std::begin(st.kfd_events), std::end(st.kfd_events), std::begin(fresh.kfd_events));
    fresh.owner = keep;
    fresh.owner_built = keep;
    fresh.owner_built_set = true;
    st = fresh;
  }

  if (!table_.set(st.info, 1, gen)) {
    st.info = table_.upsert(f_info_, {std::to_string(d.index), d.bdf, d.uuid, d.name, std::to_string(d.kfd_gpu_id),
                                      d.render_minor >= 0 ? "renderD" + std::to_string(d.render_minor) : "",
                                      std::to_string(d.hip_id), std::to_string(d.partition_id),
                                      d.compute_partition, d.memory_partition, d.dev_node});
    table_.set(st.info, 1, gen);
  }
  dput(st, i, st.up, f_up_, {}, c.ok ? 1 : 0, gen);
  if (cfg_.series_profile == "full") {
    cput(st.board, f_board_, 1, gen, [&] {
      return std::vector<std::string>{std::to_string(d.index), d.bdf, d.product_name, d.product_number,
                                      d.serial_number, d.vbios_version};
    });
    if (cfg_.firmware_info) {
      st.fw.resize(d.firmware.size());
      for (size_t k = 0; k < d.firmware.size(); ++k)
        cput(st.fw[k], f_fw_, 1, gen, [&] {
          return std::vector<std::string>{std::to_string(d.index), d.bdf, d.firmware[k].first, d.firmware[k].second};
        });
    }
  }
  if (!table_.set(st.err_ref, double(st.errors), gen)) {
    st.err_ref = table_.upsert(f_self_dev_errors_, {std::to_string(d.index)});
    table_.set(st.err_ref, double(st.errors), gen);
  }
  if (kfd_events_) {
    // counted whether or not this tick's telemetry read worked: a reset shows here first
    for (size_t k = 0; k < std::size(kKfdSubscribed); ++k)
      dput(st, i, st.kev[k], f_kfd_ev_, {kfd_event_name(kKfdSubscribed[k])},
           double(st.kfd_events[kKfdSubscribed[k]]), gen);
  }
  if (!c.ok) return;  // a failed GPU exports only up=0 (+ errors); others unaffected
  bool compact = cfg_.series_profile == "compact";

  // A compute partition (CPX/DPX/QPX) is a slice of the socket: average_gfx_activity is the
  // socket's, so the logical GPU reports the mean busy of its own XCDs instead (below).
  const bool partitioned = c.num_partition > 1 || (!d.compute_partition.empty() && d.compute_partition != "SPX");
  if (!partitioned) dput(st, i, st.gfx, f_gfx_, {}, c.gfx_activity, gen);
  dput(st, i, st.umc, f_umc_, {}, c.umc_activity, gen);
  dput(st, i, st.vram_used, f_vram_used_, {}, c.vram_used, gen);
  dput(st, i, st.vram_total, f_vram_total_, {}, c.vram_total, gen);
  dput(st, i, st.power, f_power_, {}, c.power_w, gen);
  dput(st, i, st.power_cap, f_power_cap_, {}, c.power_cap_w, gen);
  if (c.energy_valid) dput(st, i, st.energy, f_energy_, {}, double(c.energy_acc) * c.energy_unit_j, gen);
  double temps[9] = {c.temp_hotspot, c.temp_mem, c.temp_vrsoc, c.temp_edge, c.temp_vrgfx, c.temp_vrmem,
                     c.temp_hbm[0], c.temp_hbm[1], c.temp_hbm[2]};
  for (int k = 0; k < 9; ++k) dput(st, i, st.temp[k], f_temp_, {kTempNames[k]}, temps[k], gen);
  double clks[3] = {c.clk_gfx, c.clk_soc, c.clk_mem};
  for (int k = 0; k < 3; ++k)
    dput(st, i, st.clk[k], f_clk_, {kClkNames[k]}, std::isnan(clks[k]) ? kNaN : clks[k] * 1e6, gen);
  if (!std::isnan(c.umc_activity) && !std::isnan(c.vram_max_bw_gbs))
    dput(st, i, st.hbm_bw, f_hbm_bw_, {}, c.umc_activity / 100.0 * c.vram_max_bw_gbs * 1e9, gen);

  // Rates from hardware accumulators over the PMFW timestamp delta (host time fallback).
  const DeviceSample& p = st.prev;
  bool have_prev = st.have_prev && p.ok;
  double dt_dev = 0;
  if (have_prev) {
    if (c.fw_ts_10ns && p.fw_ts_10ns && c.fw_ts_10ns > p.fw_ts_10ns)
      dt_dev = double(c.fw_ts_10ns - p.fw_ts_10ns) * 1e-8;
    else if (!(c.fw_ts_10ns && c.fw_ts_10ns == p.fw_ts_10ns) && c.host_ns > p.host_ns)
      dt_dev = double(c.host_ns - p.host_ns) * 1e-9;
  }
  if (c.xgmi_valid) {
    int links_up = 0;
    for (int l = 0; l < c.num_xgmi_links; ++l) {
      if (std::isnan(c.xgmi_link_up[l])) continue;
      links_up += c.xgmi_link_up[l] > 0;
      if (compact) continue;
      const char* ls = idx_str(l);
      const char* peer = d.xgmi_peer_bdf[l].c_str();
      dput(st, i, st.xrd[l], f_xrd_, {ls, peer}, double(c.xgmi_read_kb[l]) * 1024.0, gen);
      dput(st, i, st.xwr[l], f_xwr_, {ls, peer}, double(c.xgmi_write_kb[l]) * 1024.0, gen);
    }
    dput(st, i, st.links_up, f_links_up_, {}, double(links_up), gen);
    if (have_prev && p.xgmi_valid && dt_dev > 0) {
      bool ok = true;
      for (int l = 0; l < kMaxXgmiLinks; ++l) {
        double dr, dw;
        if (!acc_delta(c.xgmi_read_kb[l], p.xgmi_read_kb[l], &dr) ||
            !acc_delta(c.xgmi_write_kb[l], p.xgmi_write_kb[l], &dw)) {
          ok = false;  // counter reset: skip one rate sample
          continue;
        }
        st.xgmi_rd_rate[l] = dr * 1024.0 / dt_dev;
        st.xgmi_wr_rate[l] = dw * 1024.0 / dt_dev;
      }
      st.rates_valid = ok || st.rates_valid;
    }
    if (st.rates_valid) {
      double rs = 0, ws = 0;
      for (int l = 0; l < kMaxXgmiLinks; ++l) {
        rs += st.xgmi_rd_rate[l];
        ws += st.xgmi_wr_rate[l];
      }
      dput(st, i, st.xrd_rate, f_xrd_rate_, {}, rs, gen);
      dput(st, i, st.xwr_rate, f_xwr_rate_, {}, ws, gen);
    }
  }
  dput(st, i, st.pcie_bw, f_pcie_bw_, {}, std::isnan(c.pcie_bw_inst) ? kNaN : c.pcie_bw_inst * 125000.0, gen);
  dput(st, i, st.pcie_replay, f_pcie_replay_, {}, c.pcie_replay, gen);
  dput(st, i, st.pcie_speed, f_pcie_speed_, {}, c.pcie_speed_gts, gen);
  dput(st, i, st.pcie_width, f_pcie_width_, {}, c.pcie_width, gen);
  if (cfg_.series_profile == "full") {
    static const char* kEcc[3] = {"correctable", "uncorrectable", "deferred"};
    static const char* kAer[3] = {"correctable", "nonfatal", "fatal"};
    const double ecc[3] = {c.ecc_ce, c.ecc_ue, c.ecc_de};
    const double aer[3] = {c.aer_cor, c.aer_nonfatal, c.aer_fatal};
    for (int k = 0; k < 3; ++k) {
      dput(st, i, st.ecc[k], f_ecc_, {kEcc[k]}, ecc[k], gen);
      dput(st, i, st.aer[k], f_aer_, {kAer[k]}, aer[k], gen);
    }
    dput(st, i, st.pages[0], f_pages_, {"retired"}, c.pages_retired, gen);
    dput(st, i, st.pages[1], f_pages_, {"pending"}, c.pages_pending, gen);
    dput(st, i, st.pages[2], f_pages_, {"unreservable"}, c.pages_unreservable, gen);
    dput(st, i, st.gtt_used, f_gtt_used_, {}, c.gtt_used, gen);
    dput(st, i, st.gtt_total, f_gtt_total_, {}, c.gtt_total, gen);
    dput(st, i, st.nak[0], f_pcie_nak_, {"sent"}, c.pcie_nak_sent, gen);
    dput(st, i, st.nak[1], f_pcie_nak_, {"received"}, c.pcie_nak_rcvd, gen);
    dput(st, i, st.recov, f_pcie_recov_, {}, c.pcie_l0_recov, gen);
    dput(st, i, st.xgmi_w, f_xgmi_width_, {}, c.xgmi_width, gen);
    dput(st, i, st.xgmi_s, f_xgmi_speed_, {}, c.xgmi_speed, gen);
    for (int x = 0; x < kMaxXcc; ++x)
      if (!std::isnan(c.clk_gfx_xcc[x]))
        dput(st, i, st.xclk[x], f_xcc_clk_, {idx_str(int(x))}, c.clk_gfx_xcc[x] * 1e6, gen);
  }

  uint32_t nx = d.num_xcc ? std::min<uint32_t>(d.num_xcc, kMaxXcc) : kMaxXcc;
  if (have_prev && c.residency_valid && p.residency_valid) {
    double dacc;
    if (acc_delta(c.accumulation_counter, p.accumulation_counter, &dacc) && dacc > 0) {
      uint64_t cr[5] = {c.res_ppt, c.res_socket_thm, c.res_vr_thm, c.res_hbm_thm, c.res_prochot};
      uint64_t pr[5] = {p.res_ppt, p.res_socket_thm, p.res_vr_thm, p.res_hbm_thm, p.res_prochot};
      for (int k = 0; k < 5; ++k) {
        double dr;
        if (acc_delta(cr[k], pr[k], &dr)) st.thr_last[k] = std::min(100.0, dr * 100.0 / dacc);
      }
      for (uint32_t x = 0; x < nx; ++x) {
        double db;
        if (acc_delta(c.gfx_busy_acc[x], p.gfx_busy_acc[x], &db)) st.xcc_last[x] = std::min(100.0, db / dacc);
      }
    }
  }
  if (partitioned) {
    double sum = 0;
    int n = 0;
    for (uint32_t x = 0; x < nx; ++x)
      if (!std::isnan(st.xcc_last[x])) {
        sum += st.xcc_last[x];
        ++n;
      }
    dput(st, i, st.gfx, f_gfx_, {}, n ? sum / n : kNaN, gen);
  }
  for (int k = 0; k < 5; ++k) dput(st, i, st.thr[k], f_thr_, {kThrNames[k]}, st.thr_last[k], gen);
  if (!compact)
    for (uint32_t x = 0; x < nx; ++x) dput(st, i, st.xcc[x], f_xcc_, {idx_str(int(x))}, st.xcc_last[x], gen);

  // Optional sources: rocprofiler counters, sentinel (real or mock-simulated).
  st.mfma_last = kNaN;
  st.flops_last[0] = st.flops_last[1] = kNaN;
  CounterReading cr;
  bool have_ctr = false;
  if (counters_) have_ctr = counters_->sample(i, dt_s, &cr) && cr.ok;
  else if (cfg_.enable_counters) have_ctr = backend_->counters(d, dt_s, &cr) && cr.ok;
  if (have_ctr) {
    // Chip-global counters are always device totals.  Wave/LDS/EA counters are exported
    // only while they are known to see every process (scope 1, or the mock); scope 0
    // (VMID-filtered to the exporter) would under-report by orders of magnitude.
    int scope = counters_ ? counters_->scope(i) : 1;
    cput(st.self_reads[3], f_self_ctr_scope_, scope < 0 ? kNaN : double(scope), gen,
         [&] { return std::vector<std::string>{std::to_string(d.index)}; });
    dput(st, i, st.ctr[0], f_mfma_, {}, cr.mfma_busy_pct, gen);
    st.mfma_last = cr.mfma_busy_pct;
    if (cfg_.series_profile == "full") {
      dput(st, i, st.mfma_util, f_mfma_util_, {}, cr.mfma_util_pct, gen);
      for (int x = 0; x < cr.nxcc && x < kMaxXcc; ++x)
        dput(st, i, st.xmfma[x], f_xcc_mfma_, {idx_str(x)}, cr.xcc_mfma_busy_pct[x], gen);
    }
    dput(st, i, st.ctr[2], f_gui_, {}, cr.gui_active_pct, gen);
    if (scope != 0) {
      dput(st, i, st.ctr[1], f_sq_busy_, {}, cr.sq_busy_pct, gen);
      dput(st, i, st.ctr[3], f_waves_, {}, cr.waves_per_s, gen);
      dput(st, i, st.ctr[4], f_lds_, {}, cr.lds_active_pct, gen);
      dput(st, i, st.ctr[5], f_lds_conf_, {}, cr.lds_bank_conflict_pct, gen);
      dput(st, i, st.ctr[6], f_hbm_rd_, {}, cr.hbm_read_bps, gen);
      dput(st, i, st.ctr[7], f_hbm_wr_, {}, cr.hbm_write_bps, gen);
      if (cfg_.series_profile == "full") {  // not part of the 64-series standard load
        dput(st, i, st.ctr[8], f_remote_rd_, {}, cr.remote_read_bps, gen);
        dput(st, i, st.ctr[9], f_remote_wr_, {}, cr.remote_write_bps, gen);
        // SQ instruction counters: VMID-filtered like the wave counts, so device scope only
        dput(st, i, st.mflops[0], f_mfma_flops_, {"bf16"}, cr.mfma_bf16_flops, gen);
        dput(st, i, st.mflops[1], f_mfma_flops_, {"fp8"}, cr.mfma_fp8_flops, gen);
        st.flops_last[0] = cr.mfma_bf16_flops;
        st.flops_last[1] = cr.mfma_fp8_flops;
      }
    }
    if (cfg_.series_profile == "full") {
      // What capped residency, from the SPI resource allocator.  Not VMID-filtered like the
      // SQ wave counters: an unprivileged exporter sees other processes' waves on every
      // hardware queue (profiles/r04/spi_scope.txt), so exported at any scope.
      static const char* kRes[4] = {"lds", "wave_slots", "vgpr", "sgpr"};
      const double lim[4] = {cr.lds_limited_pct, cr.wave_limited_pct, cr.vgpr_limited_pct, cr.sgpr_limited_pct};
      dput(st, i, st.disp_stall, f_disp_stall_, {}, cr.dispatch_stall_pct, gen);
      for (int k = 0; k < 4; ++k) dput(st, i, st.occ_lim[k], f_occ_lim_, {kRes[k]}, lim[k], gen);
    }
  }
  CounterHealth ch;
  if (counters_ && cfg_.series_profile == "full" && counters_->health(i, &ch)) {
    static const char* kEv[5] = {"read_stall", "reset", "rearm", "rescue", "rescue_release"};
    const uint64_t v[5] = {ch.stalls, ch.resets, ch.rearms, ch.rescues, ch.releases};
    for (int k = 0; k < 5; ++k)
      cput(st.ctr_health[k], f_self_ctr_events_, double(v[k]), gen,
           [&] { return std::vector<std::string>{std::to_string(d.index), kEv[k]}; });
    cput(st.ctr_health[5], f_self_ctr_rescue_, ch.rescue_active ? 1 : 0, gen,
         [&] { return std::vector<std::string>{std::to_string(d.index)}; });
  }
  SentinelReading sr;
  bool have_sen = false;
  if (sentinel_) have_sen = sentinel_->read(i, &sr) && sr.ok;
  else if (cfg_.enable_sentinel) have_sen = backend_->sentinel(d, &sr) && sr.ok;
  if (have_sen) {
    dput(st, i, st.sen[0], f_sen_sclk_, {}, sr.sclk_hz, gen);
    dput(st, i, st.sen[1], f_sen_lat_, {}, sr.dispatch_latency_s, gen);
    dput(st, i, st.sen[2], f_sen_xcc_, {}, sr.xcc_id, gen);
    dput(st, i, st.sen[3], f_sen_runs_, {}, double(sr.runs), gen);
    if (cfg_.series_profile == "full") {
      dput(st, i, st.sen_pend, f_sen_pend_, {}, sr.pending_s, gen);
      dput(st, i, st.sen_mem, f_sen_mem_, {}, sr.mem_latency_s, gen);
      for (int x = 0; x < kMaxXcc; ++x) {
        if (!std::isnan(sr.xcc_latency_s[x]))
          dput(st, i, st.sen_xlat[x], f_sen_xlat_, {idx_str(int(x))}, sr.xcc_latency_s[x], gen);
        if (!std::isnan(sr.xcc_mem_latency_s[x]))
          dput(st, i, st.sen_xmem[x], f_sen_xmem_, {idx_str(int(x))}, sr.xcc_mem_latency_s[x], gen);
      }
    }
  }
}

void Engine::emit_processes(uint64_t gen, const std::vector<std::vector<ProcSample>>& per_dev) {
  // pid -> attribution, resolved once per tick (and kept while KFD vouches for the process)
  unresolved_.clear();
  std::vector<int>& live = live_scratch_;
  live.clear();
  for (auto& lst : per_dev)
    for (auto& p : lst) {
      ProcAttr& a = attr_cache_[p.pid];
      if (a.seen == gen) continue;
      a.seen = gen;
      live.push_back(p.pid);
      if (p.kfd_id && a.kfd_id == p.kfd_id && a.ctl_epoch == ctl_epoch_) {
        if (!a.uid.empty() && a.pod.empty()) unresolved_.insert(a.uid);
        continue;
      }
      a.ns.clear();
      a.pod.clear();
      a.container.clear();
      a.uid.clear();
      a.kfd_id = p.kfd_id;
      a.ctl_epoch = ctl_epoch_;
      if (cfg_.pod_attribution) {
        const CgroupInfo* ci = resolver_->resolve(p.pid, p.kfd_id);
        if (!ci) a.kfd_id = 0;  // not looked up (unreadable /proc/<pid>): ask the resolver again
        if (ci && ci->kube) {
          a.uid = ci->pod_uid;
          auto it = pods_by_uid_.find(ci->pod_uid);
          if (it != pods_by_uid_.end()) {
            a.ns = it->second.ns;
            a.pod = it->second.name;
          } else {
            // Name unknown until the control plane reports it: pod="" meanwhile (a UID
            // in `pod` would change the series identity once the name arrives).
            unresolved_.insert(ci->pod_uid);
          }
          auto cn = container_names_.find(ci->container_id);
          if (cn != container_names_.end()) a.container = cn->second;
        }
      }
    }
  for (auto it = attr_cache_.begin(); it != attr_cache_.end();)
    it = it->second.seen != gen ? attr_cache_.erase(it) : std::next(it);
  resolver_->gc(live);

  struct PidAgg {
    double used = 0, total = 0;
  };
  std::map<int, PidAgg> legacy;
  struct PodAgg {
    double vram = 0;
    std::set<int> pids;
    int gpus = 0;
    double xrd = 0, xwr = 0, power = 0, gfx = 0, gfx_share = 0;
    double energy_j = 0;  // this tick
    double xrd_b = 0, xwr_b = 0;  // xGMI bytes this tick (owned GPUs whole, shared GPUs by share)
    double mfma = 0, hbm = 0, flops[2] = {0, 0};
    int gfx_n = 0, mfma_n = 0, hbm_n = 0, flops_n = 0;
    double alloc_s = 0, busy_s = 0;  // GPU-seconds this tick
    bool share_known = false;
  };
  std::map<std::pair<std::string, std::string>, PodAgg> pods;

  const bool legacy_only = cfg_.series_profile == "legacy";
  for (size_t di = 0; di < per_dev.size(); ++di) {
    const DeviceInfo& d = devices_[di];
    DevState& st = dstate_[di];
    double cu_sum = 0;
    bool cu_any = false;
    for (auto& p : per_dev[di])
      if (!std::isnan(p.cu_occupancy)) {
        cu_sum += p.cu_occupancy;
        cu_any = true;
      }
    // The GPU's gfx activity split over its processes.  KFD compute contexts report no
    // per-process engine time (fdinfo drm-engine-* stays empty, profiles/r01/kfd_read_costs.txt),
    // so the split uses each process's share of the occupied CUs; a sole process gets all
    // of it, and with no waves resident at the CU sample the split is even.
    const double act = st.cur.ok ? st.cur.gfx_activity : std::nan("");
    const size_t nproc = per_dev[di].size();
    // a process's fraction of the GPU: its share of the occupied CUs (see above)
    auto frac = [&](const ProcSample& p) -> double {
      if (nproc == 0) return std::nan("");
      if (nproc == 1) return 1.0;
      if (cu_any && cu_sum > 0) return std::isnan(p.cu_occupancy) ? std::nan("") : p.cu_occupancy / cu_sum;
      return 1.0 / double(nproc);
    };
    auto gfx_share = [&](const ProcSample& p) -> double { return std::isnan(act) ? act : act * frac(p); };
    // energy this GPU used since the last tick, from its hardware accumulator (exact)
    double energy_j = std::nan("");
    if (st.cur.ok && st.have_prev && st.cur.energy_valid && st.prev.energy_valid) {
      double dacc;
      if (acc_delta(st.cur.energy_acc, st.prev.energy_acc, &dacc)) energy_j = dacc * st.cur.energy_unit_j;
    }
    // this tick's length and the GPU's busy fraction over it (mean of the per-XCD busy from
    // the gfx_busy accumulators; the PMFW's gfx activity where those are missing)
    double tick_s = std::nan(""), busy_frac = std::nan("");
    if (st.cur.ok && st.have_prev && st.cur.host_ns > st.prev.host_ns) {
      tick_s = double(st.cur.host_ns - st.prev.host_ns) * 1e-9;
      if (tick_s > 60.0) tick_s = std::nan("");  // a stalled sampler: do not credit the gap
      double sum = 0;
      int n = 0;
      for (int x = 0; x < kMaxXcc; ++x)
        if (!std::isnan(st.xcc_last[x])) {
          sum += st.xcc_last[x];
          ++n;
        }
      busy_frac = n ? sum / n / 100.0 : st.cur.gfx_activity / 100.0;
    }
    // xGMI bytes this GPU moved since the last tick, summed over links (hardware accumulators)
    double xgmi_rd_b = std::nan(""), xgmi_wr_b = std::nan("");
    if (st.cur.ok && st.have_prev && st.cur.xgmi_valid && st.prev.xgmi_valid) {
      double r = 0, w = 0;
      bool ok = true;
      for (int l = 0; l < kMaxXgmiLinks && ok; ++l) {
        double dr, dw;
        ok = acc_delta(st.cur.xgmi_read_kb[l], st.prev.xgmi_read_kb[l], &dr) &&
             acc_delta(st.cur.xgmi_write_kb[l], st.prev.xgmi_write_kb[l], &dw);
        r += ok ? dr : 0;
        w += ok ? dw : 0;
      }
      if (ok) {  // a reset link skips the tick (as the rates do)
        xgmi_rd_b = r * 1024.0;
        xgmi_wr_b = w * 1024.0;
      }
    }
    const bool shared = st.owner.pod.empty();
    for (auto& p : per_dev[di]) {
      const ProcAttr& a = attr_cache_[p.pid];
      const double share = gfx_share(p);
      if (!legacy_only) {
        // handles cached per (GPU, PID) for as long as the label values stay the same
        ProcRefs& pr = proc_refs_[(uint64_t(uint32_t(di)) << 32) | uint32_t(p.pid)];
        if (pr.comm != p.name || pr.ns != a.ns || pr.pod != a.pod || pr.container != a.container) {
          pr = ProcRefs();
          pr.comm = p.name;
          pr.ns = a.ns;
          pr.pod = a.pod;
          pr.container = a.container;
        }
        pr.gen = gen;
        auto L = [&] {
          return std::vector<std::string>{std::to_string(d.index), std::to_string(p.pid), p.name, a.ns, a.pod,
                                          a.container};
        };
        cput(pr.vram, f_proc_vram_, p.vram_bytes, gen, L);
        if (!std::isnan(p.cu_occupancy)) cput(pr.cu, f_proc_cu_, p.cu_occupancy, gen, L);
        if (!std::isnan(p.sdma_us)) cput(pr.sdma, f_proc_sdma_, p.sdma_us * 1e-6, gen, L);
        if (!std::isnan(p.evicted_ms)) cput(pr.evicted, f_proc_evicted_, p.evicted_ms * 1e-3, gen, L);
        if (!std::isnan(share)) cput(pr.gfx, f_proc_gfx_, share, gen, L);
      }
      if (!a.pod.empty()) {
        auto& la = legacy[p.pid];
        la.used += p.vram_bytes;
        la.total += double(d.vram_total);
        auto& pa = pods[{a.ns, a.pod}];
        pa.vram += p.vram_bytes;
        pa.pids.insert(p.pid);
        const double f = frac(p);
        if (shared && !std::isnan(energy_j) && !std::isnan(f)) pa.energy_j += energy_j * f;
        if (shared && !std::isnan(xgmi_rd_b) && !std::isnan(f)) {
          pa.xrd_b += xgmi_rd_b * f;
          pa.xwr_b += xgmi_wr_b * f;
        }
        // a shared GPU's time is split like its busy time, so busy <= allocated for every pod
        // (the rules' busy / allocated ratio stays a ratio)
        if (shared && !std::isnan(tick_s) && !std::isnan(f)) {
          pa.alloc_s += tick_s * f;
          if (!std::isnan(busy_frac)) pa.busy_s += busy_frac * tick_s * f;
        }
        if (!std::isnan(share)) {
          pa.gfx_share += share;
          pa.share_known = true;
        }
      }
    }
    if (st.cur.ok && !legacy_only) {
      dput(st, int(di), st.nprocs, f_nprocs_, {}, double(per_dev[di].size()), gen);
      // No processes -> 0 CUs occupied (a known value, not an unknown one).
      if (cu_any || per_dev[di].empty()) dput(st, int(di), st.cu_occ, f_cu_occ_, {}, cu_sum, gen);
    }
    if (!st.owner.pod.empty()) {
      auto& pa = pods[{st.owner.ns, st.owner.pod}];
      pa.gpus += 1;
      if (st.cur.ok) {
        if (st.rates_valid)
          for (int l = 0; l < kMaxXgmiLinks; ++l) {
            pa.xrd += st.xgmi_rd_rate[l];
            pa.xwr += st.xgmi_wr_rate[l];
          }
        if (!std::isnan(st.cur.power_w)) pa.power += st.cur.power_w;
        if (!std::isnan(energy_j)) pa.energy_j += energy_j;  // an owned GPU's energy is all the pod's
        if (!std::isnan(xgmi_rd_b)) {  // ...and so is its xGMI traffic
          pa.xrd_b += xgmi_rd_b;
          pa.xwr_b += xgmi_wr_b;
        }
        if (!std::isnan(tick_s)) {  // ...and its time, busy or not
          pa.alloc_s += tick_s;
          if (!std::isnan(busy_frac)) pa.busy_s += busy_frac * tick_s;
        }
        if (!std::isnan(st.cur.gfx_activity)) {
          pa.gfx += st.cur.gfx_activity;
          pa.gfx_n += 1;
        }
        if (!std::isnan(st.mfma_last)) {
          pa.mfma += st.mfma_last;
          pa.mfma_n += 1;
        }
        if (!std::isnan(st.flops_last[0]) && !std::isnan(st.flops_last[1])) {  // an owned GPU's work is the pod's
          pa.flops[0] += st.flops_last[0];
          pa.flops[1] += st.flops_last[1];
          pa.flops_n += 1;
        }
        if (!std::isnan(st.cur.umc_activity) && st.cur.vram_max_bw_gbs > 0) {
          pa.hbm += st.cur.umc_activity / 100.0 * st.cur.vram_max_bw_gbs * 1e9;  // as amd_gpu_hbm_bandwidth
          pa.hbm_n += 1;
        }
      }
    }
  }
  if (f_legacy_mem_ >= 0) {
    // Legacy families: one series per attributed host PID, summed over GPUs (the
    // reference overwrote per device, last-device-wins, main.go:147-150).
    for (auto& kv : legacy) {
      const ProcAttr& a = attr_cache_[kv.first];
      ProcRefs& pr = legacy_refs_[uint64_t(uint32_t(kv.first))];
      if (pr.pod != a.pod) {
        pr = ProcRefs();
        pr.pod = a.pod;
      }
      pr.gen = gen;
      auto L = [&] { return std::vector<std::string>{std::to_string(kv.first), a.pod}; };
      cput(pr.vram, f_legacy_mem_, kv.second.used, gen, L);
      cput(pr.gfx, f_legacy_perc_, kv.second.total > 0 ? kv.second.used / kv.second.total * 100.0 : 0.0, gen, L);
    }
  }
  // forget the handles of processes gone this tick (their series are GC'd by the table)
  for (auto* m : {&proc_refs_, &legacy_refs_})
    for (auto it = m->begin(); it != m->end();) it = it->second.gen != gen ? m->erase(it) : std::next(it);
  if (cfg_.series_profile == "legacy") return;
  for (auto& kv : pods) {
    PodRefs& r = pod_refs_[kv.first];
    r.gen = gen;
    auto L = [&] { return std::vector<std::string>{kv.first.first, kv.first.second}; };
    const PodAgg& pa = kv.second;
    cput(r.ref[0], f_pod_vram_, pa.vram, gen, L);
    cput(r.ref[1], f_pod_procs_, double(pa.pids.size()), gen, L);
    cput(r.ref[2], f_pod_gpus_, double(pa.gpus), gen, L);
    if (pa.share_known) cput(r.ref[3], f_pod_gfx_share_, pa.gfx_share, gen, L);
    if (pa.gpus > 0) {
      cput(r.ref[4], f_pod_xrd_, pa.xrd, gen, L);
      cput(r.ref[5], f_pod_xwr_, pa.xwr, gen, L);
      cput(r.ref[6], f_pod_power_, pa.power, gen, L);
      if (pa.gfx_n) cput(r.ref[7], f_pod_gfx_, pa.gfx / pa.gfx_n, gen, L);
      if (pa.mfma_n) cput(r.ref[8], f_pod_mfma_, pa.mfma / pa.mfma_n, gen, L);
      if (pa.hbm_n) cput(r.ref[9], f_pod_hbm_, pa.hbm, gen, L);
      if (pa.flops_n) {
        static const char* kTypes[2] = {"bf16", "fp8"};
        for (int k = 0; k < 2; ++k)
          cput(r.ref[10 + k], f_pod_flops_, pa.flops[k], gen,
               [&] { return std::vector<std::string>{kv.first.first, kv.first.second, kTypes[k]}; });
      }
    }
  }
  for (auto it = pod_refs_.begin(); it != pod_refs_.end();)
    it = it->second.gen != gen ? pod_refs_.erase(it) : std::next(it);
  // Energy and xGMI bytes per pod: counters that live as long as the control plane knows
  // the pod, so a pod between GPU processes keeps its totals (and an exporter restart too,
  // through the state file).
  for (auto& kv : pods) {
    if (kv.second.energy_j > 0) pod_energy_j_[kv.first] += kv.second.energy_j;
    if (kv.second.xrd_b > 0 || kv.second.xwr_b > 0) {
      auto& x = pod_xgmi_[kv.first];
      x.first += kv.second.xrd_b;
      x.second += kv.second.xwr_b;
    }
    if (kv.second.alloc_s > 0 || kv.second.busy_s > 0) {
      auto& g = pod_gpu_s_[kv.first];
      g.first += kv.second.alloc_s;
      g.second += kv.second.busy_s;
    }
  }
  {
    std::set<std::pair<std::string, std::string>> known;
    for (auto& kv : pods_by_uid_) known.emplace(kv.second.ns, kv.second.name);
    // A pod's totals go when a complete pod list no longer has it -- or, while refreshes stay
    // partial (a metadata source keeps failing), once no applied list has had it for
    // pod_totals_ttl_s (so the maps and the state file cannot grow with every pod ever run).
    const uint64_t now_ns = mono_ns();
    auto gone = [&](const std::pair<std::string, std::string>& k) {
      if (known.count(k)) return false;
      if (pods_complete_) return true;
      auto it = pod_last_known_ns_.find(k);
      if (it == pod_last_known_ns_.end()) {  // restored from the state file, never listed yet
        pod_last_known_ns_[k] = now_ns;
        return false;
      }
      return now_ns - it->second > uint64_t(cfg_.pod_totals_ttl_s * 1e9);
    };
    for (auto it = pod_energy_j_.begin(); it != pod_energy_j_.end();) {
      if (gone(it->first)) {
        it = pod_energy_j_.erase(it);
        continue;
      }
      table_.put(f_pod_energy_, {it->first.first, it->first.second}, it->second, gen);
      ++it;
    }
    for (auto it = pod_xgmi_.begin(); it != pod_xgmi_.end();) {
      if (gone(it->first)) {
        it = pod_xgmi_.erase(it);
        continue;
      }
      table_.put(f_pod_xrd_total_, {it->first.first, it->first.second}, it->second.first, gen);
      table_.put(f_pod_xwr_total_, {it->first.first, it->first.second}, it->second.second, gen);
      ++it;
    }
    for (auto it = pod_gpu_s_.begin(); it != pod_gpu_s_.end();) {
      if (gone(it->first)) {
        it = pod_gpu_s_.erase(it);
        continue;
      }
      table_.put(f_pod_alloc_s_, {it->first.first, it->first.second}, it->second.first, gen);
      table_.put(f_pod_busy_s_, {it->first.first, it->first.second}, it->second.second, gen);
      ++it;
    }
    // a pod's stamp lives while any of its totals does (KFD event counts included: they expire
    // in emit_kfd_events against the same stamp)
    auto has_kfd = [&](const std::pair<std::string, std::string>& k) {
      auto kt = pod_kfd_events_.lower_bound(std::make_tuple(k.first, k.second, INT_MIN));
      return kt != pod_kfd_events_.end() && std::get<0>(kt->first) == k.first && std::get<1>(kt->first) == k.second;
    };
    for (auto it = pod_last_known_ns_.begin(); it != pod_last_known_ns_.end();)
      it = !known.count(it->first) && !pod_energy_j_.count(it->first) && !pod_xgmi_.count(it->first) &&
                   !pod_gpu_s_.count(it->first) && !has_kfd(it->first)
               ? pod_last_known_ns_.erase(it)
               : std::next(it);
  }
  if (rccl_) {
    std::vector<RcclTotals> tot;
    rccl_->poll(&tot);
    for (auto& t : tot) {
      ProcAttr a;
      auto it = attr_cache_.find(t.pid);
      if (it != attr_cache_.end()) a = it->second;
      else if (cfg_.pod_attribution) {
        const CgroupInfo* ci = resolver_->resolve(t.pid);
        if (ci && ci->kube) {
          auto pit = pods_by_uid_.find(ci->pod_uid);
          if (pit != pods_by_uid_.end()) {
            a.ns = pit->second.ns;
            a.pod = pit->second.name;
          } else {
            unresolved_.insert(ci->pod_uid);
          }
        }
      }
      // handles cached per (PID, op) while the labels stay the same (no label vector per tick)
      RcclRefs& r = rccl_refs_[{t.pid, t.op}];
      if (r.ns != a.ns || r.pod != a.pod || r.rank != t.rank || r.nranks != t.nranks) {
        r = RcclRefs();
        r.ns = a.ns;
        r.pod = a.pod;
        r.rank = t.rank;
        r.nranks = t.nranks;
      }
      r.gen = gen;
      auto L = [&] { return std::vector<std::string>{a.ns, a.pod, std::to_string(t.pid), t.op}; };
      cput(r.calls, f_rccl_calls_, double(t.calls), gen, L);
      cput(r.bytes, f_rccl_bytes_, double(t.bytes), gen, L);
      if (t.nranks > 0 && t.rank >= 0)
        cput(r.comm, f_rccl_comm_, 1, gen, [&] {
          return std::vector<std::string>{a.ns, a.pod, std::to_string(t.pid), std::to_string(t.rank),
                                          std::to_string(t.nranks)};
        });
    }
    for (auto it = rccl_refs_.begin(); it != rccl_refs_.end();)
      it = it->second.gen != gen ? rccl_refs_.erase(it) : std::next(it);
  }
}

void Engine::emit_self(uint64_t gen) {
  auto none = [] { return std::vector<std::string>{}; };
  cput(self_refs_[0], f_self_build_, 1, gen, [&] { return std::vector<std::string>{cfg_.version, backend_->name()}; });
  EngineStats s;
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    s = stats_;
  }
  cput(self_refs_[1], f_self_ticks_, double(s.ticks), gen, none);
  if (startup_ns_) cput(startup_ref_, f_self_startup_, double(startup_ns_) * 1e-9, gen, none);
  {
    timespec rt;
    clock_gettime(CLOCK_REALTIME, &rt);
    cput(self_refs_[2], f_self_last_, double(rt.tv_sec) + double(rt.tv_nsec) * 1e-9, gen, none);
  }
  cput(self_refs_[3], f_self_overruns_, double(s.overruns), gen, none);
  cput(self_refs_[4], f_self_unresolved_, double(unresolved_.size()), gen, none);
  cput(pods_complete_ref_, f_self_pods_complete_, pods_complete_ ? 1 : 0, gen, none);
  if (kfd_) {
    cput(kfd_scan_refs_[0], f_self_kfd_scans_, double(kfd_->lists()), gen,
         [] { return std::vector<std::string>{"list"}; });
    cput(kfd_scan_refs_[1], f_self_kfd_scans_, double(kfd_->scans() - kfd_->lists()), gen,
         [] { return std::vector<std::string>{"tracked"}; });
    cput(kfd_scan_refs_[2], f_self_kfd_tracked_, double(kfd_->tracked()), gen, none);
  }
  cput(self_refs_[5], f_self_render_bytes_, double(s.render_bytes), gen, none);
  cput(self_refs_[6], f_self_series_, double(s.series), gen, none);
  cput(self_refs_[7], f_self_cpu_, double(s.sampler_cpu_ns) * 1e-9, gen, none);
  for (int k = 0; k < kDevParts; ++k)
    cput(dev_part_refs_[k], f_self_dev_part_, dev_part_total_s_[k], gen,
         [&] { return std::vector<std::string>{dev_part_name(k)}; });
  // histograms: accumulated every tick, published every tick at <= 10 Hz (or manual ticks) and at
  // most once a second above that (see engine.h)
  const uint64_t hnow = last_tick_now_;
  const bool publish_hist = cfg_.interval_s <= 0 || cfg_.interval_s >= 0.1 || !self_hist_pub_ns_ ||
                            hnow < self_hist_pub_ns_ || hnow - self_hist_pub_ns_ >= 1000000000ull;
  if (publish_hist) self_hist_pub_ns_ = hnow;
  const std::vector<double>& sb = stage_bounds();
  for (int k = 0; k < kStages; ++k) {
    if (!self_stage_refs_[k].valid()) self_stage_refs_[k] = table_.upsert(f_self_stage_, {stage_name(k)});
    std::vector<uint64_t>& h = stage_hist_[k];
    if (h.size() != sb.size() + 1) h.assign(sb.size() + 1, 0);
    if (s.ticks) {
      const double v = double(last_stage_ns_[k]) * 1e-9;
      h[size_t(std::lower_bound(sb.begin(), sb.end(), v) - sb.begin())] += 1;
      stage_hist_sum_[k] += v;
      stage_hist_n_[k] += 1;
    }
    if (!publish_hist || !table_.set_histogram(self_stage_refs_[k], sb, h, stage_hist_sum_[k], stage_hist_n_[k], gen))
      table_.touch(self_stage_refs_[k], gen);
  }
  if (http_) {
    const HttpStats& hs = http_->stats();
    if (publish_hist || !table_.touch(self_refs_[8], gen)) {
      std::vector<uint64_t> counts(HttpStats::kBuckets + 1);
      for (int b = 0; b <= HttpStats::kBuckets; ++b) counts[size_t(b)] = hs.lat_buckets[b].load(std::memory_order_relaxed);
      uint64_t cnt = hs.lat_count.load(std::memory_order_relaxed);
      double sum = double(hs.lat_sum_ns.load(std::memory_order_relaxed)) * 1e-9;
      if (!table_.set_histogram(self_refs_[8], scrape_latency_bounds(), counts, sum, cnt, gen)) {
        self_refs_[8] = table_.upsert(f_self_scrape_, {});
        table_.set_histogram(self_refs_[8], scrape_latency_bounds(), counts, sum, cnt, gen);
      }
    }
    cput(self_refs_[9], f_self_scrapes_, double(hs.metrics_requests.load(std::memory_order_relaxed)), gen, none);
    cput(self_refs_[10], f_self_http_bytes_, double(hs.bytes_sent.load(std::memory_order_relaxed)), gen, none);
    // every mode: the mode is switched at run time (set_prewake_mode)
    cput(self_refs_[11], f_self_prewake_, double(hs.prewake_timer_wakeups.load(std::memory_order_relaxed)), gen,
         none);
    cput(prewake_hits_ref_, f_self_prewake_hits_, double(hs.prewake_hits.load(std::memory_order_relaxed)), gen,
         none);
    cput(prewake_hits_narrow_ref_, f_self_prewake_hits_narrow_,
         double(hs.prewake_hits_narrow.load(std::memory_order_relaxed)), gen, none);
    cput(prewake_spin_refs_[0], f_self_prewake_spins_, double(hs.prewake_spin_hits.load(std::memory_order_relaxed)),
         gen, [] { return std::vector<std::string>{"hit"}; });
    cput(prewake_spin_refs_[1], f_self_prewake_spins_,
         double(hs.prewake_spin_timeouts.load(std::memory_order_relaxed)), gen,
         [] { return std::vector<std::string>{"timeout"}; });
    cput(prewake_spin_refs_[2], f_self_prewake_spin_s_,
         double(hs.prewake_spin_ns.load(std::memory_order_relaxed)) * 1e-9, gen, none);
    cput(rx_moves_ref_, f_self_rx_moves_, double(hs.rx_cpu_moves.load(std::memory_order_relaxed)), gen, none);
    if (cfg_.http.enable_gzip) {
      cput(self_refs_[16], f_self_gzip_, double(gzip_eager_), gen,
           [] { return std::vector<std::string>{"sampler"}; });
      cput(self_refs_[17], f_self_gzip_, double(hs.gzip_on_demand.load(std::memory_order_relaxed)), gen,
           [] { return std::vector<std::string>{"request"}; });
    }
  }
  if (!mock_)
    for (size_t i = 0; i < devices_.size(); ++i) {
      DevState& st = dstate_[i];
      const std::string g = std::to_string(devices_[i].index);
      cput(st.self_reads[0], f_self_metrics_reads_, double(metrics_fresh_[i]), gen,
           [&] { return std::vector<std::string>{g, "fresh"}; });
      cput(st.self_reads[1], f_self_metrics_reads_, double(metrics_coalesced_[i]), gen,
           [&] { return std::vector<std::string>{g, "coalesced"}; });
      cput(st.self_reads[2], f_self_metrics_period_, backend_->metrics_period_s(devices_[i]), gen,
           [&] { return std::vector<std::string>{g}; });
      cput(st.fetch_cpu, f_self_fetch_cpu_, st.fetch_cpu_s, gen, [&] { return std::vector<std::string>{g}; });
      const double cap = cfg_.metrics_min_interval_s < 0 ? double(st.fetch_cap_ns) * 1e-9
                                                          : std::max(0.0, cfg_.metrics_min_interval_s);
      cput(st.fetch_cap, f_self_fetch_cap_, cap, gen, [&] { return std::vector<std::string>{g}; });
      const double age = st.metrics_fresh_ns && last_tick_now_ >= st.metrics_fresh_ns
                             ? double(last_tick_now_ - st.metrics_fresh_ns) * 1e-9 : kNaN;
      cput(st.metrics_age, f_self_metrics_age_, age, gen, [&] { return std::vector<std::string>{g}; });
    }
  cput(self_refs_[12], f_self_source_up_, 1, gen,
       [&] { return std::vector<std::string>{"backend:" + std::string(backend_->name())}; });
  cput(self_refs_[13], f_self_source_up_, (sentinel_ || (cfg_.enable_sentinel && mock_)) ? 1 : 0, gen,
       [] { return std::vector<std::string>{"sentinel"}; });
  cput(self_refs_[14], f_self_source_up_, (counters_ || (cfg_.enable_counters && mock_)) ? 1 : 0, gen,
       [] { return std::vector<std::string>{"counters"}; });
  cput(self_refs_[15], f_self_source_up_, rccl_ ? 1 : 0, gen, [] { return std::vector<std::string>{"rccl"}; });
  if (counters_ && cfg_.counters_mode == "continuous")
    cput(self_refs_[19], f_self_ctr_late_, double(counters_late_), gen, none);
  if (cfg_.enable_kfd_events && cfg_.series_profile == "full")
    cput(self_refs_[18], f_self_source_up_, kfd_events_ ? 1 : 0, gen,
         [] { return std::vector<std::string>{"kfd_events"}; });
  if (cfg_.series_profile == "full")
    cput(self_refs_[20], f_driver_, 1, gen, [&] { return std::vector<std::string>{driver_version_, kernel_release_}; });
  if (compiled_) {
    cput(expo_refs_[0], f_self_expo_, double(expo_relayouts_), gen, [] { return std::vector<std::string>{"relayout"}; });
    cput(expo_refs_[1], f_self_expo_, double(table_.provisional_parses()), gen,
         [] { return std::vector<std::string>{"provisional_parse"}; });
    cput(expo_refs_[2], f_self_expo_, double(table_.code_builds()), gen,
         [] { return std::vector<std::string>{"code_build"}; });
  }
  if (rccl_) {
    int a = 0, u = 0, x = 0;
    rccl_->file_states(&a, &u, &x);
    static const char* const kStates[4] = {"active", "unverified", "exited", "ignored"};
    const double v[4] = {double(a), double(u), double(x), double(rccl_->ignored())};
    for (int k = 0; k < 4; ++k)
      cput(rccl_self_refs_[k], f_self_rccl_files_, v[k], gen, [&] { return std::vector<std::string>{kStates[k]}; });
    cput(rccl_self_refs_[4], f_self_rccl_scans_, double(rccl_->scans()), gen, none);
  }
}

// metrics_min_interval "auto": all GPUs' SMU fetches together may use metrics_cpu_budget of
// one core.  With c_i the measured thread CPU of GPU i's fresh read, every GPU gets the cap
// T = sum(c_i) / budget (one fetch per GPU per T): 1 GPU at 0.25 ms and 1.5 % -> 17 ms, under
// a 10 Hz tick, so every tick is fresh; 8 GPUs -> 133 ms, a fresh table every other tick.
// A cap at or below the tick period is no cap (0); above it, the cap is rounded UP to whole
// ticks (k = ceil(T / period): a fetch every k-th tick keeps the budget) and half a period
// comes off, so tick jitter never skips one more fetch than that.
void Engine::update_fetch_policy() {
  double sum_ns = 0;
  for (const auto& st : dstate_) sum_ns += st.fetch_cost_ns;
  if (sum_ns <= 0 || cfg_.metrics_cpu_budget <= 0) return;  // nothing measured yet: no cap
  const double period = cfg_.interval_s > 0 ? cfg_.interval_s * 1e9 : 0;
  double cap = std::min(sum_ns / cfg_.metrics_cpu_budget, cfg_.metrics_max_interval_s * 1e9);
  if (period > 0) cap = cap <= period ? 0 : (std::ceil(cap / period) - 0.5) * period;
  for (size_t i = 0; i < dstate_.size(); ++i) {
    DevState& st = dstate_[i];
    const double prev = double(st.fetch_cap_ns);
    // re-set only on a 5 % change (the EWMA moves a little every fresh read)
    if (std::fabs(cap - prev) <= 0.05 * std::max(cap, prev) && !(cap == 0 && prev != 0)) continue;
    st.fetch_cap_ns = uint64_t(cap);
    backend_->update_metrics_min_interval(devices_[i], st.fetch_cap_ns);
  }
}

void Engine::tick_locked(uint64_t now) {
  uint64_t cpu0 = thread_cpu_ns();
  uint64_t gen = ++gen_;
  double dt_s = last_tick_now_ && now > last_tick_now_ ? double(now - last_tick_now_) * 1e-9 : 0.0;
  last_tick_now_ = now;
  uint64_t ts[kStages + 1], cs[kStages + 1];  // stage boundaries: wall, sampler-thread CPU
  // The per-stage CPU split is sampled on one tick in kStageCpuEvery (a thread CPU clock read is
  // a system call: 7 of them per tick were ~1 % of an 8-GPU node's tick at 10 Hz); the whole
  // tick's CPU is read every tick.  Which ticks: a hash of the generation, so a periodic stage
  // (a gpu_metrics fetch every 2nd or 4th tick) is not always in or always out of the sample.
  const bool split_cpu = ((gen * 0x9E3779B97F4A7C15ull) >> 61) % kStageCpuEvery == 0;
  auto cpu_mark = [split_cpu]() { return split_cpu ? thread_cpu_ns() : 0; };
  ts[0] = mono_ns();
  cs[0] = cpu0;
  if (!startup_ns_ && start_mono_ns_ && ts[0] > start_mono_ns_) startup_ns_ = ts[0] - start_mono_ns_;
  // continuous counters: this tick's read goes out now (or right after the device reads)
  // and is collected before the series stage, so the exported window is one tick interval
  resolver_->begin_tick(now);
  uint64_t part[kDevParts] = {};
  // "end" (auto below 50 ms ticks): the read for this tick went out at the end of the previous
  // one, so it has completed by the counters stage -- at 100 Hz most ticks have no SMU fetch
  // to hide a ~200 us PM4 read behind, and waiting for it cost 2-3 sleep/wake-ups per tick;
  // the exported window then ends one tick earlier (10 ms at 100 Hz)
  const std::string& kick_mode = counters_kick_mode_;
  const bool kick_late = kick_mode == "after_devices";
  const bool kick_end = kick_mode == "end";
  if (counters_ && !kick_late && !kick_end) {
    counters_->kick();
    part[0] = mono_ns() - ts[0];
  }
  const uint64_t c0 = mono_ns();

  // Control-plane updates (pushed from Python at low rate).
  {
    std::lock_guard<std::mutex> lk(ctl_mu_);
    if (clear_overrides_) {
      resolver_->clear_overrides();
      clear_overrides_ = false;
      ++ctl_epoch_;
    }
    if (!pending_overrides_.empty()) ++ctl_epoch_;
    for (auto& o : pending_overrides_) resolver_->set_override(o.first, o.second);
    pending_overrides_.clear();
    if (ctl_dirty_) {
      ++ctl_epoch_;
      pods_by_uid_.clear();
      container_names_.clear();
      for (auto& p : pending_pods_) {
        for (auto& c : p.containers) container_names_[lower(c.first)] = c.second;
        pods_by_uid_[lower(p.uid)] = p;
      }
      owners_.clear();
      for (auto& o : pending_owners_) owners_[lower(o.first)] = o.second;
      ctl_dirty_ = false;
      // per-pod totals (energy, xGMI bytes, KFD events; possibly restored from the state
      // file) are garbage-collected against a pod list only if that list is complete: a
      // refresh in which a source failed must not wipe them
      pods_complete_ = pending_complete_;
      const uint64_t applied = mono_ns();
      for (auto& kv : pods_by_uid_) pod_last_known_ns_[{kv.second.ns, kv.second.name}] = applied;
    }
  }
  part[1] = mono_ns() - c0;

  // 0: device telemetry (per-GPU reads fan out over the pool; each touches only its own
  // DevState and its own backend device slot)
  uint64_t errs = 0;
  // (the VRAM / RAS / GTT read times are sampled on the same ticks as the stage CPU split: two
  // clock reads each per GPU per tick otherwise, for a diagnostic)
  auto sample_one = [this, now, split_cpu](int i) {
    DevState& st = dstate_[size_t(i)];
    if (st.cur.ok) {
      st.prev = st.cur;
      st.have_prev = true;
    }
    st.cur = DeviceSample();
    st.cur.host_ns = now;
    st.cur.time_parts = split_cpu;
    backend_->sample(devices_[size_t(i)], &st.cur);
    (st.cur.metrics_coalesced ? metrics_coalesced_ : metrics_fresh_)[size_t(i)] += 1;
    if (st.cur.ok && !st.cur.metrics_coalesced) st.metrics_fresh_ns = now;
    st.ras_ns = st.gtt_ns = 0;
    if (!ras_.empty()) {
      const uint64_t r0 = split_cpu ? mono_ns() : 0;
      if (now >= ras_next_ns_[size_t(i)]) {
        ras_[size_t(i)].read(&ras_cache_[size_t(i)]);
        ras_next_ns_[size_t(i)] = now + uint64_t(cfg_.ras_interval_s * 1e9);
      }
      const RasTotals& r = ras_cache_[size_t(i)];
      st.cur.ecc_ce = r.ecc_ce;
      st.cur.ecc_ue = r.ecc_ue;
      st.cur.ecc_de = r.ecc_de;
      st.cur.aer_cor = r.aer_cor;
      st.cur.aer_nonfatal = r.aer_nonfatal;
      st.cur.aer_fatal = r.aer_fatal;
      st.cur.pages_retired = r.pages_retired;
      st.cur.pages_pending = r.pages_pending;
      st.cur.pages_unreservable = r.pages_unreservable;
      if (split_cpu) st.ras_ns = mono_ns() - r0;
    }
    if (!gtt_used_f_.empty()) {
      const uint64_t g0 = split_cpu ? mono_ns() : 0;
      uint64_t v = 0;
      if (gtt_used_f_[size_t(i)].read_u64(&v)) st.cur.gtt_used = double(v);
      st.cur.gtt_total = gtt_total_[size_t(i)];
      if (split_cpu) st.gtt_ns = mono_ns() - g0;
    }
  };
  if (pool_) {
    pool_->run(int(devices_.size()), sample_one);
  } else {
    for (size_t i = 0; i < devices_.size(); ++i) sample_one(int(i));
  }
  for (auto& st : dstate_) {
    if (!st.cur.ok) {
      st.errors += 1;
      errs += 1;
    }
    part[2] += st.cur.metrics_wall_ns;
    part[3] += kStageCpuEvery * st.cur.vram_wall_ns;  // (0 off the sampled ticks)
    part[4] += kStageCpuEvery * st.ras_ns;
    part[5] += kStageCpuEvery * st.gtt_ns;
    if (!st.cur.metrics_coalesced && st.cur.metrics_cpu_ns) {
      st.fetch_cpu_s += double(st.cur.metrics_cpu_ns) * 1e-9;
      // EWMA over fresh reads (a few outliers, e.g. a preempted read, barely move it)
      const double c = double(st.cur.metrics_cpu_ns);
      st.fetch_cost_ns = st.fetch_cost_ns > 0 ? 0.9 * st.fetch_cost_ns + 0.1 * c : c;
    }
  }
  if (cfg_.metrics_min_interval_s < 0) update_fetch_policy();
  if (counters_ && kick_late) {
    const uint64_t k0 = mono_ns();
    counters_->kick();
    part[0] = mono_ns() - k0;
  }
  ts[1] = mono_ns();
  cs[1] = cpu_mark();
  for (int k = 0; k < kDevParts; ++k) dev_part_total_s_[k] += double(part[k]) * 1e-9;

  // 1: processes
  // (reused across ticks: the lists keep their capacity, no allocation per tick)
  std::vector<std::vector<ProcSample>>& per_dev = per_dev_;
  per_dev.resize(devices_.size());
  for (auto& l : per_dev) l.clear();
  if (cfg_.process_source != "none") {
    bool from_backend = cfg_.process_source != "kfd";
    if (from_backend)
      for (size_t i = 0; i < devices_.size(); ++i)
        if (!backend_->processes(devices_[i], &per_dev[i])) {
          from_backend = false;
          break;
        }
    if (!from_backend) {
      kfd_->scan(devices_, &per_dev, now);
    } else if (cfg_.exclude_self) {
      for (auto& l : per_dev)
        l.erase(std::remove_if(l.begin(), l.end(), [this](const ProcSample& p) { return p.pid == self_pid_; }),
                l.end());
    }
  }
  ts[2] = mono_ns();
  cs[2] = cpu_mark();

  // 2: device ownership (device plugin map first, then single-pod inference).
  for (size_t i = 0; i < devices_.size(); ++i) {
    DevState& st = dstate_[i];
    DeviceOwner own;
    auto it = owners_.end();
    for (const std::string& key : owner_keys_[i]) {
      it = owners_.find(key);
      if (it != owners_.end()) break;
    }
    if (it != owners_.end()) {
      own = it->second;
    } else if (cfg_.pod_attribution && cfg_.infer_device_owner) {
      // the same processes (KFD identities, order-free) under the same control plane infer the
      // same owner: reuse it instead of resolving and building sets of label strings every tick
      uint64_t sig = 0x9E3779B97F4A7C15ull ^ ctl_epoch_;
      bool cacheable = true;
      for (auto& p : per_dev[i]) {
        cacheable = cacheable && p.kfd_id != 0;
        sig += (p.kfd_id ^ (uint64_t(uint32_t(p.pid)) << 32)) * 0xBF58476D1CE4E5B9ull;
      }
      sig = cacheable ? (sig | 1) : 0;
      if (sig && sig == st.owner_sig) {
        st.owner = st.owner_inferred;
        continue;
      }
      std::set<std::tuple<std::string, std::string, std::string>> seen;
      for (auto& p : per_dev[i]) {
        const CgroupInfo* ci = resolver_->resolve(p.pid, p.kfd_id);
        if (!ci) sig = 0;  // unreadable /proc/<pid>: ask again next tick
        if (!ci || !ci->kube) continue;
        auto pit = pods_by_uid_.find(ci->pod_uid);
        if (pit == pods_by_uid_.end()) {
          seen.emplace("", "", "");  // an unnamed pod: ownership stays unknown
          continue;
        }
        const std::string& ns = pit->second.ns;
        const std::string& name = pit->second.name;
        auto cn = container_names_.find(ci->container_id);
        seen.emplace(ns, name, cn != container_names_.end() ? cn->second : "");
      }
      std::set<std::pair<std::string, std::string>> podset;
      for (auto& t : seen) podset.emplace(std::get<0>(t), std::get<1>(t));
      if (podset.size() == 1 && !podset.begin()->second.empty()) {
        own.ns = podset.begin()->first;
        own.pod = podset.begin()->second;
        if (seen.size() == 1) own.container = std::get<2>(*seen.begin());
      }
      st.owner_sig = sig;
      st.owner_inferred = own;
    }
    st.owner = own;
  }
  ts[3] = mono_ns();
  cs[3] = cpu_mark();

  // 3: sentinel (drain previous run, launch next; never blocks on the GPU)
  if (sentinel_) sentinel_->tick(now);
  if (kfd_events_) count_kfd_events();
  ts[4] = mono_ns();
  cs[4] = cpu_mark();
  // 4: counters: wait (bounded) for this tick's read round; sampled in collect_device
  if (counters_ && !counters_->sync(cfg_.counters_sync_us)) counters_late_ += 1;
  ts[5] = mono_ns();
  cs[5] = cpu_mark();

  // 5: series
  for (size_t i = 0; i < devices_.size(); ++i) {
    if (cfg_.series_profile != "legacy") collect_device(int(i), gen, dt_s);
  }
  emit_processes(gen, per_dev);
  if (kfd_events_) emit_kfd_events(gen);
  emit_self(gen);
  ts[6] = mono_ns();
  cs[6] = cpu_mark();

  // 6: render into a free snapshot slot
  int slot = store_.begin_write();
  uint64_t rbytes = 0, nseries = 0;
  if (slot >= 0) {
    Snapshot* snap = store_.slot(slot);
    // gzip copy only when a gzip scrape is expected before the tick after next (or its
    // schedule is unknown): a 15 s Prometheus scrape costs one compression, not 150
    const uint64_t period_ns = cfg_.interval_s > 0 ? uint64_t(cfg_.interval_s * 1e9) : 1000000000ull;
    const bool want_gz = http_ && http_->gzip_due(mono_ns(), 2 * period_ns + 5000000ull);
    if (want_gz) ++gzip_eager_;
    snap->gz.clear();
    // (the slot's previous generation: only the fields changed since are copied into it)
    if (compiled_) table_.render_compiled(&snap->body, want_gz ? &snap->gz : nullptr, gen, cfg_.gc_after, snap->gen);
    else table_.render(&snap->body, gen, cfg_.gc_after);
    snap->gen = gen;
    snap->render_ns = now;
    rbytes = snap->body.size();
    nseries = table_.live_series(gen);
    snap->series = nseries;
    ts[7] = mono_ns();
    cs[7] = cpu_mark();
    // 7: gzip (classic; compiled emitted it with the body) + publish
    snap->pb.clear();
    snap->pb_gz.clear();
    const uint64_t tnow = mono_ns();
    if (want_gz && !compiled_) gzip_compress(snap->body, &snap->gz, cfg_.gzip_level);
    if (http_ && http_->proto_wanted_ns() && tnow - http_->proto_wanted_ns() < 60000000000ull) {
      table_.render_proto(&snap->pb, gen);
      if (want_gz) gzip_compress(snap->pb, &snap->pb_gz, cfg_.gzip_level);
    }
    snap->published_mono_ns = mono_ns();
    store_.publish(slot);
    if (!cfg_.state_file.empty() && tnow - state_saved_ns_ >= uint64_t(cfg_.state_interval_s * 1e9)) save_state();
    if (http_) http_->set_ready(true);
  } else {
    ts[7] = mono_ns();
    cs[7] = cpu_mark();
  }
  if (counters_ && kick_end) counters_->kick();  // next tick's read, completing while we sleep
  uint64_t tend = mono_ns();
  cs[kStages] = thread_cpu_ns();
  uint64_t stage_dur[kStages] = {ts[1] - ts[0], ts[2] - ts[1], ts[3] - ts[2], ts[4] - ts[3],
                                 ts[5] - ts[4], ts[6] - ts[5], ts[7] - ts[6], tend - ts[7]};
  for (int k = 0; k < kStages; ++k) {
    last_stage_ns_[k] = stage_dur[k];
    uint64_t start = k == 0 ? ts[0] : (k < kStages - 1 ? ts[k] : ts[7]);
    trace_event(stage_name(k), start, stage_dur[k]);
    if (k == 0 && trace_) {  // the devices stage's parts, inside its span
      trace_event("devices/control", c0, part[1]);
      for (size_t i = 0; i < dstate_.size(); ++i)  // per GPU (they overlap on the read pool)
        if (dstate_[i].cur.metrics_wall_ns) trace_event("devices/gpu_metrics", c0 + part[1], dstate_[i].cur.metrics_wall_ns);
    }
  }
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.ticks += 1;
    if (slot < 0) stats_.publish_skipped += 1;
    stats_.last_tick_ns = tend - ts[0];
    stats_.max_tick_ns = std::max(stats_.max_tick_ns, stats_.last_tick_ns);
    if (slot >= 0) {
      stats_.render_bytes = rbytes;
      stats_.series = nseries;
    }
    stats_.device_errors += errs;
    for (int k = 0; k < kStages; ++k) {
      stats_.stage_ns[k] = double(stage_dur[k]);
      if (split_cpu)  // the sampler thread's own CPU per stage, scaled up from the sampled ticks
        stats_.stage_cpu_ns[k] += kStageCpuEvery * (cs[k + 1] - cs[k]);
    }
    // every thread that worked for this tick: the sampler, the per-GPU read pool, and the
    // counter plugin's thread (its PM4 read rounds since the last tick)
    // The sampler thread charges its whole clock since the last tick (timerfd wake-ups
    // included); a manual tick_now() from another thread charges the tick itself.
    const uint64_t own = cs[kStages];
    uint64_t cpu = own - cpu0;
    if (tl_sampler_thread) {
      if (sampler_cpu_seen_ && own >= sampler_cpu_seen_) cpu = own - sampler_cpu_seen_;
      sampler_cpu_seen_ = own;
    }
    if (pool_) {
      const uint64_t p = pool_->cpu_ns_total();
      if (p >= pool_cpu_seen_) cpu += p - pool_cpu_seen_;
      pool_cpu_seen_ = p;
    }
    if (counters_) {
      const uint64_t c = counters_->cpu_ns();
      if (c >= counters_cpu_seen_) cpu += c - counters_cpu_seen_;
      counters_cpu_seen_ = c;
    }
    stats_.sampler_cpu_ns += cpu;
    stats_.gzip_eager = gzip_eager_;
    stats_.relayouts += table_.last_relayouts();
    stats_.families_skipped += table_.last_skipped();
    stats_.families_rendered += table_.last_walked();
    expo_relayouts_ += table_.last_relayouts();
    stats_.code_builds = table_.code_builds();
  }
}

std::string Engine::snapshot_text() {
  auto pin = store_.acquire();
  return pin ? pin->body : std::string();
}

EngineStats Engine::stats() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  return stats_;
}

std::string Engine::source_status() {
  std::string s = std::string("backend=") + (backend_ ? backend_->name() : "none") + " sentinel=" + sentinel_status_ +
                  " counters=" + counters_status_ + " rccl=" + (rccl_ ? cfg_.rccl_dir : "disabled") +
                  " kfd_events=" + kfd_events_status_ + " state=" + state_status();
  if (backend_)
    for (const auto& d : devices_) s += " gpu" + std::to_string(d.index) + "=[" + backend_->describe(d) + "]";
  return s;
}

}  // namespace gpuexp
