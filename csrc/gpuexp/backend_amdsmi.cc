// amdsmi backend (BASELINE config 2: "1xMI355X amdsmi util/HBM/power/temp").
//
// NVML call sites in the reference (/root/reference/main.go:45-137) map
// to: amdsmi_init / amdsmi_get_socket_handles / amdsmi_get_processor_handles (enumerated
// ONCE, not per cycle like DeviceGetCount at main.go:117), amdsmi_get_gpu_device_bdf /
// _uuid / _enumeration_info / _kfd_info for stable identity, amdsmi_get_link_metrics for
// the xGMI peer map (once; 643 us/call measured), and per tick the gpu_metrics blob.
//
// Per-tick cost: amdsmi_get_gpu_metrics_info measured 152 us/call on MI355X; the same
// blob via a cached-fd pread + GpuMetricsV1_8 decode is the fast path.  At init both are
// read back-to-back and compared field by field (static fields exactly, accumulators
// monotone and within slack); a mismatch keeps amdsmi as the per-tick source.
#include <amd_smi/amdsmi.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "gpuexp/backends.h"

namespace gpuexp {

namespace {

std::string smi_err(amdsmi_status_t st) {
  const char* s = nullptr;
  amdsmi_status_code_to_string(st, &s);
  return s ? std::string(s) : ("amdsmi status " + std::to_string(int(st)));
}

inline double u16v(uint16_t v) { return v == 0xFFFF ? kNaN : double(v); }

// amdsmi's decoded struct -> DeviceSample (the slow-path per-tick source).
void from_amdsmi_metrics(const amdsmi_gpu_metrics_t& m, DeviceSample* out, int xcp, int nxcc) {
  out->temp_edge = u16v(m.temperature_edge);
  out->temp_hotspot = u16v(m.temperature_hotspot);
  out->temp_mem = u16v(m.temperature_mem);
  out->temp_vrgfx = u16v(m.temperature_vrgfx);
  out->temp_vrsoc = u16v(m.temperature_vrsoc);
  out->temp_vrmem = u16v(m.temperature_vrmem);
  for (int i = 0; i < kMaxHbm; ++i) out->temp_hbm[i] = u16v(m.temperature_hbm[i]);
  out->gfx_activity = u16v(m.average_gfx_activity);
  out->umc_activity = u16v(m.average_umc_activity);
  out->mm_activity = u16v(m.average_mm_activity);
  out->power_w = m.current_socket_power != 0xFFFF ? double(m.current_socket_power)
                                                  : u16v(m.average_socket_power);
  out->energy_valid = m.energy_accumulator != ~0ull;
  out->energy_acc = m.energy_accumulator;
  out->energy_unit_j = 15.259e-6;
  out->fw_ts_10ns = m.firmware_timestamp == ~0ull ? 0 : m.firmware_timestamp;
  // this partition's XCDs only (same selection as decode_gpu_metrics_v1_8)
  if (xcp < 0 || xcp >= 8) xcp = 0;
  const int nx = nxcc > 0 && nxcc <= kMaxXcc ? nxcc : kMaxXcc;
  const int first = xcp * nx < kMaxXcc ? xcp * nx : 0;
  double sum = 0;
  int n = 0;
  for (int i = 0; i < nx && first + i < AMDSMI_MAX_NUM_GFX_CLKS; ++i) {
    const uint16_t c = m.current_gfxclks[first + i];
    if (c != 0xFFFF && c != 0) {
      sum += c;
      out->clk_gfx_xcc[i] = c;
      ++n;
    }
  }
  out->clk_gfx = n ? sum / n : u16v(m.current_gfxclk);
  out->num_partition = m.num_partition == 0xFFFF ? 0 : m.num_partition;
  out->clk_soc = m.current_socclks[0] != 0xFFFF ? double(m.current_socclks[0]) : u16v(m.current_socclk);
  out->clk_mem = u16v(m.current_uclk);
  int nl = 0;
  for (int l = 0; l < kMaxXgmiLinks; ++l) {
    out->xgmi_read_kb[l] = m.xgmi_read_data_acc[l] == ~0ull ? 0 : m.xgmi_read_data_acc[l];
    out->xgmi_write_kb[l] = m.xgmi_write_data_acc[l] == ~0ull ? 0 : m.xgmi_write_data_acc[l];
    out->xgmi_link_up[l] = m.xgmi_link_status[l] == 0xFFFF ? kNaN : double(m.xgmi_link_status[l] ? 1 : 0);
    if (m.xgmi_link_status[l] != 0xFFFF) nl = l + 1;
  }
  out->num_xgmi_links = nl;
  out->xgmi_valid = true;
  out->pcie_width = u16v(m.pcie_link_width);
  out->pcie_speed_gts = m.pcie_link_speed == 0xFFFF ? kNaN : m.pcie_link_speed / 10.0;
  out->pcie_bw_acc = m.pcie_bandwidth_acc;
  out->pcie_bw_inst = m.pcie_bandwidth_inst == ~0ull ? kNaN : double(m.pcie_bandwidth_inst);
  out->pcie_replay = m.pcie_replay_count_acc == ~0ull ? kNaN : double(m.pcie_replay_count_acc);
  out->pcie_nak_sent = m.pcie_nak_sent_count_acc == 0xFFFFFFFFu ? kNaN : double(m.pcie_nak_sent_count_acc);
  out->pcie_nak_rcvd = m.pcie_nak_rcvd_count_acc == 0xFFFFFFFFu ? kNaN : double(m.pcie_nak_rcvd_count_acc);
  out->pcie_l0_recov = m.pcie_l0_to_recov_count_acc == ~0ull ? kNaN : double(m.pcie_l0_to_recov_count_acc);
  out->xgmi_width = u16v(m.xgmi_link_width);
  out->xgmi_speed = u16v(m.xgmi_link_speed);
  out->residency_valid = m.accumulation_counter != ~0ull;
  out->accumulation_counter = m.accumulation_counter;
  out->res_ppt = m.ppt_residency_acc;
  out->res_socket_thm = m.socket_thm_residency_acc;
  out->res_vr_thm = m.vr_thm_residency_acc;
  out->res_hbm_thm = m.hbm_thm_residency_acc;
  out->res_prochot = m.prochot_residency_acc;
  out->vram_max_bw_gbs = m.vram_max_bandwidth == ~0ull ? kNaN : double(m.vram_max_bandwidth);
  for (int c = 0; c < kMaxXcc; ++c) out->gfx_busy_acc[c] = m.xcp_stats[xcp].gfx_busy_acc[c];
}

bool same_or_both_nan(double a, double b, double tol) {
  if (std::isnan(a) && std::isnan(b)) return true;
  return std::fabs(a - b) <= tol;
}

}  // namespace

class AmdsmiBackend : public Backend {
  struct Dev {
    amdsmi_processor_handle h = nullptr;
    GpuMetricsReader gm;
    bool fast_ok = false;
    std::string validate_msg;
    int validated_fields = 0;
    uint64_t raw_failures = 0;  // __atomic_* access: sampler writes, describe() reads
    CachedFile vram_used_file;
    uint32_t socket = 0;  // index of its amdsmi socket handle (the partitions of one GPU share it)
    double power_cap_w = kNaN;
    int xcp = 0, nxcc = 0;  // compute partition of this logical GPU (see DeviceInfo)
    std::vector<amdsmi_proc_info_t> procbuf = std::vector<amdsmi_proc_info_t>(64);
  };

 public:
  AmdsmiBackend(std::string root, bool amdsmi_procs, bool force_amdsmi_metrics)
      : root_(std::move(root)), amdsmi_procs_(amdsmi_procs), force_smi_(force_amdsmi_metrics) {
    if (!root_.empty() && root_.back() == '/') root_.pop_back();
  }
  ~AmdsmiBackend() override { shutdown(); }
  const char* name() const override { return "amdsmi"; }

  bool init(std::vector<DeviceInfo>* devices, std::string* err) override {
    // amdsmi caches gpu_metrics tables for AMDSMI_GPU_METRICS_CACHE_MS: two calls around a
    // raw read can then return one older table (seen on MI355X: equal system_clock_counter
    // around a newer raw value).  Its reads here are validation and fallback, both of which
    // want the current table, so no cache unless the user set one.
    ::setenv("AMDSMI_GPU_METRICS_CACHE_MS", "0", 0);
    amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
    if (st != AMDSMI_STATUS_SUCCESS) {
      *err = "amdsmi_init: " + smi_err(st);
      return false;
    }
    inited_ = true;
    uint32_t nsock = 0;
    if ((st = amdsmi_get_socket_handles(&nsock, nullptr)) != AMDSMI_STATUS_SUCCESS) {
      *err = "amdsmi_get_socket_handles: " + smi_err(st);
      return false;
    }
    std::vector<amdsmi_socket_handle> socks(nsock);
    amdsmi_get_socket_handles(&nsock, socks.data());
    devices->clear();
    for (uint32_t s = 0; s < nsock; ++s) {
      uint32_t np = 0;
      amdsmi_get_processor_handles(socks[s], &np, nullptr);
      std::vector<amdsmi_processor_handle> ph(np);
      amdsmi_get_processor_handles(socks[s], &np, ph.data());
      for (uint32_t p = 0; p < np; ++p) {
        processor_type_t type;
        if (amdsmi_get_processor_type(ph[p], &type) == AMDSMI_STATUS_SUCCESS &&
            type != AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          continue;
        Dev d;
        d.h = ph[p];
        d.socket = s;
        DeviceInfo info;
        amdsmi_bdf_t bdf{};
        if (amdsmi_get_gpu_device_bdf(d.h, &bdf) == AMDSMI_STATUS_SUCCESS) {
          char b[32];
          std::snprintf(b, sizeof(b), "%04llx:%02x:%02x.%x", (unsigned long long)bdf.domain_number,
                        unsigned(bdf.bus_number), unsigned(bdf.device_number),
                        unsigned(bdf.function_number));
          info.bdf = b;
        }
        char uuid[AMDSMI_GPU_UUID_SIZE + 1] = {0};
        unsigned int ul = AMDSMI_GPU_UUID_SIZE;
        if (amdsmi_get_gpu_device_uuid(d.h, &ul, uuid) == AMDSMI_STATUS_SUCCESS) info.uuid = uuid;
        amdsmi_enumeration_info_t en{};
        if (amdsmi_get_gpu_enumeration_info(d.h, &en) == AMDSMI_STATUS_SUCCESS) {
          info.render_minor = int(en.drm_render);
          info.card = int(en.drm_card);
          info.hip_id = int(en.hip_id);
        }
        amdsmi_kfd_info_t kfd{};
        if (amdsmi_get_gpu_kfd_info(d.h, &kfd) == AMDSMI_STATUS_SUCCESS) {
          if (kfd.kfd_id != ~0ull) info.kfd_gpu_id = uint32_t(kfd.kfd_id);
          if (kfd.current_partition_id != 0xFFFFFFFFu && kfd.current_partition_id < 8)
            info.partition_id = int(kfd.current_partition_id);
        }
        char part[32] = {0};
        if (amdsmi_get_gpu_compute_partition(d.h, part, sizeof(part) - 1) == AMDSMI_STATUS_SUCCESS)
          info.compute_partition = trim(part);
        std::memset(part, 0, sizeof(part));
        if (amdsmi_get_gpu_memory_partition(d.h, part, sizeof(part) - 1) == AMDSMI_STATUS_SUCCESS)
          info.memory_partition = trim(part);
        amdsmi_asic_info_t asic{};
        if (amdsmi_get_gpu_asic_info(d.h, &asic) == AMDSMI_STATUS_SUCCESS) {
          info.name = asic.market_name;
          info.num_cu = asic.num_of_compute_units;
        }
        uint16_t xcd = 0;  // XCDs in this partition (8 on an SPX-mode MI355X)
        if (amdsmi_get_gpu_xcd_counter(d.h, &xcd) == AMDSMI_STATUS_SUCCESS && xcd > 0 && xcd <= kMaxXcc)
          info.num_xcc = xcd;
        uint64_t total = 0;
        if (amdsmi_get_gpu_memory_total(d.h, AMDSMI_MEM_TYPE_VRAM, &total) == AMDSMI_STATUS_SUCCESS)
          info.vram_total = total;
        amdsmi_power_cap_info_t cap{};
        if (amdsmi_get_power_cap_info(d.h, 0, &cap) == AMDSMI_STATUS_SUCCESS)
          d.power_cap_w = double(cap.power_cap) * 1e-6;
        // xGMI peer map: static topology, so read it once (amdsmi.h:5526).
        amdsmi_link_metrics_t lm{};
        if (amdsmi_get_link_metrics(d.h, &lm) == AMDSMI_STATUS_SUCCESS) {
          // Every slot, not the first num_links: on MI355X num_links counts the 7 connected
          // links while slot 0 is the unconnected one, so the 7th peer sits in slot 7
          // (measured, tests/test_gpu.py::test_xgmi_links_carry_amdsmi_peers).
          for (uint32_t l = 0; l < uint32_t(kMaxXgmiLinks); ++l) {
            const auto& b = lm.links[l].bdf;
            if (b.bus_number == 0xff) continue;  // unconnected slot (measured: ff:1f.7)
            char pb[32];
            std::snprintf(pb, sizeof(pb), "%04llx:%02x:%02x.%x", (unsigned long long)b.domain_number,
                          unsigned(b.bus_number), unsigned(b.device_number), unsigned(b.function_number));
            info.xgmi_peer_bdf[l] = pb;
          }
        }
        bool any_peer = false;
        for (const auto& pb : info.xgmi_peer_bdf) any_peer = any_peer || !pb.empty();
        if (!any_peer) xgmi_peers_from_sysfs(root_, info.bdf, info.xgmi_peer_bdf);  // amdgpu's own port map
        info.index = int(devs_.size());
        info.dev_node = render_dev_node(root_, info.render_minor, info.bdf);
        read_board_info(root_, &info);
        if (info.render_minor >= 0) {
          std::string dir = root_ + "/sys/class/drm/renderD" + std::to_string(info.render_minor) + "/device";
          // partitions >= 1 sit on an XCP platform device: socket files are on the PCI function
          if (info.dev_node != info.bdf && ::access((dir + "/gpu_metrics").c_str(), F_OK) != 0)
            dir = root_ + "/sys/bus/pci/devices/" + info.bdf;
          d.vram_used_file.open(dir + "/mem_info_vram_used");
          std::string e;
          d.gm.set_partition(info.partition_id, int(info.num_xcc));
          d.xcp = info.partition_id;
          d.nxcc = int(info.num_xcc);
          if (!force_smi_ && d.gm.open(dir + "/gpu_metrics", &e)) {
            // a bracket can still straddle a PMFW refresh oddly: a few attempts, 25 ms apart
            for (int attempt = 0; attempt < 3 && !d.fast_ok; ++attempt) {
              if (attempt) ::usleep(25000);
              d.fast_ok = validate(d);
            }
          }
          d.gm.set_coalesce(coalesce_metrics_);
          d.gm.set_min_fresh_interval(metrics_min_ns_);
          d.gm.set_fake_cost(fake_metrics_cost_ns_);
          if (!d.fast_ok)
            GPUEXP_LOG(LogLevel::kInfo, "amdsmi",
                       "gpu " + std::to_string(info.index) + ": using amdsmi_get_gpu_metrics_info per tick (" +
                           (e.empty() ? d.validate_msg : e) + ")");
        }
        devs_.push_back(std::move(d));
        devices->push_back(info);
      }
    }
    if (devices->empty()) {
      *err = "amdsmi found no AMD GPUs";
      return false;
    }
    // (the partitions of a socket are the GPU processors of one amdsmi socket handle)
    share_socket_fetches(devices, [this](size_t i) { return devs_[i].fast_ok ? &devs_[i].gm : nullptr; },
                         [this](size_t i) { return std::to_string(devs_[i].socket); });
    return true;
  }

  // Reads the blob through amdsmi, directly, and through amdsmi again, and compares every
  // field the engine exports: hardware accumulators must lie between the two amdsmi reads,
  // static fields must agree exactly, instantaneous ones within a sensor's jitter.
  bool validate(Dev& d) {
    DeviceSample a, b1, b2;
    amdsmi_gpu_metrics_t m1{}, m2{};
    if (amdsmi_get_gpu_metrics_info(d.h, &m1) != AMDSMI_STATUS_SUCCESS) {
      d.validate_msg = "amdsmi metrics failed";
      return false;
    }
    if (!d.gm.read(&a)) {
      d.validate_msg = "raw read failed";
      return false;
    }
    if (amdsmi_get_gpu_metrics_info(d.h, &m2) != AMDSMI_STATUS_SUCCESS) {
      d.validate_msg = "amdsmi metrics failed";
      return false;
    }
    from_amdsmi_metrics(m1, &b1, d.xcp, d.nxcc);
    from_amdsmi_metrics(m2, &b2, d.xcp, d.nxcc);
    int fields = 0;
    std::string bad;
    auto between = [&](const char* f, double lo, double v, double hi) {
      ++fields;
      const bool ok = (std::isnan(lo) && std::isnan(v) && std::isnan(hi)) || (lo <= v && v <= hi);
      if (!ok && bad.empty()) bad = f;
    };
    auto near = [&](const char* f, double x, double v, double y, double tol) {
      ++fields;
      const bool nan = std::isnan(x) && std::isnan(v) && std::isnan(y);
      const bool ok = nan || (v >= std::min(x, y) - tol && v <= std::max(x, y) + tol);
      if (!ok && bad.empty()) bad = f;
    };
    auto acc = [&](const char* f, uint64_t lo, uint64_t v, uint64_t hi) {
      between(f, double(lo), double(v), double(hi));
    };
    acc("energy_accumulator", b1.energy_acc, a.energy_acc, b2.energy_acc);
    acc("firmware_timestamp", b1.fw_ts_10ns, a.fw_ts_10ns, b2.fw_ts_10ns);
    acc("accumulation_counter", b1.accumulation_counter, a.accumulation_counter, b2.accumulation_counter);
    acc("ppt_residency_acc", b1.res_ppt, a.res_ppt, b2.res_ppt);
    acc("socket_thm_residency_acc", b1.res_socket_thm, a.res_socket_thm, b2.res_socket_thm);
    acc("vr_thm_residency_acc", b1.res_vr_thm, a.res_vr_thm, b2.res_vr_thm);
    acc("hbm_thm_residency_acc", b1.res_hbm_thm, a.res_hbm_thm, b2.res_hbm_thm);
    acc("prochot_residency_acc", b1.res_prochot, a.res_prochot, b2.res_prochot);
    acc("pcie_bandwidth_acc", b1.pcie_bw_acc, a.pcie_bw_acc, b2.pcie_bw_acc);
    between("pcie_replay_count_acc", b1.pcie_replay, a.pcie_replay, b2.pcie_replay);
    between("pcie_nak_sent_count_acc", b1.pcie_nak_sent, a.pcie_nak_sent, b2.pcie_nak_sent);
    between("pcie_nak_rcvd_count_acc", b1.pcie_nak_rcvd, a.pcie_nak_rcvd, b2.pcie_nak_rcvd);
    between("pcie_l0_to_recov_count_acc", b1.pcie_l0_recov, a.pcie_l0_recov, b2.pcie_l0_recov);
    for (int l = 0; l < kMaxXgmiLinks; ++l) {
      acc("xgmi_read_data_acc", b1.xgmi_read_kb[l], a.xgmi_read_kb[l], b2.xgmi_read_kb[l]);
      acc("xgmi_write_data_acc", b1.xgmi_write_kb[l], a.xgmi_write_kb[l], b2.xgmi_write_kb[l]);
      near("xgmi_link_status", b1.xgmi_link_up[l], a.xgmi_link_up[l], b2.xgmi_link_up[l], 0);
    }
    for (int x = 0; x < kMaxXcc; ++x) {
      acc("xcp_stats.gfx_busy_acc", b1.gfx_busy_acc[x], a.gfx_busy_acc[x], b2.gfx_busy_acc[x]);
      near("current_gfxclks", b1.clk_gfx_xcc[x], a.clk_gfx_xcc[x], b2.clk_gfx_xcc[x], 400);
    }
    near("vram_max_bandwidth", b1.vram_max_bw_gbs, a.vram_max_bw_gbs, b2.vram_max_bw_gbs, 0);
    near("pcie_link_width", b1.pcie_width, a.pcie_width, b2.pcie_width, 0);
    near("pcie_link_speed", b1.pcie_speed_gts, a.pcie_speed_gts, b2.pcie_speed_gts, 0);
    near("xgmi_link_width", b1.xgmi_width, a.xgmi_width, b2.xgmi_width, 0);
    near("xgmi_link_speed", b1.xgmi_speed, a.xgmi_speed, b2.xgmi_speed, 0);
    near("current_uclk", b1.clk_mem, a.clk_mem, b2.clk_mem, 0);
    near("current_socclk", b1.clk_soc, a.clk_soc, b2.clk_soc, 400);
    near("temperature_hotspot", b1.temp_hotspot, a.temp_hotspot, b2.temp_hotspot, 3);
    near("temperature_mem", b1.temp_mem, a.temp_mem, b2.temp_mem, 3);
    near("temperature_vrsoc", b1.temp_vrsoc, a.temp_vrsoc, b2.temp_vrsoc, 3);
    near("current_socket_power", b1.power_w, a.power_w, b2.power_w, 100);
    near("average_gfx_activity", b1.gfx_activity, a.gfx_activity, b2.gfx_activity, 25);
    near("average_umc_activity", b1.umc_activity, a.umc_activity, b2.umc_activity, 25);
    near("pcie_bandwidth_inst", b1.pcie_bw_inst, a.pcie_bw_inst, b2.pcie_bw_inst, 64);
    ++fields;
    if ((a.num_partition != b1.num_partition || a.num_xgmi_links != b1.num_xgmi_links) && bad.empty())
      bad = "num_partition/num_xgmi_links";
    const bool ok = bad.empty();
    d.validated_fields = fields;
    d.validate_msg = ok ? "raw gpu_metrics v1.8 validated against amdsmi (" + std::to_string(fields) + " checks)"
                        : "raw decode disagrees with amdsmi on " + bad;
    return ok;
  }

  void sample(const DeviceInfo& dev, DeviceSample* out) override {
    Dev& d = devs_.at(size_t(dev.index));
    bool ok = false;
    if (d.fast_ok) {
      ok = d.gm.read(out, out->host_ns);
      if (!ok && __atomic_fetch_add(&d.raw_failures, 1, __ATOMIC_RELAXED) == 0)
        GPUEXP_LOG(LogLevel::kWarn, "amdsmi", "gpu " + std::to_string(dev.index) + ": raw gpu_metrics read failed (" +
                                                  out->error + "); falling back to amdsmi_get_gpu_metrics_info");
    }
    if (!ok) {
      out->error.clear();
      amdsmi_gpu_metrics_t m{};
      const uint64_t w0 = mono_ns(), c0 = thread_cpu_ns();
      amdsmi_status_t st = amdsmi_get_gpu_metrics_info(d.h, &m);
      out->metrics_cpu_ns = thread_cpu_ns() - c0;
      out->metrics_wall_ns = mono_ns() - w0;
      if (st != AMDSMI_STATUS_SUCCESS) {
        out->ok = false;
        out->error = "amdsmi_get_gpu_metrics_info: " + smi_err(st);
        return;
      }
      from_amdsmi_metrics(m, out, d.xcp, d.nxcc);
    }
    uint64_t used = 0;
    const uint64_t v0 = out->time_parts ? mono_ns() : 0;
    if (!out->read_memory) {
    } else if (d.vram_used_file.read_u64(&used)) {
      out->vram_used = double(used);
    } else if (amdsmi_get_gpu_memory_usage(d.h, AMDSMI_MEM_TYPE_VRAM, &used) == AMDSMI_STATUS_SUCCESS) {
      out->vram_used = double(used);
    }
    if (out->time_parts) out->vram_wall_ns = mono_ns() - v0;
    out->vram_total = double(dev.vram_total);
    out->power_cap_w = d.power_cap_w;
    out->ok = true;
  }

  bool processes(const DeviceInfo& dev, std::vector<ProcSample>* out) override {
    if (!amdsmi_procs_) return false;
    Dev& d = devs_.at(size_t(dev.index));
    out->clear();
    uint32_t n = uint32_t(d.procbuf.size());
    amdsmi_status_t st = amdsmi_get_gpu_process_list(d.h, &n, d.procbuf.data());
    if (st == AMDSMI_STATUS_OUT_OF_RESOURCES || n > d.procbuf.size()) {
      d.procbuf.resize(size_t(n) + 16);
      n = uint32_t(d.procbuf.size());
      st = amdsmi_get_gpu_process_list(d.h, &n, d.procbuf.data());
    }
    if (st != AMDSMI_STATUS_SUCCESS) return true;
    for (uint32_t i = 0; i < n && i < d.procbuf.size(); ++i) {
      const auto& p = d.procbuf[i];
      ProcSample ps;
      ps.pid = int(p.pid);
      ps.device = dev.index;
      ps.vram_bytes = double(p.memory_usage.vram_mem ? p.memory_usage.vram_mem : p.mem);
      ps.cu_occupancy = double(p.cu_occupancy);
      ps.gfx_ns = double(p.engine_usage.gfx);
      ps.name = p.name;
      out->push_back(ps);
    }
    return true;
  }

  double metrics_period_s(const DeviceInfo& dev) override {
    return double(devs_.at(size_t(dev.index)).gm.period_ns()) * 1e-9;
  }

  void update_metrics_min_interval(const DeviceInfo& dev, uint64_t ns, uint64_t not_before_ns = 0) override {
    devs_.at(size_t(dev.index)).gm.set_min_fresh_interval(ns);
    devs_.at(size_t(dev.index)).gm.defer_fresh_until(not_before_ns);
  }

  std::string describe(const DeviceInfo& dev) override {
    const Dev& d = devs_.at(size_t(dev.index));
    const uint64_t fails = __atomic_load_n(&d.raw_failures, __ATOMIC_RELAXED);  // sampler thread writes
    if (d.fast_ok && fails)
      return "raw gpu_metrics v1.8 with " + std::to_string(fails) + " failed reads (amdsmi fallback)";
    return d.fast_ok ? "raw gpu_metrics v1.8 (validated against amdsmi: " + std::to_string(d.validated_fields) +
                           " field checks)"
                     : "amdsmi_get_gpu_metrics_info (" + d.validate_msg + ")";
  }

  void shutdown() override {
    if (inited_) amdsmi_shut_down();
    inited_ = false;
  }

 private:
  std::string root_;
  bool amdsmi_procs_;
  bool force_smi_;
  bool inited_ = false;
  std::vector<Dev> devs_;
};

std::unique_ptr<Backend> make_amdsmi_backend(const std::string& host_root, bool amdsmi_procs,
                                             bool force_amdsmi_metrics) {
  return std::make_unique<AmdsmiBackend>(host_root, amdsmi_procs, force_amdsmi_metrics);
}

}  // namespace gpuexp
