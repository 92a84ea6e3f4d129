// Mock GPU backend (BASELINE config 1: "mock-GPU backend on CPU, 1 fake device").
// Values are smooth deterministic functions of the injected sample time, so tests can
// assert exact rates; every field can be pinned and faults injected from Python.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "gpuexp/backends.h"

namespace gpuexp {

MockBackend::MockBackend(int num_devices, uint32_t kfd_id_base)
    : n_(num_devices), kfd_base_(kfd_id_base), scripts_(size_t(num_devices > 0 ? num_devices : 0)) {}

bool MockBackend::init(std::vector<DeviceInfo>* devices, std::string* err) {
  if (n_ <= 0) {
    *err = "mock backend needs >= 1 device";
    return false;
  }
  devices->clear();
  for (int i = 0; i < n_; ++i) {
    DeviceInfo d;
    d.index = i;
    char buf[64];
    std::snprintf(buf, sizeof(buf), "0000:%02x:00.0", 0x10 + 0x10 * i);
    d.bdf = buf;
    d.dev_node = d.bdf;
    std::snprintf(buf, sizeof(buf), "e2ff75a3-0000-1000-80%02x-00000000%04x", i, 0xa000 + i);
    d.uuid = buf;
    d.name = "AMD Instinct MI355X (mock)";
    d.vbios_version = "113-M3550100-100";
    d.product_name = "AMD Instinct MI355X";
    d.product_number = "102-M3550-00";
    std::snprintf(buf, sizeof(buf), "MOCK%08d", i);
    d.serial_number = buf;
    d.firmware = {{"mec", "0x0000009f"}, {"rlc", "0x00000036"}, {"smc", "0x00554500"}, {"sos", "0x00360054"}};
    d.kfd_gpu_id = kfd_base_ + uint32_t(i);
    d.render_minor = 128 + i;
    d.card = i;
    d.hip_id = i;
    d.vram_total = 309220868096ull;  // measured MI355X mem_info_vram_total
    d.num_xcc = 8;
    d.num_cu = 256;
    // Fully connected 8-GPU OAM mesh: link 0 unsupported, links 1..7 to peers.
    for (int l = 1; l < kMaxXgmiLinks; ++l) {
      int peer = (i + l) % 8;
      std::snprintf(buf, sizeof(buf), "0000:%02x:00.0", 0x10 + 0x10 * peer);
      d.xgmi_peer_bdf[l] = buf;
    }
    devices->push_back(d);
  }
  return true;
}

double MockBackend::get(const Script& s, const char* field, double dflt) const {
  auto it = s.overrides.find(field);
  return it == s.overrides.end() ? dflt : it->second;
}

void MockBackend::sample(const DeviceInfo& dev, DeviceSample* out) {
  std::lock_guard<std::mutex> lk(mu_);
  Script& s = scripts_[size_t(dev.index)];
  uint64_t now = out->host_ns;
  if (s.fault == "error" || s.fault == "vanish") {
    out->ok = false;
    out->error = s.fault == "vanish" ? "device vanished" : "AMDSMI_STATUS_DRM_ERROR (injected)";
    return;
  }
  double dt = s.started && now > s.last_ns ? double(now - s.last_ns) * 1e-9 : 0.0;
  s.started = true;
  s.last_ns = now;
  double t = double(now) * 1e-9;
  double ph = 0.7 * dev.index;

  out->ok = true;
  out->fw_ts_10ns = now / 10;
  out->gfx_activity = get(s, "gfx_activity", std::round(50 + 45 * std::sin(0.5 * t + ph)));
  out->umc_activity = get(s, "umc_activity", std::round(30 + 25 * std::sin(0.3 * t + ph)));
  out->vram_total = double(dev.vram_total);
  out->vram_used = get(s, "vram_used", 297766912.0 + 1e9 * dev.index);
  out->power_w = get(s, "power_w", std::round(600 + 300 * std::sin(0.2 * t + ph)));
  out->power_cap_w = get(s, "power_cap_w", 1400);
  out->temp_hotspot = get(s, "temp_hotspot", std::round(55 + 10 * std::sin(0.1 * t + ph)));
  out->temp_mem = get(s, "temp_mem", std::round(45 + 5 * std::sin(0.1 * t + ph)));
  out->temp_vrsoc = get(s, "temp_vrsoc", 41);
  out->clk_gfx = get(s, "clk_gfx", 2100);
  for (uint32_t x = 0; x < dev.num_xcc && x < uint32_t(kMaxXcc); ++x) out->clk_gfx_xcc[x] = out->clk_gfx;
  out->clk_soc = get(s, "clk_soc", 1000);
  out->clk_mem = get(s, "clk_mem", 2000);
  out->pcie_width = 16;
  out->pcie_speed_gts = 32;
  out->pcie_bw_inst = get(s, "pcie_bw_gbs", 18) * 8000.0;  // PMFW unit: Mb/s
  out->pcie_replay = 0;
  out->pcie_nak_sent = get(s, "pcie_nak_sent", 0);
  out->pcie_nak_rcvd = get(s, "pcie_nak_rcvd", 0);
  out->pcie_l0_recov = get(s, "pcie_l0_recov", 0);
  out->xgmi_width = 16;
  out->xgmi_speed = 32;
  out->ecc_ce = get(s, "ecc_ce", 0);
  out->ecc_ue = get(s, "ecc_ue", 0);
  out->aer_cor = get(s, "aer_cor", 0);
  out->aer_nonfatal = get(s, "aer_nonfatal", 0);
  out->aer_fatal = get(s, "aer_fatal", 0);
  out->pages_retired = get(s, "pages_retired", 0);
  out->pages_pending = get(s, "pages_pending", 0);
  out->pages_unreservable = get(s, "pages_unreservable", 0);
  out->gtt_total = get(s, "gtt_total", 1024.0 * (1ull << 30));
  out->gtt_used = get(s, "gtt_used", 2.0 * (1ull << 30));
  out->vram_max_bw_gbs = 8192;

  // Integrate accumulators with the scripted rates (none on a traffic-file rehearsal).
  s.energy_units += out->power_w * dt / 15.259e-6;
  const bool traffic = !traffic_path_.empty();
  double rd_rate = traffic ? 0.0 : get(s, "xgmi_read_rate_kbps", 1000.0);   // per link
  double wr_rate = traffic ? 0.0 : get(s, "xgmi_write_rate_kbps", 1000.0);
  for (int l = 1; l < kMaxXgmiLinks; ++l) {
    double r = s.xgmi_frac[0][l] + rd_rate * dt, w = s.xgmi_frac[1][l] + wr_rate * dt;
    s.xgmi_rd_kb[l] += uint64_t(r);
    s.xgmi_wr_kb[l] += uint64_t(w);
    s.xgmi_frac[0][l] = r - std::floor(r);
    s.xgmi_frac[1][l] = w - std::floor(w);
  }
  s.accum += dt * 1000.0;  // accumulation counter ticks at 1 kHz in the mock
  for (int c = 0; c < kMaxXcc; ++c) s.busy_acc[c] += out->gfx_activity * dt * 1000.0;
  s.res_ppt += get(s, "ppt_residency_percent", 0.0) / 100.0 * dt * 1000.0;
  s.pcie_acc += out->pcie_bw_inst * dt;

  if (s.fault == "counter_reset") {
    s.energy_units = 0;
    for (int l = 0; l < kMaxXgmiLinks; ++l) s.xgmi_rd_kb[l] = s.xgmi_wr_kb[l] = 0;
    s.fault = "none";
  } else if (s.fault == "wrap") {
    for (int l = 0; l < kMaxXgmiLinks; ++l) s.xgmi_rd_kb[l] = ~uint64_t(0) - 100;
    s.fault = "none";
  }

  out->energy_valid = true;
  out->energy_acc = uint64_t(s.energy_units);
  out->energy_unit_j = 15.259e-6;
  out->num_xgmi_links = kMaxXgmiLinks;
  out->xgmi_valid = true;
  out->xgmi_link_up[0] = kNaN;
  std::vector<uint64_t> m;
  const bool have_m = traffic && read_traffic(&m);
  for (int l = 1; l < kMaxXgmiLinks; ++l) {
    out->xgmi_read_kb[l] = s.xgmi_rd_kb[l];
    out->xgmi_write_kb[l] = s.xgmi_wr_kb[l];
    const int peer = (dev.index + l) % 8;  // the mesh of init()
    if (have_m && peer < n_) {
      out->xgmi_write_kb[l] += m[size_t(dev.index) * size_t(n_) + size_t(peer)] / 1024;
      out->xgmi_read_kb[l] += m[size_t(peer) * size_t(n_) + size_t(dev.index)] / 1024;
    }
    out->xgmi_link_up[l] = 1;
  }
  out->residency_valid = true;
  out->accumulation_counter = uint64_t(s.accum);
  out->res_ppt = uint64_t(s.res_ppt);
  out->pcie_bw_acc = uint64_t(s.pcie_acc);
  for (int c = 0; c < kMaxXcc; ++c) out->gfx_busy_acc[c] = uint64_t(s.busy_acc[c]);
}

bool MockBackend::processes(const DeviceInfo& dev, std::vector<ProcSample>* out) {
  std::lock_guard<std::mutex> lk(mu_);
  bool any = false;
  for (auto& s : scripts_) any = any || s.has_procs;
  if (!any) return false;
  out->clear();
  const Script& s = scripts_[size_t(dev.index)];
  if (s.fault == "error" || s.fault == "vanish") return true;
  for (auto p : s.procs) {
    p.device = dev.index;
    out->push_back(p);
  }
  return true;
}

bool MockBackend::counters(const DeviceInfo& dev, double dt_s, CounterReading* out) {
  std::lock_guard<std::mutex> lk(mu_);
  const Script& s = scripts_[size_t(dev.index)];
  if (s.fault == "error" || s.fault == "vanish") return false;
  double busy = get(s, "gfx_activity", 50);
  out->ok = true;
  out->gui_active_pct = get(s, "gui_active_pct", busy);
  out->sq_busy_pct = get(s, "sq_busy_pct", busy * 0.95);
  out->mfma_busy_pct = get(s, "mfma_busy_pct", busy * 0.6);
  // while-active utilisation = busy share of the GUI-active share
  const double gui = out->gui_active_pct;
  out->mfma_util_pct = get(s, "mfma_util_pct", gui > 0 ? std::min(100.0, out->mfma_busy_pct * 100.0 / gui) : 0.0);
  out->waves_per_s = get(s, "waves_per_s", 1e6 * busy);
  out->lds_active_pct = get(s, "lds_active_pct", busy * 0.3);
  out->lds_bank_conflict_pct = get(s, "lds_bank_conflict_pct", 1.5);
  out->hbm_read_bps = get(s, "hbm_read_bps", 4e12 * busy / 100);
  out->hbm_write_bps = get(s, "hbm_write_bps", 1e12 * busy / 100);
  out->remote_read_bps = get(s, "remote_read_bps", 0.0);
  out->remote_write_bps = get(s, "remote_write_bps", 0.0);
  // a bf16 pod at the MFMA busy share of a 2.5 PFLOP/s dense peak unless scripted
  out->mfma_bf16_flops = get(s, "mfma_bf16_flops", 2.5e15 * out->mfma_busy_pct / 100);
  out->mfma_fp8_flops = get(s, "mfma_fp8_flops", 0.0);
  // occupancy limiters: waves wait for a CU a quarter of the busy time, mostly for LDS
  out->dispatch_stall_pct = get(s, "dispatch_stall_pct", busy * 0.25);
  out->lds_limited_pct = get(s, "lds_limited_pct", 80.0);
  out->wave_limited_pct = get(s, "wave_limited_pct", 10.0);
  out->vgpr_limited_pct = get(s, "vgpr_limited_pct", 0.0);
  out->sgpr_limited_pct = get(s, "sgpr_limited_pct", 0.0);
  // every XCD equally busy unless scripted ("xcc_mfma_busy_pct" sets them all)
  out->nxcc = int(std::min<uint32_t>(dev.num_xcc, uint32_t(kMaxXcc)));
  for (int x = 0; x < out->nxcc; ++x) out->xcc_mfma_busy_pct[x] = get(s, "xcc_mfma_busy_pct", out->mfma_busy_pct);
  (void)dt_s;
  return true;
}

bool MockBackend::sentinel(const DeviceInfo& dev, SentinelReading* out) {
  std::lock_guard<std::mutex> lk(mu_);
  const Script& s = scripts_[size_t(dev.index)];
  if (s.fault == "error" || s.fault == "vanish") return false;
  out->ok = true;
  out->sclk_hz = get(s, "sentinel_sclk_hz", 2.1e9);
  out->dispatch_latency_s = get(s, "sentinel_latency_s", 8e-6);
  out->xcc_id = double(dev.index % 8);
  // One wave per XCD; later workgroups of the round-robin deal start a little later.
  out->mem_latency_s = get(s, "sentinel_memory_latency_s", 1.2e-6);
  for (uint32_t x = 0; x < dev.num_xcc && x < uint32_t(kMaxXcc); ++x) {
    out->xcc_latency_s[x] = out->dispatch_latency_s + 0.1e-6 * x;
    out->xcc_mem_latency_s[x] = out->mem_latency_s;
  }
  out->runs = s.started ? uint64_t(s.accum) : 0;
  out->pending_s = get(s, "sentinel_pending_s", 0.0);
  return true;
}

void MockBackend::set_value(int dev, const std::string& field, double v) {
  std::lock_guard<std::mutex> lk(mu_);
  if (dev < 0 || dev >= n_) return;
  if (std::isnan(v))
    scripts_[size_t(dev)].overrides.erase(field);
  else
    scripts_[size_t(dev)].overrides[field] = v;
}

void MockBackend::set_processes(int dev, const std::vector<ProcSample>& procs) {
  std::lock_guard<std::mutex> lk(mu_);
  if (dev < 0 || dev >= n_) return;
  scripts_[size_t(dev)].procs = procs;
  for (auto& s : scripts_) s.has_procs = true;
}

void MockBackend::clear_processes() {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& s : scripts_) {
    s.procs.clear();
    s.has_procs = false;
  }
}

void MockBackend::set_fault(int dev, const std::string& fault) {
  std::lock_guard<std::mutex> lk(mu_);
  if (dev < 0 || dev >= n_) return;
  scripts_[size_t(dev)].fault = fault;
}

void MockBackend::set_traffic_file(const std::string& path) {
  std::lock_guard<std::mutex> lk(mu_);
  traffic_path_ = path;
}

bool MockBackend::read_traffic(std::vector<uint64_t>* m) const {
  const size_t n = size_t(n_) * size_t(n_);
  m->assign(n, 0);
  const int fd = ::open(traffic_path_.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  const ssize_t r = ::pread(fd, m->data(), n * sizeof(uint64_t), 0);
  ::close(fd);
  if (r < 0) return false;
  if (size_t(r) < n * sizeof(uint64_t))  // a short file: the rest has not been written yet
    std::memset(reinterpret_cast<char*>(m->data()) + r, 0, n * sizeof(uint64_t) - size_t(r));
  return true;
}

}  // namespace gpuexp
