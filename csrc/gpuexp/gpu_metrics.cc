#include "gpuexp/gpu_metrics.h"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <map>
#include <cstring>
#include <utility>

namespace gpuexp {

namespace {
inline double u16v(uint16_t v) { return v == 0xFFFF ? kNaN : double(v); }
}  // namespace

bool decode_gpu_metrics_v1_8(const void* blob, size_t len, DeviceSample* out, int xcp, int nxcc) {
  if (len < sizeof(GpuMetricsV1_8)) return false;
  GpuMetricsV1_8 m;
  std::memcpy(&m, blob, sizeof(m));
  if (m.header.format_revision != 1 || m.header.content_revision != 8) return false;
  out->temp_hotspot = u16v(m.temperature_hotspot);
  out->temp_mem = u16v(m.temperature_mem);
  out->temp_vrsoc = u16v(m.temperature_vrsoc);
  out->power_w = u16v(m.curr_socket_power);
  out->gfx_activity = u16v(m.average_gfx_activity);
  out->umc_activity = u16v(m.average_umc_activity);
  out->vram_max_bw_gbs = m.mem_max_bandwidth == ~0ull ? kNaN : double(m.mem_max_bandwidth);
  out->energy_valid = m.energy_accumulator != ~0ull;
  out->energy_acc = m.energy_accumulator;
  out->energy_unit_j = 15.259e-6;
  out->residency_valid = m.accumulation_counter != 0xFFFFFFFFu;
  out->accumulation_counter = m.accumulation_counter;
  out->res_prochot = m.prochot_residency_acc;
  out->res_ppt = m.ppt_residency_acc;
  out->res_socket_thm = m.socket_thm_residency_acc;
  out->res_vr_thm = m.vr_thm_residency_acc;
  out->res_hbm_thm = m.hbm_thm_residency_acc;
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
  int nl = 0;
  for (int l = 0; l < kMaxXgmiLinks; ++l) {
    out->xgmi_read_kb[l] = m.xgmi_read_data_acc[l] == ~0ull ? 0 : m.xgmi_read_data_acc[l];
    out->xgmi_write_kb[l] = m.xgmi_write_data_acc[l] == ~0ull ? 0 : m.xgmi_write_data_acc[l];
    out->xgmi_link_up[l] = m.xgmi_link_status[l] == 0xFFFF ? kNaN : double(m.xgmi_link_status[l] ? 1 : 0);
    if (m.xgmi_link_status[l] != 0xFFFF) nl = l + 1;
  }
  out->num_xgmi_links = nl;
  out->xgmi_valid = true;
  out->fw_ts_10ns = m.firmware_timestamp == ~0ull ? 0 : m.firmware_timestamp;
  // This partition's XCDs: their gfx clocks (mean of the valid ones = clk_gfx) and busy
  // accumulators (its own xcp_stats slot).
  if (xcp < 0 || xcp >= 8) xcp = 0;
  const int nx = nxcc > 0 && nxcc <= kMaxXcc ? nxcc : kMaxXcc;
  const int first = xcp * nx < kMaxXcc ? xcp * nx : 0;
  double sum = 0;
  int n = 0;
  for (int i = 0; i < nx && first + i < kMaxXcc; ++i) {
    const uint16_t c = m.current_gfxclk[first + i];
    if (c != 0xFFFF && c != 0) {
      sum += c;
      out->clk_gfx_xcc[i] = c;
      ++n;
    }
  }
  out->clk_gfx = n ? sum / n : kNaN;
  out->clk_soc = u16v(m.current_socclk[0]);
  out->clk_mem = u16v(m.current_uclk);
  out->num_partition = m.num_partition == 0xFFFF ? 0 : m.num_partition;
  for (int c = 0; c < kMaxXcc; ++c) out->gfx_busy_acc[c] = m.xcp_stats[xcp].gfx_busy_acc[c];
  return true;
}

void share_socket_fetches(std::vector<DeviceInfo>* devs, const std::function<GpuMetricsReader*(size_t)>& reader,
                          const std::function<std::string(size_t)>& socket) {
  std::map<std::string, std::vector<size_t>> by_bdf;
  for (size_t i = 0; i < devs->size(); ++i) {
    const std::string key = socket ? socket(i) : (*devs)[i].bdf;
    if (!key.empty()) by_bdf[key].push_back(i);
  }
  int group = 0;
  for (const auto& kv : by_bdf) {
    if (kv.second.size() < 2) continue;  // a whole GPU
    auto shared = std::make_shared<GpuMetricsShared>();
    for (size_t i : kv.second) {
      (*devs)[i].socket_group = group;
      if (GpuMetricsReader* r = reader(i)) r->set_shared(shared);
    }
    ++group;
  }
}

GpuMetricsReader::~GpuMetricsReader() {
  if (fd_ >= 0) ::close(fd_);
}

GpuMetricsReader::GpuMetricsReader(GpuMetricsReader&& o) noexcept { *this = std::move(o); }

GpuMetricsReader& GpuMetricsReader::operator=(GpuMetricsReader&& o) noexcept {
  if (this == &o) return *this;
  if (fd_ >= 0) ::close(fd_);
  fd_ = o.fd_;
  o.fd_ = -1;
  path_ = std::move(o.path_);
  fmt_ = o.fmt_;
  content_ = o.content_;
  coalesce_ = o.coalesce_;
  min_fresh_ns_ = o.min_fresh_ns_;
  not_before_ns_ = o.not_before_ns_;
  fake_cost_ns_ = o.fake_cost_ns_;
  xcp_ = o.xcp_;
  nxcc_ = o.nxcc_;
  last_n_ = o.last_n_;
  last_fw_ts_ = o.last_fw_ts_;
  t_change_ns_ = o.t_change_ns_;
  last_read_ns_ = o.last_read_ns_;
  last_was_fresh_ = o.last_was_fresh_;
  period_ns_ = o.period_ns_;
  std::copy(o.steps_, o.steps_ + kSteps, steps_);
  nsteps_ = o.nsteps_;
  fresh_reads_ = o.fresh_reads_;
  shared_ = std::move(o.shared_);
  coalesced_reads_ = o.coalesced_reads_;
  std::memcpy(buf_, o.buf_, sizeof(buf_));
  return *this;
}

bool GpuMetricsReader::open(const std::string& path, std::string* err) {
  if (fd_ >= 0) ::close(fd_);
  path_ = path;
  fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd_ < 0) {
    *err = "open " + path + " failed";
    return false;
  }
  long n = pread_once(fd_, reinterpret_cast<char*>(buf_), sizeof(buf_));
  if (n < long(sizeof(GpuMetricsHeader))) {
    *err = "short gpu_metrics read";
    ::close(fd_);
    fd_ = -1;
    return false;
  }
  auto* h = reinterpret_cast<const GpuMetricsHeader*>(buf_);
  fmt_ = h->format_revision;
  content_ = h->content_revision;
  if (!(fmt_ == 1 && content_ == 8)) {
    *err = "unsupported gpu_metrics format " + std::to_string(fmt_) + "." + std::to_string(content_);
    ::close(fd_);
    fd_ = -1;
    return false;
  }
  return true;
}

bool GpuMetricsReader::read(DeviceSample* out, uint64_t now_ns) {
  if (fd_ < 0) {
    out->error = "gpu_metrics not open";
    return false;
  }
  // Re-read 1.5 ms before the expected refresh so jitter in the PMFW period never costs a
  // whole period of staleness.
  constexpr uint64_t kGuardNs = 1500000;
  const uint64_t window = std::min(period_ns_, kMaxCoalesceNs);
  if (coalesce_ && now_ns && last_n_ > 0 && window > kGuardNs && t_change_ns_ && now_ns >= t_change_ns_ &&
      now_ns < t_change_ns_ + window - kGuardNs) {
    coalesced_reads_ += 1;
    last_was_fresh_ = false;
    out->metrics_coalesced = true;
    return decode_gpu_metrics_v1_8(buf_, size_t(last_n_), out, xcp_, nxcc_);
  }
  if ((min_fresh_ns_ && now_ns && last_n_ > 0 && last_read_ns_ && now_ns > last_read_ns_ &&
       now_ns - last_read_ns_ < min_fresh_ns_) ||
      (not_before_ns_ && now_ns && last_n_ > 0 && now_ns < not_before_ns_)) {
    coalesced_reads_ += 1;
    last_was_fresh_ = false;
    out->metrics_coalesced = true;
    return decode_gpu_metrics_v1_8(buf_, size_t(last_n_), out, xcp_, nxcc_);
  }
  long n = 0;
  if (shared_ && now_ns && shared_->tick_ns == now_ns && shared_->n > 0) {
    // another partition of this socket fetched at this tick: the same table, no SMU round trip
    n = shared_->n;
    std::memcpy(buf_, shared_->buf, size_t(n));
    out->metrics_shared = true;
  } else {
    const uint64_t w0 = mono_ns(), c0 = thread_cpu_ns();
    n = pread_once(fd_, reinterpret_cast<char*>(buf_), sizeof(buf_));
    if (fake_cost_ns_) {
      uint64_t c = c0;
      while ((c = thread_cpu_ns()) - c0 < fake_cost_ns_) {
      }
      fake_cpu_burnt_ns().fetch_add(c - c0, std::memory_order_relaxed);
    }
    out->metrics_cpu_ns = thread_cpu_ns() - c0;
    out->metrics_wall_ns = mono_ns() - w0;
    if (shared_ && n > 0) {
      std::memcpy(shared_->buf, buf_, size_t(n));
      shared_->n = n;
      shared_->tick_ns = now_ns;
    }
  }
  if (n <= 0) {
    last_n_ = 0;
    out->error = "gpu_metrics read failed";
    return false;
  }
  last_n_ = n;
  fresh_reads_ += 1;
  if (!decode_gpu_metrics_v1_8(buf_, size_t(n), out, xcp_, nxcc_)) {
    last_n_ = 0;
    out->error = "gpu_metrics decode failed";
    return false;
  }
  if (out->fw_ts_10ns && out->fw_ts_10ns != last_fw_ts_) {
    const bool bracketed = last_was_fresh_ && last_read_ns_ && now_ns > last_read_ns_;
    if (bracketed && last_fw_ts_ && out->fw_ts_10ns > last_fw_ts_) {
      steps_[nsteps_ % kSteps] = (out->fw_ts_10ns - last_fw_ts_) * 10;
      nsteps_ += 1;
      if (nsteps_ >= 5) {
        const int k = std::min(nsteps_, kSteps);
        uint64_t tmp[kSteps];
        std::copy(steps_, steps_ + k, tmp);
        std::nth_element(tmp, tmp + k / 2, tmp + k);
        period_ns_ = tmp[k / 2];
      }
    }
    last_fw_ts_ = out->fw_ts_10ns;
    // The table appeared between the previous fresh read and this one: take the midpoint.
    t_change_ns_ = bracketed ? last_read_ns_ + (now_ns - last_read_ns_) / 2 : now_ns;
  }
  last_read_ns_ = now_ns;
  last_was_fresh_ = true;
  return true;
}

}  // namespace gpuexp
