// sysfs backend: KFD topology for identity, drm sysfs + raw gpu_metrics for telemetry.
// Every path is prefixed with the host root, so tests build a fake tree (SURVEY.md §4.2
// "fake sysfs/procfs root") and a DaemonSet mounts the host's /sys read-only.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <sstream>

#include "gpuexp/backends.h"

namespace gpuexp {

CachedFile::~CachedFile() { close(); }

CachedFile& CachedFile::operator=(CachedFile&& o) noexcept {
  close();
  fd_ = o.fd_;
  path_ = std::move(o.path_);
  o.fd_ = -1;
  return *this;
}

bool CachedFile::open(const std::string& path) {
  close();
  path_ = path;
  fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  return fd_ >= 0;
}

long CachedFile::read(char* buf, size_t cap) {
  if (fd_ < 0) return -1;
  return pread_once(fd_, buf, cap);
}

bool CachedFile::read_u64(uint64_t* v) {
  char buf[64];
  long n = read(buf, sizeof(buf) - 1);
  if (n <= 0) return false;
  return parse_u64(buf, size_t(n), v);
}

void CachedFile::close() {
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

// Parses "key value\n" lines of a KFD topology `properties` file.
static std::map<std::string, uint64_t> parse_properties(const std::string& text) {
  std::map<std::string, uint64_t> kv;
  std::istringstream is(text);
  std::string k;
  std::string v;
  while (is >> k >> v) {
    uint64_t x = 0;
    if (parse_u64(v.c_str(), v.size(), &x)) kv[k] = x;
  }
  return kv;
}

namespace {
bool file_exists(const std::string& p) { return ::access(p.c_str(), F_OK) == 0; }
}  // namespace

std::string render_dev_node(const std::string& root, int render_minor, const std::string& bdf) {
  if (render_minor < 0) return bdf;
  char buf[4096];
  const std::string link = root + "/sys/class/drm/renderD" + std::to_string(render_minor) + "/device";
  if (!::realpath(link.c_str(), buf)) return bdf;
  std::string p(buf);
  const size_t sl = p.rfind('/');
  std::string base = sl == std::string::npos ? p : p.substr(sl + 1);
  // a PCI function ("dddd:bb:dd.f") or an XCP platform device ("amdgpu_xcp.<n>")
  const bool pci = base.size() == 12 && base[4] == ':' && base[7] == ':' && base[10] == '.';
  const bool xcp = base.compare(0, 11, "amdgpu_xcp.") == 0 || base.compare(0, 11, "amdgpu_xcp_") == 0;
  return pci || xcp ? base : bdf;
}

namespace {
// One xgmi_port_num line: "<node>:<port> ->  <peer node>:<peer port>" (hex, node ids from 1,
// shared by every GPU of the hive; amdgpu_xgmi.c).
bool parse_port_line(const std::string& line, unsigned* node, unsigned* port, unsigned* peer) {
  unsigned pp = 0;
  return std::sscanf(line.c_str(), " %x:%x -> %x:%x", node, port, peer, &pp) == 4;
}
}  // namespace

int xgmi_peers_from_sysfs(const std::string& root, const std::string& bdf, std::string peers[kMaxXgmiLinks]) {
  // node id -> BDF, from the first line of every GPU's own listing
  std::map<unsigned, std::string> node_bdf;
  const std::string pci = root + "/sys/bus/pci/devices";
  std::string body;
  for (const std::string& dev : list_dir(pci)) {
    if (!read_small_file(pci + "/" + dev + "/xgmi_port_num", &body)) continue;
    unsigned node = 0, port = 0, peer = 0;
    if (parse_port_line(body.substr(0, body.find('\n')), &node, &port, &peer)) node_bdf[node] = dev;
  }
  if (!read_small_file(pci + "/" + bdf + "/xgmi_port_num", &body)) return 0;
  int n = 0;
  size_t pos = 0;
  while (pos < body.size()) {
    size_t eol = body.find('\n', pos);
    if (eol == std::string::npos) eol = body.size();
    unsigned node = 0, port = 0, peer = 0;
    if (parse_port_line(body.substr(pos, eol - pos), &node, &port, &peer) && port < unsigned(kMaxXgmiLinks)) {
      auto it = node_bdf.find(peer);
      if (it != node_bdf.end()) {
        peers[port] = it->second;
        ++n;
      }
    }
    pos = eol + 1;
  }
  return n;
}

void read_board_info(const std::string& root, DeviceInfo* d) {
  const std::string dir = root + "/sys/bus/pci/devices/" + d->bdf;
  auto rd = [&](const char* f) {
    std::string v;
    return read_small_file(dir + "/" + f, &v, 256) ? trim(v) : std::string();
  };
  d->vbios_version = rd("vbios_version");
  d->product_name = rd("product_name");
  d->product_number = rd("product_number");
  d->serial_number = rd("serial_number");
  d->firmware.clear();
  const std::string suffix = "_fw_version";
  std::vector<std::string> files = list_dir(dir + "/fw_version");
  std::sort(files.begin(), files.end());
  for (const std::string& f : files) {
    if (f.size() <= suffix.size() || f.compare(f.size() - suffix.size(), suffix.size(), suffix) != 0) continue;
    std::string v;
    if (!read_small_file(dir + "/fw_version/" + f, &v, 64)) continue;
    v = trim(v);
    if (v.empty() || v == "0x00000000") continue;  // block not loaded on this ASIC
    d->firmware.emplace_back(f.substr(0, f.size() - suffix.size()), v);
  }
}

std::vector<std::string> device_owner_keys(const DeviceInfo& d) {
  auto low = [](std::string s) {
    for (auto& c : s) c = char(::tolower(static_cast<unsigned char>(c)));
    return s;
  };
  std::vector<std::string> k;
  const std::string node = low(d.dev_node.empty() ? d.bdf : d.dev_node);
  const std::string bdf = low(d.bdf);
  if (node != bdf) {
    k.push_back(node);
    std::string alt = node;
    for (auto& c : alt)
      if (c == '.') c = '_';
    if (alt != node) k.push_back(alt);
  }
  if (!bdf.empty()) k.push_back(bdf + "/" + std::to_string(d.partition_id));
  if (d.render_minor >= 0) {
    k.push_back("renderd" + std::to_string(d.render_minor));
    k.push_back("/dev/dri/renderd" + std::to_string(d.render_minor));
  }
  if (d.kfd_gpu_id) k.push_back("kfd:" + std::to_string(d.kfd_gpu_id));
  if (!d.uuid.empty()) k.push_back(low(d.uuid));
  if (node == bdf && !bdf.empty()) k.push_back(bdf);
  return k;
}

std::string SysfsBackend::uuid_from_unique_id(uint64_t unique_id, uint32_t device_id) {
  // amdsmi format: <b0>ff<devid16>-0000-1000-80<b1>-<b2..b7>, where b0..b7 are the
  // big-endian bytes of the KFD unique_id (checked against amdsmi on MI355X:
  // unique_id e296a367fef9a1be, device 0x75a3 -> e2ff75a3-0000-1000-8096-a367fef9a1be).
  char hex[17];
  std::snprintf(hex, sizeof(hex), "%016llx", static_cast<unsigned long long>(unique_id));
  char out[64];
  std::snprintf(out, sizeof(out), "%.2sff%04x-0000-1000-80%.2s-%.12s", hex, device_id & 0xFFFF,
                hex + 2, hex + 4);
  return out;
}

SysfsBackend::SysfsBackend(std::string host_root) : root_(std::move(host_root)) {
  if (!root_.empty() && root_.back() == '/') root_.pop_back();
}

bool SysfsBackend::init(std::vector<DeviceInfo>* devices, std::string* err) {
  devices->clear();
  devs_.clear();
  std::string nodes_dir = root_ + "/sys/class/kfd/kfd/topology/nodes";
  std::vector<std::string> nodes = list_dir(nodes_dir);
  std::sort(nodes.begin(), nodes.end(), [](const std::string& a, const std::string& b) {
    return std::atoi(a.c_str()) < std::atoi(b.c_str());
  });
  struct Found {
    uint64_t bdf_sort;
    DeviceInfo info;
  };
  std::vector<Found> found;
  for (auto& n : nodes) {
    uint64_t gpu_id = 0;
    if (!read_u64_file(nodes_dir + "/" + n + "/gpu_id", &gpu_id) || gpu_id == 0) continue;
    std::string props;
    if (!read_small_file(nodes_dir + "/" + n + "/properties", &props)) continue;
    auto kv = parse_properties(props);
    DeviceInfo d;
    d.kfd_gpu_id = uint32_t(gpu_id);
    uint64_t loc = kv["location_id"], dom = kv["domain"];
    char bdf[32];
    std::snprintf(bdf, sizeof(bdf), "%04llx:%02llx:%02llx.%llx", (unsigned long long)dom,
                  (unsigned long long)((loc >> 8) & 0xFF), (unsigned long long)((loc >> 3) & 0x1F),
                  (unsigned long long)(loc & 0x7));
    d.bdf = bdf;
    d.render_minor = int(kv.count("drm_render_minor") ? kv["drm_render_minor"] : 0);
    d.num_xcc = uint32_t(kv["num_xcc"]);
    uint64_t cus = kv["simd_count"] && kv["simd_per_cu"] ? kv["simd_count"] / kv["simd_per_cu"] : 0;
    d.num_cu = uint32_t(cus);
    d.uuid = uuid_from_unique_id(kv["unique_id"], uint32_t(kv["device_id"]));
    std::string name;
    if (read_small_file(nodes_dir + "/" + n + "/name", &name)) d.name = trim(name);
    found.push_back({(dom << 16) | (loc & 0xFFFF), d});
  }
  // Stable exporter index order = PCI order (what HIP/amdsmi enumerate by default).  The
  // partitions of one socket (CPX/DPX/QPX) share its BDF; KFD lists them in partition
  // order, which the stable sort keeps, so the k-th node of a BDF is partition k.
  std::stable_sort(found.begin(), found.end(),
                   [](const Found& a, const Found& b) { return a.bdf_sort < b.bdf_sort; });
  for (size_t i = 0; i < found.size(); ++i) {
    DeviceInfo d = found[i].info;
    d.index = int(i);
    d.hip_id = int(i);
    for (size_t j = i; j > 0 && found[j - 1].bdf_sort == found[i].bdf_sort; --j) d.partition_id += 1;
    auto dev = std::make_unique<Dev>();
    dev->dev_dir = root_ + "/sys/class/drm/renderD" + std::to_string(d.render_minor) + "/device";
    std::string part;
    if (read_small_file(dev->dev_dir + "/current_compute_partition", &part)) d.compute_partition = trim(part);
    if (read_small_file(dev->dev_dir + "/current_memory_partition", &part)) d.memory_partition = trim(part);
    d.dev_node = render_dev_node(root_, d.render_minor, d.bdf);
    read_board_info(root_, &d);
    // Socket-level files (gpu_metrics, mem_info_*, hwmon) live on the PCI function; an
    // XCP platform device (partitions >= 1) may not carry them.
    if (d.dev_node != d.bdf && !file_exists(dev->dev_dir + "/gpu_metrics")) {
      const std::string pci = root_ + "/sys/bus/pci/devices/" + d.bdf;
      if (file_exists(pci + "/gpu_metrics")) dev->dev_dir = pci;
    }
    dev->xcp = d.partition_id;
    dev->nxcc = int(d.num_xcc);
    uint64_t total = 0;
    if (read_u64_file(dev->dev_dir + "/mem_info_vram_total", &total)) d.vram_total = total;
    xgmi_peers_from_sysfs(root_, d.bdf, d.xgmi_peer_bdf);
    open_dev_files(dev.get());
    devices->push_back(d);
    devs_.push_back(std::move(dev));
  }
  if (devices->empty()) {
    *err = "no KFD GPU nodes under " + nodes_dir;
    return false;
  }
  share_socket_fetches(devices, [this](size_t i) { return devs_[i]->gm_ok ? &devs_[i]->gm : nullptr; });
  return true;
}

void SysfsBackend::open_dev_files(Dev* d) {
  std::string e;
  d->gm_ok = d->gm.open(d->dev_dir + "/gpu_metrics", &e);
  d->gm.set_coalesce(coalesce_metrics_);
  d->gm.set_min_fresh_interval(metrics_min_ns_);
  d->gm.set_fake_cost(fake_metrics_cost_ns_);
  d->gm.set_partition(d->xcp, d->nxcc);
  d->vram_used.open(d->dev_dir + "/mem_info_vram_used");
  d->busy.open(d->dev_dir + "/gpu_busy_percent");
  d->mem_busy.open(d->dev_dir + "/mem_busy_percent");
  // hwmon: power1_input (uW), temp*_input with labels junction/mem/edge.
  for (auto& h : list_dir(d->dev_dir + "/hwmon")) {
    std::string hd = d->dev_dir + "/hwmon/" + h;
    if (!d->power.open(hd + "/power1_input")) d->power.open(hd + "/power1_average");
    uint64_t cap = 0;
    if (read_u64_file(hd + "/power1_cap", &cap)) d->power_cap_w = double(cap) * 1e-6;
    for (int t = 1; t <= 8; ++t) {
      std::string label;
      if (!read_small_file(hd + "/temp" + std::to_string(t) + "_label", &label)) continue;
      label = trim(label);
      std::string in = hd + "/temp" + std::to_string(t) + "_input";
      if (label == "junction" || label == "hotspot") d->temp_hot.open(in);
      else if (label == "mem") d->temp_mem.open(in);
      else if (label == "edge") d->temp_edge.open(in);
    }
    break;
  }
}

void SysfsBackend::sample_fallback(Dev& d, DeviceSample* out) {
  uint64_t v = 0;
  if (d.busy.read_u64(&v)) out->gfx_activity = double(v);
  if (d.mem_busy.read_u64(&v)) out->umc_activity = double(v);
  if (d.power.read_u64(&v)) out->power_w = double(v) * 1e-6;
  if (d.temp_hot.read_u64(&v)) out->temp_hotspot = double(v) * 1e-3;
  if (d.temp_mem.read_u64(&v)) out->temp_mem = double(v) * 1e-3;
  if (d.temp_edge.read_u64(&v)) out->temp_edge = double(v) * 1e-3;
}

void SysfsBackend::sample(const DeviceInfo& dev, DeviceSample* out) {
  Dev& d = *devs_.at(size_t(dev.index));
  bool any = false;
  if (d.gm_ok) {
    if (d.gm.read(out, out->host_ns)) {
      any = true;
    } else {
      // The blob can vanish with the device (hot-unplug/reset): retry open once.
      std::string e;
      d.gm_ok = d.gm.open(d.dev_dir + "/gpu_metrics", &e) && d.gm.read(out);
      any = d.gm_ok;
    }
  }
  if (!any) sample_fallback(d, out);
  uint64_t used = 0;
  const uint64_t v0 = out->time_parts ? mono_ns() : 0;
  if (!out->read_memory) {
    any = any || d.vram_used.is_open();
  } else if (d.vram_used.read_u64(&used)) {
    out->vram_used = double(used);
    any = true;
  } else if (d.vram_used.open(d.dev_dir + "/mem_info_vram_used") && d.vram_used.read_u64(&used)) {
    out->vram_used = double(used);
    any = true;
  }
  if (out->time_parts) out->vram_wall_ns = mono_ns() - v0;
  out->vram_total = double(dev.vram_total);
  out->power_cap_w = d.power_cap_w;
  out->ok = any || !std::isnan(out->gfx_activity) || !std::isnan(out->power_w);
  if (!out->ok && out->error.empty()) out->error = "no readable telemetry under " + d.dev_dir;
}

}  // namespace gpuexp
