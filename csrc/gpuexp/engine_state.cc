// Checkpoint of the exporter's own accumulations (per-pod energy, xGMI bytes, GPU-seconds,
// KFD event counts; per-GPU event counts) so they continue across exporter restarts.
//
// Reference counterpart: none -- all of the reference's state is rebuilt every cycle
// (/root/reference/main.go:84) and its gauges are lost on restart.
#include <fcntl.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>

#include "gpuexp/engine.h"
#include "gpuexp/engine_util.h"

namespace gpuexp {

std::string Engine::device_key(size_t i) const {
  return engine_util::lower(devices_[i].bdf) + "/" + std::to_string(devices_[i].partition_id);
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

}  // namespace gpuexp
