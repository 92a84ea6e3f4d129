// Loaders for the optional sources: the rocprofiler-sdk counter plugin (dlopen'd so the
// core never registers itself as a profiler tool in processes that only want the
// exporter's other parts) and the RCCL tracer shared-memory files.
#include <dirent.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <map>
#include <unordered_map>

#include "gpuexp/common.h"
#include "gpuexp/rccl_shm.h"
#include "gpuexp/sources.h"

namespace gpuexp {

namespace {

// C ABI of _gpuexp_rocprof.so (csrc/gpuexp/rocprof_plugin.cc).
using rp_init_fn = int (*)(int ndev, const char* const* bdfs, char* err, int errlen);
using rp_sample_fn = int (*)(int dev, double dt_s, double* out8);
using rp_shutdown_fn = void (*)();
using rp_status_fn = const char* (*)();
using rp_scope_fn = int (*)(int dev);

class PluginCounters : public CounterSource {
 public:
  PluginCounters(std::string path, int window_ms, int interval_ms)
      : path_(std::move(path)), window_ms_(window_ms), interval_ms_(interval_ms) {}
  ~PluginCounters() override { stop(); }

  bool start(const std::vector<DeviceInfo>& devs, std::string* err) override {
    handle_ = ::dlopen(path_.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!handle_) {
      const char* e = ::dlerror();
      *err = std::string("dlopen ") + path_ + ": " + (e ? e : "?");
      return false;
    }
    init_ = reinterpret_cast<rp_init_fn>(::dlsym(handle_, "gpuexp_rp_init"));
    sample_ = reinterpret_cast<rp_sample_fn>(::dlsym(handle_, "gpuexp_rp_sample"));
    shutdown_ = reinterpret_cast<rp_shutdown_fn>(::dlsym(handle_, "gpuexp_rp_shutdown"));
    status_fn_ = reinterpret_cast<rp_status_fn>(::dlsym(handle_, "gpuexp_rp_status"));
    scope_fn_ = reinterpret_cast<rp_scope_fn>(::dlsym(handle_, "gpuexp_rp_scope"));
    if (!init_ || !sample_ || !shutdown_) {
      *err = "plugin " + path_ + " lacks the gpuexp_rp_* ABI";
      return false;
    }
    using duty_fn = void (*)(int, int);
    if (auto duty = reinterpret_cast<duty_fn>(::dlsym(handle_, "gpuexp_rp_set_duty")))
      duty(window_ms_, interval_ms_);
    std::vector<const char*> bdfs;
    for (auto& d : devs) bdfs.push_back(d.bdf.c_str());
    char ebuf[512] = {0};
    int n = init_(int(devs.size()), bdfs.data(), ebuf, sizeof(ebuf));
    if (n <= 0) {
      *err = ebuf[0] ? ebuf : "rocprofiler device counting unavailable";
      return false;
    }
    started_ = true;
    return true;
  }

  bool sample(int dev, double dt_s, CounterReading* out) override {
    if (!started_) return false;
    double v[8];
    if (sample_(dev, dt_s, v) != 0) return false;
    out->ok = true;
    out->mfma_busy_pct = v[0];
    out->sq_busy_pct = v[1];
    out->gui_active_pct = v[2];
    out->waves_per_s = v[3];
    out->lds_active_pct = v[4];
    out->lds_bank_conflict_pct = v[5];
    out->hbm_read_bps = v[6];
    out->hbm_write_bps = v[7];
    return true;
  }

  int scope(int dev) override { return started_ && scope_fn_ ? scope_fn_(dev) : -1; }

  void stop() override {
    if (started_ && shutdown_) shutdown_();
    started_ = false;
    // The plugin stays loaded: rocprofiler-sdk does not support re-registration, and the
    // aqlprofile plugin keeps HSA's refcount balanced itself.
  }

  std::string status() const override {
    return status_fn_ ? std::string(status_fn_()) : std::string("rocprof plugin");
  }

 private:
  std::string path_;
  int window_ms_, interval_ms_;
  void* handle_ = nullptr;
  rp_init_fn init_ = nullptr;
  rp_sample_fn sample_ = nullptr;
  rp_shutdown_fn shutdown_ = nullptr;
  rp_status_fn status_fn_ = nullptr;
  rp_scope_fn scope_fn_ = nullptr;
  bool started_ = false;
};

uint64_t pidns_inode(const std::string& proc_pid_dir) {
  struct stat st;
  if (::stat((proc_pid_dir + "/ns/pid").c_str(), &st) != 0) return 0;
  return uint64_t(st.st_ino);
}

// Last NSpid entry of /proc/<pid>/status = the PID inside the innermost namespace.
int innermost_nspid(const std::string& proc_pid_dir) {
  std::string s;
  if (!read_small_file(proc_pid_dir + "/status", &s, 8192)) return -1;
  size_t p = s.find("NSpid:");
  if (p == std::string::npos) return -1;
  size_t e = s.find('\n', p);
  std::string line = s.substr(p + 6, e == std::string::npos ? std::string::npos : e - p - 6);
  int last = -1;
  size_t i = 0;
  while (i < line.size()) {
    while (i < line.size() && (line[i] == ' ' || line[i] == '\t')) ++i;
    size_t j = i;
    while (j < line.size() && line[j] >= '0' && line[j] <= '9') ++j;
    if (j > i) last = std::atoi(line.substr(i, j - i).c_str());
    i = j + 1;
  }
  return last;
}

class ShmRcclSource : public RcclSource {
 public:
  explicit ShmRcclSource(std::string dir) : dir_(std::move(dir)) { self_ns_ = pidns_inode("/proc/self"); }
  ~ShmRcclSource() override {
    for (auto& kv : maps_) ::munmap(kv.second.base, sizeof(RcclShmFile));
  }

  void poll(std::vector<RcclTotals>* out) override {
    out->clear();
    std::map<std::string, bool> present;
    for (const std::string& name : list_dir(dir_)) {
      if (name.compare(0, 12, "gpuexp-rccl-") != 0) continue;
      present[name] = true;
      if (!maps_.count(name)) {
        int fd = ::open((dir_ + "/" + name).c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) continue;
        struct stat st;
        if (::fstat(fd, &st) != 0 || size_t(st.st_size) < sizeof(RcclShmFile)) {
          ::close(fd);
          continue;
        }
        void* p = ::mmap(nullptr, sizeof(RcclShmFile), PROT_READ, MAP_SHARED, fd, 0);
        ::close(fd);
        if (p == MAP_FAILED) continue;
        maps_[name] = Mapping{static_cast<RcclShmFile*>(p), -1};
      }
      Mapping& m = maps_[name];
      if (m.base->magic != kRcclShmMagic) continue;
      if (m.host_pid < 0) m.host_pid = host_pid_for(m.base->pidns_ino, m.base->ns_pid);
      if (m.host_pid < 0) continue;
      for (int op = 0; op < kOpNumOps; ++op) {
        uint64_t c = m.base->ops[op].calls.load(std::memory_order_relaxed);
        if (!c) continue;
        RcclTotals t;
        t.pid = m.host_pid;
        t.op = rccl_op_name(op);
        t.calls = c;
        t.bytes = m.base->ops[op].bytes.load(std::memory_order_relaxed);
        t.rank = reinterpret_cast<volatile int32_t*>(&m.base->rank)[0];
        t.nranks = reinterpret_cast<volatile int32_t*>(&m.base->nranks)[0];
        out->push_back(t);
      }
    }
    for (auto it = maps_.begin(); it != maps_.end();) {
      if (!present.count(it->first)) {
        ::munmap(it->second.base, sizeof(RcclShmFile));
        it = maps_.erase(it);
      } else {
        ++it;
      }
    }
  }

 private:
  struct Mapping {
    RcclShmFile* base;
    int host_pid;
  };
  int host_pid_for(uint64_t ns_ino, int ns_pid) {
    if (ns_ino == self_ns_ || ns_ino == 0) return ns_pid;  // same PID namespace
    for (const std::string& d : list_dir("/proc")) {
      if (d[0] < '0' || d[0] > '9') continue;
      std::string pd = "/proc/" + d;
      if (pidns_inode(pd) != ns_ino) continue;
      if (innermost_nspid(pd) == ns_pid) return std::atoi(d.c_str());
    }
    return -1;
  }
  std::string dir_;
  uint64_t self_ns_ = 0;
  std::unordered_map<std::string, Mapping> maps_;
};

// Directory of the core module itself (the HIP/rocprof plugins are installed beside it).
std::string self_dir() {
  Dl_info info{};
  if (::dladdr(reinterpret_cast<void*>(&self_dir), &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    size_t s = p.rfind('/');
    return s == std::string::npos ? std::string(".") : p.substr(0, s);
  }
  return ".";
}

}  // namespace

std::unique_ptr<SentinelSource> make_hip_sentinel(int ring_slots, int spin_iters) {
  // RTLD_GLOBAL is not needed: the plugin only exports its factory.  If the process has
  // already loaded a HIP runtime (e.g. torch's bundled one, same SONAME), the plugin's
  // DT_NEEDED libamdhip64.so.7 binds to it instead of loading a second copy.
  std::string path = self_dir() + "/libgpuexp_hip.so";
  void* h = ::dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    const char* e = ::dlerror();
    GPUEXP_LOG(LogLevel::kWarn, "sentinel", std::string("dlopen ") + path + ": " + (e ? e : "?"));
    return nullptr;
  }
  using factory_t = SentinelSource* (*)(int, int);
  auto f = reinterpret_cast<factory_t>(::dlsym(h, "gpuexp_make_hip_sentinel"));
  if (!f) return nullptr;
  return std::unique_ptr<SentinelSource>(f(ring_slots, spin_iters));
}

std::unique_ptr<SentinelSource> make_queue_sentinel(const std::string& counters_plugin, int ring_slots,
                                                   int spin_iters) {
  // Only from a counters plugin that is already loaded and running (RTLD_NOLOAD).
  void* h = ::dlopen(counters_plugin.c_str(), RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
  if (!h) return nullptr;
  using factory_t = SentinelSource* (*)(int, int);
  auto f = reinterpret_cast<factory_t>(::dlsym(h, "gpuexp_make_hsa_sentinel"));
  ::dlclose(h);  // drops only the NOLOAD reference; the counters source keeps it loaded
  if (!f) return nullptr;
  return std::unique_ptr<SentinelSource>(f(ring_slots, spin_iters));
}

// Default counter backend: the aqlprofile plugin (no spinning runtime thread); the
// rocprofiler-sdk plugin (_gpuexp_rocprof.so) is selectable through counters_plugin.
std::string default_rocprof_plugin() { return self_dir() + "/_gpuexp_aqlpmc.so"; }

std::unique_ptr<CounterSource> make_rocprof_counters(const std::string& plugin_path, int window_ms,
                                                     int interval_ms) {
  return std::make_unique<PluginCounters>(plugin_path, window_ms, interval_ms);
}

std::unique_ptr<RcclSource> make_rccl_source(const std::string& dir) {
  return std::make_unique<ShmRcclSource>(dir);
}

}  // namespace gpuexp
