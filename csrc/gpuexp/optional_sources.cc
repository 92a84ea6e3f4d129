// Loaders for the optional sources: the rocprofiler-sdk counter plugin (dlopen'd so the
// core never registers itself as a profiler tool in processes that only want the
// exporter's other parts) and the RCCL tracer shared-memory files.
#include <dirent.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/sysmacros.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdlib>
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
using rp_sample_fn = int (*)(int dev, double dt_s, double* out);  // kCounterOutputs doubles
using rp_shutdown_fn = void (*)();
using rp_status_fn = const char* (*)();
using rp_scope_fn = int (*)(int dev);

using rp_kick_fn = void (*)();
using rp_cpu_fn = uint64_t (*)();
using rp_sample_xcc_fn = int (*)(int, double*, int);
using rp_sync_fn = int (*)(int timeout_us);
using rp_health_fn = int (*)(int dev, uint64_t* out, int n);

}  // namespace

void fill_counter_reading(const double* v, CounterReading* out) {
  out->ok = true;
  out->mfma_busy_pct = v[0];
  out->mfma_util_pct = v[10];
  out->sq_busy_pct = v[1];
  out->gui_active_pct = v[2];
  out->waves_per_s = v[3];
  out->lds_active_pct = v[4];
  out->lds_bank_conflict_pct = v[5];
  out->hbm_read_bps = v[6];
  out->hbm_write_bps = v[7];
  out->remote_read_bps = v[8];
  out->remote_write_bps = v[9];
  out->mfma_bf16_flops = v[11];
  out->mfma_fp8_flops = v[12];
  out->dispatch_stall_pct = v[13];
  out->lds_limited_pct = v[14];
  out->wave_limited_pct = v[15];
  out->vgpr_limited_pct = v[16];
  out->sgpr_limited_pct = v[17];
}

namespace {

class PluginCounters : public CounterSource {
 public:
  PluginCounters(std::string path, int window_ms, int interval_ms, bool continuous, bool inline_rounds)
      : path_(std::move(path)),
        window_ms_(window_ms),
        interval_ms_(interval_ms),
        continuous_(continuous),
        inline_(inline_rounds) {}
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
    using cont_fn = void (*)(int);
    auto cont = reinterpret_cast<cont_fn>(::dlsym(handle_, "gpuexp_rp_set_continuous"));
    if (continuous_ && cont) {
      // counting never stops; one read per engine tick (kick/sync), or every interval_ms
      // when no tick kicks (manual-tick engines)
      cont(interval_ms_);
      using inline_fn = void (*)(int);
      if (auto inl = reinterpret_cast<inline_fn>(::dlsym(handle_, "gpuexp_rp_set_inline"))) inl(inline_ ? 1 : 0);
      kick_ = reinterpret_cast<rp_kick_fn>(::dlsym(handle_, "gpuexp_rp_kick"));
      sync_ = reinterpret_cast<rp_sync_fn>(::dlsym(handle_, "gpuexp_rp_sync"));
    } else if (auto duty = reinterpret_cast<duty_fn>(::dlsym(handle_, "gpuexp_rp_set_duty"))) {
      duty(window_ms_, interval_ms_);
    }
    cpu_ = reinterpret_cast<rp_cpu_fn>(::dlsym(handle_, "gpuexp_rp_cpu_ns"));
    sample_xcc_ = reinterpret_cast<rp_sample_xcc_fn>(::dlsym(handle_, "gpuexp_rp_sample_xcc"));  // optional
    health_ = reinterpret_cast<rp_health_fn>(::dlsym(handle_, "gpuexp_rp_health"));  // optional
    // ABI: a BDF prefixed with '-' reserves that device's HSA agent (partition order) but
    // gets no queue.
    std::vector<std::string> names;
    for (auto& d : devs) names.push_back((d.queue_enabled ? "" : "-") + d.bdf);
    std::vector<const char*> bdfs;
    for (auto& n : names) bdfs.push_back(n.c_str());
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
    double v[kCounterOutputs];
    if (sample_(dev, dt_s, v) != 0) return false;
    fill_counter_reading(v, out);
    out->nxcc = sample_xcc_ ? std::max(0, sample_xcc_(dev, out->xcc_mfma_busy_pct, kMaxXcc)) : 0;
    return true;
  }

  int scope(int dev) override { return started_ && scope_fn_ ? scope_fn_(dev) : -1; }

  bool health(int dev, CounterHealth* out) override {
    uint64_t v[6] = {};
    if (!started_ || !health_ || health_(dev, v, 6) != 0) return false;
    out->stalls = v[0];
    out->resets = v[1];
    out->rearms = v[2];
    out->rescues = v[3];
    out->releases = v[4];
    out->rescue_active = v[5] != 0;
    return true;
  }

  void kick() override {
    if (started_ && kick_) kick_();
  }

  uint64_t cpu_ns() override { return started_ && cpu_ ? cpu_() : 0; }

  bool sync(int timeout_us) override { return !(started_ && sync_) || sync_(timeout_us) == 0; }

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
  bool continuous_;
  bool inline_;  // continuous: the engine's sampler runs each read round (gpuexp_rp_set_inline)
  rp_kick_fn kick_ = nullptr;
  rp_sync_fn sync_ = nullptr;
  rp_cpu_fn cpu_ = nullptr;
  rp_sample_xcc_fn sample_xcc_ = nullptr;
  rp_health_fn health_ = nullptr;
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

// Start time (field 22 of /proc/<pid>/stat) in clock ticks; 0 if the process is gone.
uint64_t proc_starttime(int pid) {
  std::string s;
  if (!read_small_file("/proc/" + std::to_string(pid) + "/stat", &s, 4096)) return 0;
  size_t p = s.rfind(')');
  if (p == std::string::npos) return 0;
  int field = 2;
  size_t i = p + 1;
  while (i < s.size()) {
    while (i < s.size() && s[i] == ' ') ++i;
    if (++field == 22) break;
    while (i < s.size() && s[i] != ' ') ++i;
  }
  return std::strtoull(s.c_str() + i, nullptr, 10);
}

// The identity /proc/<pid>/maps gives a mapped file: device major:minor and inode.
struct MapsId {
  unsigned long maj = 0, mn = 0;
  unsigned long long ino = 0;
  bool operator==(const MapsId& o) const { return maj == o.maj && mn == o.mn && ino == o.ino; }
};

// Reads a maps file whole; 0 ok, -1 unreadable for lack of access, -2 other failure.
int read_maps(const std::string& path, std::string* all) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return errno == EACCES || errno == EPERM ? -1 : -2;
  char buf[65536];
  for (;;) {
    ssize_t n = ::read(fd, buf, sizeof(buf));
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) {
      if (n < 0 && all->empty()) {
        const int err = errno;
        ::close(fd);
        return err == EACCES || err == EPERM ? -1 : -2;
      }
      break;
    }
    all->append(buf, size_t(n));
  }
  ::close(fd);
  return 0;
}

// Calls fn(start address, identity) for each file-backed line of a maps text until fn
// returns true; returns whether it did.
template <class F>
bool scan_maps(const std::string& all, F fn) {
  size_t i = 0;
  while (i < all.size()) {
    size_t e = all.find('\n', i);
    if (e == std::string::npos) e = all.size();
    // address perms offset dev inode [path]
    const char* p = all.c_str() + i;
    const char* end = all.c_str() + e;
    int f = 0;
    const char* tok[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    while (p < end && f < 5) {
      while (p < end && *p == ' ') ++p;
      tok[f++] = p;
      while (p < end && *p != ' ') ++p;
    }
    if (f == 5) {
      char* q = nullptr;
      MapsId id;
      id.maj = std::strtoul(tok[3], &q, 16);
      if (q && *q == ':') {
        id.mn = std::strtoul(q + 1, nullptr, 16);
        id.ino = std::strtoull(tok[4], nullptr, 10);
        if (id.ino && fn(std::strtoull(tok[0], nullptr, 16), id)) return true;
      }
    }
    i = e + 1;
  }
  return false;
}

// The identity /proc/<pid>/maps shows for a mapping of `fd`'s file.  It is not always
// fstat()'s: on overlayfs (a container's /tmp) maps names the backing upper file's device,
// fstat() the overlay's (MI355X gpurun box: 00:d1 vs 00:d2, same inode).  So the exporter
// maps one page of the file itself — read-only and never touched, so a writer truncating
// it cannot fault us — and reads its own mapping's line.  Falls back to fstat().
MapsId maps_identity(int fd, const struct stat& st) {
  MapsId id;
  id.maj = major(st.st_dev);
  id.mn = minor(st.st_dev);
  id.ino = (unsigned long long)st.st_ino;
  void* p = ::mmap(nullptr, 4096, PROT_READ, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) return id;
  std::string all;
  if (read_maps("/proc/self/maps", &all) == 0) {
    const unsigned long long want = (unsigned long long)(uintptr_t)p;
    scan_maps(all, [&](unsigned long long start, const MapsId& m) {
      if (start != want) return false;
      id = m;
      return true;
    });
  }
  ::munmap(p, 4096);
  return id;
}

// True if /proc/<pid>/maps has a mapping of the file with exactly this identity: proof
// that `pid` is the process that writes it (the tracer keeps its counters file mapped for
// its whole life).  -1 if the maps file is unreadable (no ptrace-read access to that process).
int maps_file(int pid, const MapsId& want) {
  std::string all;
  const int rc = read_maps("/proc/" + std::to_string(pid) + "/maps", &all);
  if (rc != 0) return rc == -1 ? -1 : 0;
  return scan_maps(all, [&](unsigned long long, const MapsId& m) { return m == want; }) ? 1 : 0;
}

// Reads the RCCL tracer's counter files from a directory that every workload pod can
// write to (a hostPath), so nothing in them is trusted:
//  - files are opened O_NOFOLLOW|O_NONBLOCK and must be regular (no FIFO can block the
//    sampler, no symlink can point elsewhere), and are copied with pread() every poll (a
//    writer truncating its file cannot fault the exporter, as a live mapping would);
//  - the name must agree with the identity inside, and the identity must name a process
//    that maps this very file (/proc/<pid>/maps dev:inode), in the PID namespace it
//    claims — a pod cannot get its counters attributed to another pod's process;
//  - the writer's liveness is checked every poll (pidfd, else start time): a file left by
//    a killed process stops being exported at once and never moves to a reused PID.
// Cost is bounded whatever the directory holds (a pod can fill it):
//  - the directory is listed only when its mtime changed, and then at most once per
//    `scan_interval` (1 s default); a tick otherwise touches only the files already proven
//    active (one fstatat, two preads and a pidfd poll each);
//  - at most kMaxTracked names are tracked; everything else (names that are not tracer
//    files, non-regular entries, names over the cap) is only counted, as "ignored";
//  - a file whose writer is unproven is retried with a doubling backoff (1 s .. 64 s); one
//    whose writer exited is re-examined only when its inode, size or mtime changes (a new
//    writer re-creating it), never on a timer;
//  - /proc is walked at most once per listing, into one (pidns, nspid) -> pid map that
//    every identification of that listing shares.
class ShmRcclSource : public RcclSource {
 public:
  static constexpr size_t kMaxTracked = 1024;

  ShmRcclSource(std::string dir, bool verify_maps, uint64_t scan_interval_ns)
      : dir_(std::move(dir)), verify_maps_(verify_maps), scan_interval_ns_(scan_interval_ns) {
    self_ns_ = pidns_inode("/proc/self");
  }
  ~ShmRcclSource() override {
    for (auto& kv : files_) close_entry(&kv.second);
    if (dfd_ >= 0) ::close(dfd_);
  }

  void poll(std::vector<RcclTotals>* out) override {
    out->clear();
    const uint64_t now = mono_ns();
    if (dfd_ < 0) {
      dfd_ = ::open(dir_.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
      if (dfd_ < 0) {
        for (auto& kv : files_) close_entry(&kv.second);
        files_.clear();
        return;
      }
      scanned_ = false;
    }
    struct stat dst;
    if (::fstat(dfd_, &dst) != 0 || dst.st_nlink == 0) {  // directory removed: reopen next poll
      ::close(dfd_);
      dfd_ = -1;
      return;
    }
    const bool changed = !scanned_ || dst.st_mtim.tv_sec != dir_mtime_.tv_sec ||
                         dst.st_mtim.tv_nsec != dir_mtime_.tv_nsec;
    // a listing when the directory changed (rate-limited) or a retry is due
    if ((changed || (next_retry_ns_ && now >= next_retry_ns_)) && (!scanned_ || now - last_scan_ns_ >= scan_interval_ns_)) {
      dir_mtime_ = dst.st_mtim;
      scan(now);
    }
    for (auto& kv : files_) {
      Entry& e = kv.second;
      if (e.state != kActive || e.fd < 0) continue;
      struct stat st;
      if (::fstatat(dfd_, kv.first.c_str(), &st, AT_SYMLINK_NOFOLLOW) != 0 || st.st_dev != e.dev ||
          st.st_ino != e.ino) {
        close_entry(&e);  // unlinked or replaced: the next listing sees what is there now
        e.state = kNew;
        continue;
      }
      RcclShmFile snap;
      if (!read_consistent(e.fd, &snap) || snap.magic != kRcclShmMagic || snap.pidns_ino != e.name_ino ||
          snap.ns_pid != e.name_pid)
        continue;  // truncated or rewritten under us: nothing to export this tick
      if (!alive(&e)) {
        mark_exited(&e, st);
        continue;
      }
      for (int op = 0; op < kOpNumOps; ++op) {
        const uint64_t c = snap.ops[op].calls.load(std::memory_order_relaxed);
        if (!c) continue;
        RcclTotals t;
        t.pid = e.host_pid;
        t.op = rccl_op_name(op);
        t.calls = c;
        t.bytes = snap.ops[op].bytes.load(std::memory_order_relaxed);
        t.rank = snap.rank;
        t.nranks = snap.nranks;
        out->push_back(t);
      }
    }
  }

  void file_states(int* active, int* unverified, int* exited) const override {
    *active = *unverified = *exited = 0;
    for (const auto& kv : files_) {
      if (kv.second.state == kActive) ++*active;
      else if (kv.second.state == kExited) ++*exited;
      else if (kv.second.state == kUnverified) ++*unverified;
    }
  }

  int ignored() const override { return ignored_; }
  uint64_t scans() const override { return scans_; }

 private:
  enum State { kNew, kActive, kUnverified, kExited };
  struct Entry {
    int fd = -1;
    dev_t dev = 0;
    ino_t ino = 0;
    uint64_t name_ino = 0;  // identity the name claims
    int name_pid = 0;
    MapsId maps_id;  // how /proc/<pid>/maps names this file (see maps_identity)
    int host_pid = -1;
    int pidfd = -1;
    uint64_t starttime = 0;
    uint64_t retry_ns = 0;
    int fails = 0;
    State state = kNew;
    // kExited: the file as it was when its writer was found gone
    ino_t gone_ino = 0;
    off_t gone_size = 0;
    struct timespec gone_mtime {};
  };
  using ProcMap = std::map<std::pair<uint64_t, int>, std::vector<int>>;  // (pidns, nspid) -> host pids

  static bool parse_name(const std::string& name, uint64_t* ino, int* pid) {
    static const char kPrefix[] = "gpuexp-rccl-";
    if (name.compare(0, sizeof(kPrefix) - 1, kPrefix) != 0) return false;
    const char* p = name.c_str() + sizeof(kPrefix) - 1;
    char* q = nullptr;
    if (*p < '0' || *p > '9') return false;
    *ino = std::strtoull(p, &q, 10);
    if (!q || *q != '-' || q[1] < '0' || q[1] > '9') return false;
    char* r = nullptr;
    long v = std::strtol(q + 1, &r, 10);
    if (!r || *r != '\0' || v <= 0 || v > (1 << 30)) return false;
    *pid = int(v);
    return true;
  }

  // One listing: new names are examined (capped), gone names forgotten, exited files
  // re-examined only if they changed, unverified ones when their backoff expires.
  void scan(uint64_t now) {
    last_scan_ns_ = now;
    scanned_ = true;
    ++scans_;
    int ignored = 0;
    next_retry_ns_ = 0;
    std::unordered_map<std::string, bool> present;
    std::unique_ptr<ProcMap> procs;  // built on first need, shared by this listing
    const int lfd = ::dup(dfd_);
    DIR* d = lfd >= 0 ? ::fdopendir(lfd) : nullptr;
    if (!d) {
      if (lfd >= 0) ::close(lfd);
      return;
    }
    ::rewinddir(d);
    while (dirent* de = ::readdir(d)) {
      if (de->d_name[0] == '.') continue;
      const std::string name(de->d_name);
      uint64_t name_ino = 0;
      int name_pid = 0;
      if (!parse_name(name, &name_ino, &name_pid)) {
        ++ignored;  // not a tracer file: no syscall spent on it
        continue;
      }
      auto it = files_.find(name);
      if (it == files_.end() && files_.size() >= kMaxTracked) {
        ++ignored;
        continue;
      }
      if (it != files_.end() && it->second.state == kActive && it->second.fd >= 0) {
        present[name] = true;  // checked every tick
        continue;
      }
      struct stat st;
      if (::fstatat(dfd_, name.c_str(), &st, AT_SYMLINK_NOFOLLOW) != 0 || !S_ISREG(st.st_mode)) {
        ++ignored;  // FIFO, symlink, directory, ...: never opened
        if (it != files_.end()) {
          close_entry(&it->second);
          files_.erase(it);
        }
        continue;
      }
      present[name] = true;
      Entry& e = it != files_.end() ? it->second : files_[name];
      e.name_ino = name_ino;
      e.name_pid = name_pid;
      if (e.state == kExited) {
        if (st.st_ino == e.gone_ino && st.st_size == e.gone_size && st.st_mtim.tv_sec == e.gone_mtime.tv_sec &&
            st.st_mtim.tv_nsec == e.gone_mtime.tv_nsec)
          continue;  // same leftover file: nothing new to prove
        // it changed (a new writer re-creating the name?): examine once, and not again
        // until it changes again
        e.gone_ino = st.st_ino;
        e.gone_size = st.st_size;
        e.gone_mtime = st.st_mtim;
      }
      if (e.state == kUnverified && now < e.retry_ns) {
        note_retry(e.retry_ns);
        continue;
      }
      examine(name, &e, now, &procs);
    }
    ::closedir(d);
    ignored_ = ignored;
    for (auto it = files_.begin(); it != files_.end();) {
      if (!present.count(it->first)) {
        close_entry(&it->second);
        it = files_.erase(it);
      } else {
        ++it;
      }
    }
  }

  // Opens a tracer file, checks its content against its name and proves its writer.
  void examine(const std::string& name, Entry* e, uint64_t now, std::unique_ptr<ProcMap>* procs) {
    close_entry(e);
    e->fd = ::openat(dfd_, name.c_str(), O_RDONLY | O_NOFOLLOW | O_NONBLOCK | O_CLOEXEC);
    struct stat fst;
    if (e->fd < 0 || ::fstat(e->fd, &fst) != 0 || !S_ISREG(fst.st_mode)) {
      close_entry(e);
      unverified(e, now);
      return;
    }
    e->dev = fst.st_dev;
    e->ino = fst.st_ino;
    RcclShmFile snap;
    if (!read_consistent(e->fd, &snap) || snap.magic != kRcclShmMagic || snap.pidns_ino != e->name_ino ||
        snap.ns_pid != e->name_pid || snap.pidns_ino == 0 || snap.ns_pid <= 0) {
      // not (yet) a complete file, or one whose content disagrees with its name
      close_entry(e);
      unverified(e, now);
      return;
    }
    e->maps_id = maps_identity(e->fd, fst);
    if (!identify(e, snap.pidns_ino, snap.ns_pid, procs)) {
      close_entry(e);  // no fd for a file nobody is proven to write
      unverified(e, now);
      return;
    }
    e->state = kActive;
    e->fails = 0;
  }

  void unverified(Entry* e, uint64_t now) {
    if (e->state == kExited) return;  // re-examined when the file changes, not on a timer
    e->state = kUnverified;
    const int f = std::min(e->fails, 6);
    e->retry_ns = now + (1000000000ull << f);  // 1 s .. 64 s
    e->fails += 1;
    note_retry(e->retry_ns);
  }

  void note_retry(uint64_t t) {
    if (!next_retry_ns_ || t < next_retry_ns_) next_retry_ns_ = t;
  }

  void mark_exited(Entry* e, const struct stat& st) {
    close_entry(e);  // writer exited (or was killed): its leftover file is not exported
    e->state = kExited;
    e->fails = 0;
    e->gone_ino = st.st_ino;
    e->gone_size = st.st_size;
    e->gone_mtime = st.st_mtim;
  }

  // Two identical preads: the writer updates the counters with relaxed atomics while we
  // copy, so a torn 64-bit value could look like a counter reset.  Returns false on a
  // short file (truncated, or not written yet) or when it never settles.
  static bool read_consistent(int fd, RcclShmFile* out) {
    alignas(RcclShmFile) unsigned char a[sizeof(RcclShmFile)], b[sizeof(RcclShmFile)];
    if (::pread(fd, a, sizeof(a), 0) != ssize_t(sizeof(a))) return false;
    for (int attempt = 0; attempt < 4; ++attempt) {
      if (::pread(fd, b, sizeof(b), 0) != ssize_t(sizeof(b))) return false;
      if (std::memcmp(a, b, sizeof(a)) == 0) {
        std::memcpy(static_cast<void*>(out), b, sizeof(b));
        return true;
      }
      std::memcpy(a, b, sizeof(a));
    }
    return false;
  }

  void release_owner(Entry* e) {
    if (e->pidfd >= 0) ::close(e->pidfd);
    e->pidfd = -1;
    e->host_pid = -1;
    e->starttime = 0;
  }

  void close_entry(Entry* e) {
    release_owner(e);
    if (e->fd >= 0) ::close(e->fd);
    e->fd = -1;
  }

  bool alive(Entry* e) {
    if (e->pidfd >= 0) {
      pollfd p{e->pidfd, POLLIN, 0};
      return ::poll(&p, 1, 0) == 0;  // a pidfd turns readable when its process exits
    }
    return proc_starttime(e->host_pid) == e->starttime;
  }

  static std::unique_ptr<ProcMap> build_proc_map() {
    auto m = std::make_unique<ProcMap>();
    for (const std::string& d : list_dir("/proc")) {
      if (d.empty() || d[0] < '1' || d[0] > '9') continue;
      const std::string pd = "/proc/" + d;
      const uint64_t ns = pidns_inode(pd);
      const int nspid = ns ? innermost_nspid(pd) : -1;
      if (nspid > 0) (*m)[{ns, nspid}].push_back(std::atoi(d.c_str()));
    }
    return m;
  }

  // Finds the host PID of (ns_ino, ns_pid) and proves it is this file's writer.
  bool identify(Entry* e, uint64_t ns_ino, int ns_pid, std::unique_ptr<ProcMap>* procs) {
    std::vector<int> cands;
    if (ns_ino == self_ns_) {
      cands.push_back(ns_pid);
    } else {
      if (!*procs) *procs = build_proc_map();
      auto it = (*procs)->find({ns_ino, ns_pid});
      if (it != (*procs)->end()) cands = it->second;
    }
    for (int pid : cands) {
      // Pin the process first, then check it, then check the pin still holds: no PID
      // reuse can slip between the check and the export.
      int pfd = int(::syscall(SYS_pidfd_open, pid, 0));
      const uint64_t st0 = proc_starttime(pid);
      if (!st0) {
        if (pfd >= 0) ::close(pfd);
        continue;
      }
      const std::string pd = "/proc/" + std::to_string(pid);
      bool ok = pidns_inode(pd) == ns_ino && innermost_nspid(pd) == ns_pid;
      if (ok && verify_maps_) {
        const int m = maps_file(pid, e->maps_id);
        if (m < 0 && !warned_maps_) {
          warned_maps_ = true;
          GPUEXP_LOG(LogLevel::kWarn, "rccl",
                     "cannot read /proc/" + std::to_string(pid) +
                         "/maps (needs ptrace-read access): RCCL counter files stay unattributed");
        }
        ok = m == 1;
      }
      if (ok) {
        if (pfd >= 0) {
          pollfd p{pfd, POLLIN, 0};
          ok = ::poll(&p, 1, 0) == 0;
        } else {
          ok = proc_starttime(pid) == st0;
        }
      }
      if (!ok) {
        if (pfd >= 0) ::close(pfd);
        continue;
      }
      e->host_pid = pid;
      e->pidfd = pfd;
      e->starttime = st0;
      return true;
    }
    return false;
  }

  std::string dir_;
  bool verify_maps_;
  uint64_t scan_interval_ns_;
  bool warned_maps_ = false;
  uint64_t self_ns_ = 0;
  int dfd_ = -1;
  bool scanned_ = false;
  struct timespec dir_mtime_ {};
  uint64_t last_scan_ns_ = 0, next_retry_ns_ = 0, scans_ = 0;
  int ignored_ = 0;
  std::unordered_map<std::string, Entry> files_;
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
                                                     int interval_ms, bool continuous, bool inline_rounds) {
  return std::make_unique<PluginCounters>(plugin_path, window_ms, interval_ms, continuous, inline_rounds);
}

std::unique_ptr<RcclSource> make_rccl_source(const std::string& dir, bool verify_maps, double scan_interval_s) {
  return std::make_unique<ShmRcclSource>(dir, verify_maps, uint64_t(std::max(0.0, scan_interval_s) * 1e9));
}

}  // namespace gpuexp
