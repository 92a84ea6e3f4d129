#include "gpuexp/procs.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <unordered_set>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

namespace gpuexp {

KfdProcReader::KfdProcReader(std::string host_root, int self_pid, bool read_cu_occupancy,
                             uint64_t detail_interval_ns, uint64_t rescan_interval_ns, bool read_sdma)
    : root_(std::move(host_root)), self_(self_pid), read_cu_(read_cu_occupancy), read_sdma_(read_sdma),
      detail_every_ns_(detail_interval_ns), rescan_ns_(rescan_interval_ns) {
  if (!root_.empty() && root_.back() == '/') root_.pop_back();
}

KfdProcReader::~KfdProcReader() {
  if (dir_fd_ >= 0) ::close(dir_fd_);
}

void KfdProcReader::scan(const std::vector<DeviceInfo>& devs,
                         std::vector<std::vector<ProcSample>>* per_dev, uint64_t now_ns, bool defer_listing) {
  per_dev->resize(devs.size());
  for (auto& l : *per_dev) l.clear();
  ++scan_no_;
  const std::string base = root_ + "/sys/class/kfd/kfd/proc";
  // The directory listing is the scan's most expensive step (a cold getdents: ~20 us on
  // MI355X sysfs, profiles/r03/read_costs.txt, more on a busy host) and new GPU processes are
  // rare: list when the directory's mtime moved (kernfs stamps it on add/remove where it
  // keeps attributes), at least every rescan_ns, and whenever a tracked process vanished;
  // in between, read the tracked processes' files only (an exited process's reads fail).
  struct stat sb {};
  if (dir_fd_ < 0) {
    // no KFD proc directory (a node without the driver, the mock): a failed open is retried at
    // the rescan interval, not every tick
    if (open_tried_ns_ && now_ns && rescan_ns_ && now_ns >= open_tried_ns_ && now_ns - open_tried_ns_ < rescan_ns_)
      return;
    dir_fd_ = ::open(base.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    open_tried_ns_ = dir_fd_ < 0 ? now_ns : 0;
    if (dir_fd_ < 0 && now_ns && rescan_ns_) {
      pids_.clear();  // (the directory went away: nothing tracked is readable)
      return;
    }
  }
  bool have_mtime = dir_fd_ >= 0 && ::fstat(dir_fd_, &sb) == 0;
  if (have_mtime && sb.st_nlink == 0) {  // the directory itself was removed (KFD reloaded): reopen
    ::close(dir_fd_);
    dir_fd_ = ::open(base.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    have_mtime = dir_fd_ >= 0 && ::fstat(dir_fd_, &sb) == 0;
  }
  const bool moved = have_mtime && (sb.st_mtim.tv_sec != mtime_.tv_sec || sb.st_mtim.tv_nsec != mtime_.tv_nsec);
  if (have_mtime) mtime_ = sb.st_mtim;
  // (a rescan-timer listing may wait while the engine levels a heavy tick, at most to twice the
  // interval; a moved mtime or a vanished process lists at once)
  const bool timer_due = now_ns - last_list_ns_ >= rescan_ns_ &&
                         !(defer_listing && now_ns - last_list_ns_ < 2 * rescan_ns_);
  const bool list = !now_ns || !rescan_ns_ || moved || relist_ || timer_due || now_ns < last_list_ns_;
  deferred_ = !list && defer_listing && now_ns - last_list_ns_ >= rescan_ns_;
  if (!list) {
    for (auto it = pids_.begin(); it != pids_.end();) {
      if (emit(it->second, it->first, per_dev, now_ns) == 0 && !it->second.devs.empty()) {
        relist_ = true;  // gone (or its PID reused): the next tick lists the directory again
        it = pids_.erase(it);
        continue;
      }
      ++it;
    }
    return;
  }
  relist_ = false;
  last_list_ns_ = now_ns;
  ++lists_;
  // A full listing also checks that dir_fd_ is still the directory at `base`: after a KFD
  // reload the kept fd names the dead node, whose mtime never moves again.  st_nlink == 0 (above)
  // catches that on tmpfs, never on sysfs (kernfs reports a directory's nlink as subdirs + 2),
  // so compare identities: one stat per listing (at most every rescan_ns on a quiet node).
  struct stat ps {};
  if (::stat(base.c_str(), &ps) == 0 &&
      (dir_fd_ < 0 || !have_mtime || ps.st_ino != sb.st_ino || ps.st_dev != sb.st_dev)) {
    if (dir_fd_ >= 0) ::close(dir_fd_);
    dir_fd_ = ::open(base.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    if (dir_fd_ >= 0 && ::fstat(dir_fd_, &sb) == 0) mtime_ = sb.st_mtim;
    ++dir_reopens_;
  }
  // Opens device `di`'s files of a process directory; false if it has no context there (yet).
  auto open_dev = [&](const std::string& pdir, size_t di, PerDev* pd) {
    const DeviceInfo& d = devs[di];
    pd->dev = int(di);  // position in `devs` (the engine's device order)
    const std::string id = std::to_string(d.kfd_gpu_id);
    if (!pd->vram.open(pdir + "/vram_" + id)) return false;
    if (read_cu_) pd->cu.open(pdir + "/stats_" + id + "/cu_occupancy");
    if (read_sdma_) pd->sdma.open(pdir + "/sdma_" + id);
    pd->evicted.open(pdir + "/stats_" + id + "/evicted_ms");
    return true;
  };
  // Opens the files of every device in `devs` the process has a vram_<gpu_id> file for and `e`
  // does not track yet: one listing of the process directory, not an open per device (a
  // process on 1 of 8 GPUs cost 7 failed path lookups per look, ~40 us per tick at 10 Hz for
  // 32 processes on a fake 8-GPU node).
  auto probe_devs = [&](const std::string& pdir, Entry* e) {
    for (const std::string& f : list_dir(pdir)) {
      if (f.compare(0, 5, "vram_") != 0) continue;
      const uint64_t id = std::strtoull(f.c_str() + 5, nullptr, 10);
      for (size_t di = 0; di < devs.size(); ++di) {
        if (devs[di].kfd_gpu_id != id) continue;
        bool have = false;
        for (const PerDev& pd : e->devs) have = have || pd.dev == int(di);
        PerDev pd;
        if (!have && open_dev(pdir, di, &pd)) e->devs.push_back(std::move(pd));
      }
    }
    // the engine's device order, whatever order the directory listed them in
    std::sort(e->devs.begin(), e->devs.end(), [](const PerDev& a, const PerDev& b) { return a.dev < b.dev; });
  };
  for (const std::string& name : list_dir(base)) {
    int pid = std::atoi(name.c_str());
    if (pid <= 0 || pid == self_) continue;
    const std::string pdir = base + "/" + name;
    auto make_entry = [&]() {
      // New process: find which of OUR devices it has a KFD context on.
      Entry e;
      probe_devs(pdir, &e);
      std::string comm;
      if (read_small_file(root_ + "/proc/" + name + "/comm", &comm, 64)) e.comm = trim(comm);
      e.id = ++next_id_;
      // each process at its own phase of the re-probe period: processes one listing found
      // would otherwise list their directories on the same tick every few seconds (32 listings
      // on one tick at 8 GPUs x 4 processes, the heaviest tick of a 10 Hz sampler)
      const uint64_t phase = (e.id * 0x9E3779B97F4A7C15ull >> 24) % kReprobeNs;
      e.probe_ns = now_ns > phase ? now_ns - phase : now_ns;
      return pids_.insert_or_assign(pid, std::move(e)).first;
    };
    auto it = pids_.find(pid);
    const bool fresh = it == pids_.end();
    if (fresh) {
      it = make_entry();
    } else if (it->second.comm.empty() && it->second.comm_tries < kCommTries) {
      // comm unreadable when the process was found (mid-exec, or /proc lagging KFD): retry
      // at the next few listings instead of keeping comm="" for the process's lifetime
      ++it->second.comm_tries;
      std::string comm;
      if (read_small_file(root_ + "/proc/" + name + "/comm", &comm, 64)) it->second.comm = trim(comm);
    }
    if (!fresh && it->second.devs.size() < devs.size() &&
        (!now_ns || now_ns < it->second.probe_ns || now_ns - it->second.probe_ns >= it->second.probe_every_ns)) {
      // KFD adds a process's vram_<gpu_id> when it first uses that GPU, which can be after its
      // directory appeared (or after the listing that found it, mid-creation): look for the
      // GPUs it had no files for at a listing every kReprobeNs, or it would never show on them
      // (one listing of its directory per look).
      // (a process on 1 of 8 GPUs stays there, as a rule: the look backs off to every kReprobeMaxNs
      // while it finds nothing, and is back to every kReprobeNs once it found a GPU)
      it->second.probe_ns = now_ns;
      const size_t had = it->second.devs.size();
      probe_devs(pdir, &it->second);
      it->second.probe_every_ns =
          it->second.devs.size() > had ? kReprobeNs : std::min(kReprobeMaxNs, 2 * it->second.probe_every_ns);
    }
    if (emit(it->second, pid, per_dev, now_ns) == 0 && !fresh && !it->second.devs.empty()) {
      // Cached fds of a PID whose KFD directory was removed and re-created between two
      // scans (the PID was reused) point at dead kobjects: every read fails although
      // the directory exists.  Reopen once, so the new process (and its comm) shows.
      it = make_entry();
      emit(it->second, pid, per_dev, now_ns);
    }
  }
  // Forget processes that left the KFD proc directory (closes their fds).
  for (auto it = pids_.begin(); it != pids_.end();)
    it = it->second.seen != scan_no_ ? pids_.erase(it) : std::next(it);
}

int KfdProcReader::emit(Entry& e, int pid, std::vector<std::vector<ProcSample>>* per_dev, uint64_t now_ns) {
  char buf[128];
  int ok = 0;
  e.seen = scan_no_;
  for (auto& pd : e.devs) {
    {
      uint64_t v = 0;
      if (!pd.vram.read_u64(&v)) continue;  // process exiting
      ++ok;
      ProcSample ps;
      ps.pid = pid;
      ps.device = pd.dev;
      ps.vram_bytes = double(v);
      if (!pd.detail_read || !now_ns || detail_every_ns_ == 0 || now_ns - pd.detail_ns >= detail_every_ns_) {
        long n;
        if (pd.cu.is_open() && (n = pd.cu.read(buf, sizeof(buf) - 1)) > 0 && parse_u64(buf, size_t(n), &v))
          pd.cu_last = double(v);
        if (pd.sdma.is_open() && (n = pd.sdma.read(buf, sizeof(buf) - 1)) > 0 && parse_u64(buf, size_t(n), &v))
          pd.sdma_last = double(v);
        if (pd.evicted.is_open() && (n = pd.evicted.read(buf, sizeof(buf) - 1)) > 0 &&
            parse_u64(buf, size_t(n), &v))
          pd.evicted_last = double(v);
        // After the first read, each (process, GPU) keeps its own phase of detail_every_ns_:
        // processes found by one listing would otherwise read their details on the same tick
        // forever (64 more reads every 10th tick at 8 GPUs x 4 processes and 10 Hz).
        const uint64_t phase = pd.detail_read || !now_ns || detail_every_ns_ == 0
                                   ? 0
                                   : ((e.id * 0x9E3779B97F4A7C15ull + uint64_t(pd.dev)) >> 20) % detail_every_ns_;
        pd.detail_ns = now_ns >= phase ? now_ns - phase : now_ns;
        pd.detail_read = true;
      }
      ps.cu_occupancy = pd.cu_last;
      ps.sdma_us = pd.sdma_last;
      ps.evicted_ms = pd.evicted_last;
      ps.name = e.comm;
      ps.kfd_id = e.id;
      (*per_dev)[size_t(pd.dev)].push_back(ps);
    }
  }
  return ok;
}

// ---------------------------------------------------------------------------------
// cgroup path parsing

namespace {

bool is_uid_char(char c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F') || c == '-' ||
         c == '_';
}

bool is_hex(const std::string& s) {
  if (s.empty()) return false;
  for (char c : s)
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
  return true;
}

std::vector<std::string> split_path(const std::string& p) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i <= p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    if (j > i) out.push_back(p.substr(i, j - i));
    i = j + 1;
  }
  return out;
}

// Finds "pod<36-char uid>" inside a component; returns the dashed uid.
bool extract_pod_uid(const std::string& comp, std::string* uid) {
  size_t pos = 0;
  while ((pos = comp.find("pod", pos)) != std::string::npos) {
    size_t s = pos + 3;
    size_t e = s;
    while (e < comp.size() && is_uid_char(comp[e])) ++e;
    if (e - s == 36) {
      std::string u = comp.substr(s, 36);
      std::replace(u.begin(), u.end(), '_', '-');
      std::transform(u.begin(), u.end(), u.begin(), ::tolower);
      // 8-4-4-4-12
      if (u[8] == '-' && u[13] == '-' && u[18] == '-' && u[23] == '-') {
        *uid = u;
        return true;
      }
    }
    pos = s;
  }
  return false;
}

bool strip_prefix(std::string* s, const char* p) {
  size_t n = std::strlen(p);
  if (s->compare(0, n, p) == 0) {
    s->erase(0, n);
    return true;
  }
  return false;
}

bool strip_suffix(std::string* s, const char* p) {
  size_t n = std::strlen(p);
  if (s->size() >= n && s->compare(s->size() - n, n, p) == 0) {
    s->erase(s->size() - n);
    return true;
  }
  return false;
}

// Container component forms: cri-containerd-<id>.scope, crio-<id>.scope,
// docker-<id>.scope, <id> (cgroupfs), ...:cri-containerd:<id>.
bool extract_container(std::string comp, std::string* id, std::string* runtime) {
  size_t colon = comp.rfind(':');
  if (colon != std::string::npos) {
    std::string rt = comp.substr(0, colon);
    comp = comp.substr(colon + 1);
    if (rt.find("containerd") != std::string::npos) *runtime = "containerd";
    else if (rt.find("crio") != std::string::npos) *runtime = "crio";
    else if (rt.find("docker") != std::string::npos) *runtime = "docker";
  }
  strip_suffix(&comp, ".scope");
  if (strip_prefix(&comp, "cri-containerd-")) *runtime = "containerd";
  else if (strip_prefix(&comp, "crio-conmon-")) return false;  // conmon, not a container
  else if (strip_prefix(&comp, "crio-")) *runtime = "crio";
  else if (strip_prefix(&comp, "docker-")) *runtime = "docker";
  else if (strip_prefix(&comp, "containerd-")) *runtime = "containerd";
  std::transform(comp.begin(), comp.end(), comp.begin(), ::tolower);
  if (comp.size() >= 12 && is_hex(comp)) {
    *id = comp;
    if (runtime->empty()) *runtime = "unknown";
    return true;
  }
  return false;
}

}  // namespace

bool parse_kube_cgroup_path(const std::string& path, CgroupInfo* out) {
  *out = CgroupInfo();
  out->path = path;
  auto comps = split_path(path);
  int pod_idx = -1;
  for (size_t i = 0; i < comps.size(); ++i) {
    std::string uid;
    if (comps[i].find("kubepods") != std::string::npos || comps[i].compare(0, 3, "pod") == 0) {
      if (extract_pod_uid(comps[i], &uid)) {
        out->pod_uid = uid;
        pod_idx = int(i);
      }
    }
  }
  if (pod_idx < 0) return false;
  out->kube = true;
  out->qos = "guaranteed";
  for (int i = 0; i <= pod_idx; ++i) {
    if (comps[size_t(i)].find("burstable") != std::string::npos) out->qos = "burstable";
    if (comps[size_t(i)].find("besteffort") != std::string::npos) out->qos = "besteffort";
  }
  for (size_t i = size_t(pod_idx) + 1; i < comps.size(); ++i) {
    std::string id, rt;
    if (extract_container(comps[i], &id, &rt)) {
      out->container_id = id;
      out->runtime = rt;
      break;
    }
  }
  // Some runtimes put the pod and container in ONE component ("...pod<uid>.slice:cri-containerd:<id>").
  if (out->container_id.empty()) {
    std::string id, rt;
    if (extract_container(comps[size_t(pod_idx)], &id, &rt)) {
      out->container_id = id;
      out->runtime = rt;
    }
  }
  return true;
}

bool parse_proc_cgroup(const std::string& content, CgroupInfo* out) {
  // Prefer the unified (v2) hierarchy; otherwise any v1 controller line that names a pod.
  std::string v2;
  std::vector<std::string> v1;
  size_t i = 0;
  while (i < content.size()) {
    size_t e = content.find('\n', i);
    if (e == std::string::npos) e = content.size();
    std::string line = content.substr(i, e - i);
    i = e + 1;
    size_t c1 = line.find(':');
    if (c1 == std::string::npos) continue;
    size_t c2 = line.find(':', c1 + 1);
    if (c2 == std::string::npos) continue;
    std::string hier = line.substr(0, c1), ctrl = line.substr(c1 + 1, c2 - c1 - 1);
    std::string path = line.substr(c2 + 1);
    if (hier == "0" && ctrl.empty()) v2 = path;
    else v1.push_back(path);
  }
  if (!v2.empty() && parse_kube_cgroup_path(v2, out)) return true;
  for (auto& p : v1)
    if (parse_kube_cgroup_path(p, out)) return true;
  *out = CgroupInfo();
  out->path = v2.empty() && !v1.empty() ? v1.front() : v2;
  return false;
}

PidResolver::PidResolver(std::string host_root) : root_(std::move(host_root)) {
  if (!root_.empty() && root_.back() == '/') root_.pop_back();
}

bool PidResolver::read_starttime(int pid, uint64_t* st) {
  std::string s;
  if (!read_small_file(root_ + "/proc/" + std::to_string(pid) + "/stat", &s, 4096)) return false;
  // Field 22 (starttime), counted after the ")" that ends comm.
  size_t p = s.rfind(')');
  if (p == std::string::npos) return false;
  int field = 2;
  size_t i = p + 1;
  while (i < s.size() && field < 22) {
    while (i < s.size() && s[i] == ' ') ++i;
    ++field;
    if (field == 22) break;
    while (i < s.size() && s[i] != ' ') ++i;
  }
  return parse_u64(s.c_str() + i, s.size() - i, st);
}

const CgroupInfo* PidResolver::resolve(int pid, uint64_t kfd_id) {
  auto ov = overrides_.find(pid);
  if (ov != overrides_.end()) {
    Entry& e = cache_[pid];
    if (e.info.path != ov->second || !e.ok) {
      e.ok = true;
      parse_kube_cgroup_path(ov->second, &e.info);
      e.info.path = ov->second;
    }
    return &e.info;
  }
  auto it = cache_.find(pid);
  if (it != cache_.end() && !it->second.ok) {  // failed before: not again this tick or for a while
    const Entry& e = it->second;
    if (e.epoch == epoch_ || (now_ns_ >= e.failed_ns && now_ns_ - e.failed_ns < kRetryFailedNs)) return nullptr;
  }
  if (it != cache_.end() && it->second.ok) {
    Entry& e = it->second;
    if (e.epoch == epoch_) return &e.info;  // already checked this tick
    if (kfd_id && e.kfd_id == kfd_id) {     // KFD read this same process this tick
      e.epoch = epoch_;
      return &e.info;
    }
    char b[32];
    const bool alive = !e.comm || e.comm->read(b, sizeof(b)) > 0;
    if (alive && now_ns_ >= e.st_checked_ns && now_ns_ - e.st_checked_ns < kStarttimeEveryNs) {
      e.epoch = epoch_;
      if (kfd_id) e.kfd_id = kfd_id;
      return &e.info;
    }
    uint64_t st = 0;
    const bool have_st = read_starttime(pid, &st);
    if (!have_st || e.starttime == st) {
      // Same process (its start time matches), or /proc/<pid> is gone: the process exited (its
      // comm read fails with ESRCH).  A PID whose /proc entry does not exist cannot have been
      // reused, so the cached attribution still names it -- count_kfd_events attributes the VM
      // fault of a process that fault killed (engine.cc) -- until gc() drops it with the PID.
      // Never replaced by a failed lookup.
      e.epoch = epoch_;
      e.st_checked_ns = now_ns_;
      if (kfd_id && have_st) e.kfd_id = kfd_id;  // (a gone process is not vouched for by KFD)
      return &e.info;
    }
  }
  uint64_t st = 0;
  const bool have_st = read_starttime(pid, &st);
  std::string content;
  const std::string dir = root_ + "/proc/" + std::to_string(pid);
  if (!read_small_file(dir + "/cgroup", &content)) {
    Entry& f = cache_[pid];
    f = Entry();  // ok = false
    f.epoch = epoch_;
    f.failed_ns = now_ns_;
    return nullptr;
  }
  Entry& e = cache_[pid];
  e = Entry();
  e.starttime = have_st ? st : 0;
  e.ok = true;
  e.epoch = epoch_;
  e.st_checked_ns = now_ns_;
  e.comm = std::make_shared<CachedFile>();
  if (!e.comm->open(dir + "/comm")) e.comm.reset();
  e.kfd_id = kfd_id;
  parse_proc_cgroup(content, &e.info);
  return &e.info;
}

void PidResolver::set_override(int pid, const std::string& cgroup_path) {
  overrides_[pid] = cgroup_path;
  cache_.erase(pid);
}

void PidResolver::clear_overrides() {
  for (auto& kv : overrides_) cache_.erase(kv.first);
  overrides_.clear();
}

void PidResolver::gc(const std::vector<int>& live_pids) {
  // (every tick: a sorted scratch vector, no hash set built and freed each time)
  gc_live_.assign(live_pids.begin(), live_pids.end());
  std::sort(gc_live_.begin(), gc_live_.end());
  for (auto it = cache_.begin(); it != cache_.end();)
    it = std::binary_search(gc_live_.begin(), gc_live_.end(), it->first) ? std::next(it) : cache_.erase(it);
}

}  // namespace gpuexp
