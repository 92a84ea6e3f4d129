#include "gpuexp/kfd_events.h"

#include <fcntl.h>
#include <linux/kfd_ioctl.h>
#include <poll.h>
#include <sys/ioctl.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace gpuexp {

namespace {

constexpr uint64_t mask_of(int id) { return 1ull << (id - 1); }
constexpr int kAllProcessesBit = 64;  // KFD_SMI_EVENT_ALL_PROCESS: every process's events (CAP_SYS_ADMIN)

// CapEff bit 21 = CAP_SYS_ADMIN (what kfd_smi_event_open records as the client's `suser`).
bool has_cap_sys_admin() {
  FILE* f = std::fopen("/proc/self/status", "r");
  if (!f) return false;
  char line[256];
  bool yes = false;
  while (std::fgets(line, sizeof(line), f)) {
    if (std::strncmp(line, "CapEff:", 7) == 0) {
      yes = (std::strtoull(line + 7, nullptr, 16) >> 21) & 1;
      break;
    }
  }
  std::fclose(f);
  return yes;
}

bool parse_hex(const char*& p, const char* end, uint64_t* v) {
  const char* s = p;
  uint64_t x = 0;
  while (p < end) {
    const char c = *p;
    int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
    if (d < 0) break;
    x = x * 16 + uint64_t(d);
    ++p;
  }
  *v = x;
  return p > s;
}

}  // namespace

const char* kfd_event_name(int id) {
  switch (id) {
    case kKfdVmFault: return "vm_fault";
    case kKfdThermalThrottle: return "thermal_throttle";
    case kKfdGpuPreReset: return "gpu_pre_reset";
    case kKfdGpuPostReset: return "gpu_post_reset";
    case kKfdMigrateStart: return "migrate_start";
    case kKfdMigrateEnd: return "migrate_end";
    case kKfdPageFaultStart: return "page_fault_start";
    case kKfdPageFaultEnd: return "page_fault_end";
    case kKfdQueueEviction: return "queue_eviction";
    case kKfdQueueRestore: return "queue_restore";
    case kKfdUnmapFromGpu: return "unmap_from_gpu";
    default: return "";
  }
}

bool parse_kfd_event(const char* s, size_t n, int* event, int* pid) {
  const char* p = s;
  const char* end = s + n;
  uint64_t id = 0;
  if (!parse_hex(p, end, &id) || id == 0 || id >= uint64_t(kKfdEventIds) || p >= end || *p != ' ') return false;
  ++p;
  *event = int(id);
  *pid = -1;
  if (id == kKfdVmFault) {
    // "<pid hex>:<task name>"
    uint64_t v = 0;
    if (!parse_hex(p, end, &v) || p >= end || *p != ':') return false;
    *pid = int(v);
  } else if (id >= kKfdMigrateStart) {
    // "<timestamp ns> -<pid decimal> ..."
    while (p < end && *p != ' ') ++p;
    if (p + 2 > end || p[1] != '-') return false;
    p += 2;
    long v = 0;
    const char* d = p;
    while (p < end && *p >= '0' && *p <= '9') v = v * 10 + (*p++ - '0');
    if (p == d) return false;
    *pid = int(v);
  }
  return true;
}

KfdEventSource::~KfdEventSource() { close_all(); }

void KfdEventSource::close_all() {
  for (int& fd : fds_) {
    if (fd >= 0) ::close(fd);
    fd = -1;
  }
  if (kfd_fd_ >= 0) ::close(kfd_fd_);
  kfd_fd_ = -1;
}

int KfdEventSource::open(const std::vector<DeviceInfo>& devs, const std::string& kfd_path, std::string* err) {
  close_all();
  set_devices(devs.size());
  kfd_fd_ = ::open(kfd_path.c_str(), O_RDWR | O_CLOEXEC);
  if (kfd_fd_ < 0) {
    *err = "open " + kfd_path + ": " + std::strerror(errno);
    return 0;
  }
  all_processes_ = has_cap_sys_admin();
  uint64_t mask = 0;
  for (int id : kKfdSubscribed) mask |= mask_of(id);
  mask |= mask_of(kAllProcessesBit);  // honoured only for a CAP_SYS_ADMIN client
  int opened = 0;
  for (size_t i = 0; i < devs.size(); ++i) {
    if (!devs[i].kfd_gpu_id) continue;
    kfd_ioctl_smi_events_args a{};
    a.gpuid = devs[i].kfd_gpu_id;
    if (::ioctl(kfd_fd_, AMDKFD_IOC_SMI_EVENTS, &a) != 0) {
      *err = "AMDKFD_IOC_SMI_EVENTS gpu_id " + std::to_string(devs[i].kfd_gpu_id) + ": " + std::strerror(errno);
      continue;
    }
    const int fd = int(a.anon_fd);
    ::fcntl(fd, F_SETFD, FD_CLOEXEC);
    ::fcntl(fd, F_SETFL, ::fcntl(fd, F_GETFL) | O_NONBLOCK);
    if (::write(fd, &mask, sizeof(mask)) != ssize_t(sizeof(mask))) {
      *err = std::string("event mask write: ") + std::strerror(errno);
      ::close(fd);
      continue;
    }
    fds_[i] = fd;
    ++opened;
  }
  if (!opened && err->empty()) *err = "no device with a KFD gpu_id";
  return opened;
}

void KfdEventSource::drain(std::vector<KfdEvent>* out) {
  // one poll over every GPU's event fd per tick (a quiet node: one system call, not one read
  // per GPU); only the readable ones are read
  pfds_.clear();
  for (size_t i = 0; i < fds_.size(); ++i)
    if (fds_[i] >= 0) pfds_.push_back({fds_[i], POLLIN, 0});
  if (pfds_.empty() || ::poll(pfds_.data(), nfds_t(pfds_.size()), 0) <= 0) return;
  char buf[4096];
  size_t p = 0;
  for (size_t i = 0; i < fds_.size(); ++i) {
    if (fds_[i] < 0) continue;
    if (!(pfds_[p++].revents & (POLLIN | POLLERR | POLLHUP))) continue;
    for (int rounds = 0; rounds < 16; ++rounds) {  // the kernel FIFO is small: a few reads empty it
      const ssize_t r = ::read(fds_[i], buf, sizeof(buf));
      if (r <= 0) break;  // EAGAIN: empty
      feed(int(i), buf, size_t(r), out);
    }
  }
}

void KfdEventSource::feed(int dev, const char* bytes, size_t n, std::vector<KfdEvent>* out) {
  if (dev < 0 || size_t(dev) >= partial_.size()) return;
  std::string& tail = partial_[size_t(dev)];
  tail.append(bytes, n);
  size_t start = 0;
  for (size_t nl; (nl = tail.find('\n', start)) != std::string::npos; start = nl + 1) {
    KfdEvent e;
    e.dev = dev;
    if (nl > start && parse_kfd_event(tail.data() + start, nl - start, &e.event, &e.pid))
      out->push_back(e);
    else if (nl > start)
      ++malformed_;
  }
  tail.erase(0, start);
  if (tail.size() > 1024) {  // no newline in a KiB: not an event stream we understand
    ++malformed_;
    tail.clear();
  }
}

}  // namespace gpuexp
