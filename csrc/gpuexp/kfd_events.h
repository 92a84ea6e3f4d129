// KFD SMI events: the kernel's per-GPU event stream (AMDKFD_IOC_SMI_EVENTS on /dev/kfd;
// what rocm-smi / amdsmi_get_gpu_event_notification read): GPU VM faults (the failure a
// bad kernel produces on MI355X — the HIP runtime then aborts the process), thermal
// throttling, GPU resets, and queue evictions / restores (a process's queues taken off the
// GPU, e.g. for memory eviction).  The reference watched no failure signal at all (it
// crashed on any NVML error, /root/reference/main.go:119-137); here each event is counted
// per GPU and, when the kernel names the process, per pod.
//
// One anonymous event fd per GPU, drained non-blocking every tick (a read of an empty fd
// returns EAGAIN; the kernel keeps a small FIFO per fd).  Without CAP_SYS_ADMIN the kernel
// delivers device-wide events (throttling, resets) and only this process's own per-process
// events; the DaemonSet's privileged container sees every process's.  The high-volume SVM
// events (page faults, migrations, unmaps) are not subscribed: they would overrun the FIFO.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include <poll.h>

#include "gpuexp/device.h"

namespace gpuexp {

// KFD_SMI_EVENT_* ids (linux/kfd_ioctl.h; 5-11 from ROCm's kfd_ioctl.h).
enum KfdEventId : int {
  kKfdVmFault = 1,
  kKfdThermalThrottle = 2,
  kKfdGpuPreReset = 3,
  kKfdGpuPostReset = 4,
  kKfdMigrateStart = 5,
  kKfdMigrateEnd = 6,
  kKfdPageFaultStart = 7,
  kKfdPageFaultEnd = 8,
  kKfdQueueEviction = 9,
  kKfdQueueRestore = 10,
  kKfdUnmapFromGpu = 11,
};
constexpr int kKfdEventIds = 12;  // ids 1..11 (0 unused)
// The subscribed events, in export order.
constexpr int kKfdSubscribed[] = {kKfdVmFault, kKfdThermalThrottle, kKfdGpuPreReset, kKfdGpuPostReset,
                                  kKfdQueueEviction, kKfdQueueRestore};

// "vm_fault", "thermal_throttle", ... ("" for an unknown id).
const char* kfd_event_name(int id);

// Parses one event message "<id hex> <payload>" (the kernel's kfd_smi_event_add format).
// *pid is the process the kernel names (VM fault "<pid hex>:<comm>", queue / SVM events
// "<ns> -<pid dec> ..."), or -1 for device-wide events.  False for a malformed line.
bool parse_kfd_event(const char* s, size_t n, int* event, int* pid);

struct KfdEvent {
  int dev = 0;  // engine device index
  int event = 0;
  int pid = -1;
};

class KfdEventSource {
 public:
  KfdEventSource() = default;
  ~KfdEventSource();
  KfdEventSource(const KfdEventSource&) = delete;
  KfdEventSource& operator=(const KfdEventSource&) = delete;

  // Opens one event fd per device (KFD gpu_id) through `kfd_path`.  Returns the number
  // opened; *err says why one failed.
  int open(const std::vector<DeviceInfo>& devs, const std::string& kfd_path, std::string* err);
  // Drains every fd; appends complete events.
  void drain(std::vector<KfdEvent>* out);
  // Appends the events in `bytes` read from device `dev`'s fd (a message may arrive split
  // over two reads: the tail after the last newline is kept for the next call).  Also the
  // test hook for the CPU tiers.
  void feed(int dev, const char* bytes, size_t n, std::vector<KfdEvent>* out);
  void close_all();
  size_t devices() const { return partial_.size(); }
  void set_devices(size_t n) { partial_.assign(n, std::string()); fds_.assign(n, -1); }
  // Tests: drain() these (non-blocking) fds as devices 0..n-1 instead of KFD's (owned: closed).
  void adopt_fds(const std::vector<int>& fds) {
    set_devices(fds.size());
    fds_ = fds;
  }
  // CAP_SYS_ADMIN was effective at open: every process's per-process events are delivered.
  bool all_processes() const { return all_processes_; }
  uint64_t malformed() const { return malformed_; }

 private:
  int kfd_fd_ = -1;
  std::vector<int> fds_;
  std::vector<struct pollfd> pfds_;  // drain()'s poll set (reused)
  std::vector<std::string> partial_;
  bool all_processes_ = false;
  uint64_t malformed_ = 0;
};

}  // namespace gpuexp
