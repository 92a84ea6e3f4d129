// GPU process discovery (KFD sysfs) and PID -> pod attribution (cgroup v2/v1 paths).
//
// Reference: NVML GetComputeRunningProcesses (host PIDs, /root/reference/main.go:135)
// joined against `kubectl exec <pod> -- ps -e -o pid=` output (container-namespace PIDs,
// main.go:101) with `for pid := range pids` comparing an INDEX to a PID (main.go:144) —
// broken twice.  Here: host PIDs from /sys/class/kfd/kfd/proc/<pid>/
// vram_<gpu_id> (exactly the GPUs that process has a KFD context on, measured on the
// box), then /proc/<pid>/cgroup -> pod UID + container ID, no subprocesses, no exec RBAC.
#pragma once

#include <cstdint>
#include <ctime>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "gpuexp/backends.h"
#include "gpuexp/device.h"

namespace gpuexp {

class KfdProcReader {
 public:
  // detail_interval_ns: cu_occupancy / sdma are re-read at most this often (0 = every
  // scan).  Measured on MI355X (profiles/r01/kfd_read_costs.txt): vram_<id> ~6 us,
  // stats_<id>/cu_occupancy ~15 us (KFD asks the hardware), sdma_<id> ~7 us per process
  // per GPU — VRAM is what the legacy families and attribution need every tick.
  // read_sdma: also read sdma_<id> (the engine's kfd_sdma; off by default, see EngineConfig).
  KfdProcReader(std::string host_root, int self_pid, bool read_cu_occupancy, uint64_t detail_interval_ns = 0,
                uint64_t rescan_interval_ns = 0, bool read_sdma = true);
  ~KfdProcReader();
  KfdProcReader(const KfdProcReader&) = delete;
  KfdProcReader& operator=(const KfdProcReader&) = delete;
  // Fills per_dev[d] with the processes that have a KFD context on device d.
  // `defer_listing`: a listing due only to the rescan timer waits for a later scan (a tick that
  // already carries more SMU fetches than most; the engine's tick leveling, engine.cc).
  void scan(const std::vector<DeviceInfo>& devs, std::vector<std::vector<ProcSample>>* per_dev,
            uint64_t now_ns = 0, bool defer_listing = false);
  size_t tracked() const { return pids_.size(); }
  uint64_t lists() const { return lists_; }    // scans that listed the directory
  bool listing_deferred() const { return deferred_; }  // the last scan put off a due listing
  uint64_t dir_reopens() const { return dir_reopens_; }  // the proc directory was replaced (KFD reload)
  uint64_t scans() const { return scan_no_; }  // all scans

 private:
  struct PerDev {
    int dev = -1;
    CachedFile vram, cu, sdma, evicted;
    double cu_last = kNaN, sdma_last = kNaN, evicted_last = kNaN;
    uint64_t detail_ns = 0;  // last cu/sdma read
    bool detail_read = false;
  };
  struct Entry {
    std::vector<PerDev> devs;
    std::string comm;
    int comm_tries = 0;  // re-reads of an empty comm at later listings
    uint64_t probe_ns = 0;  // last look for GPUs it had no files for
    uint64_t probe_every_ns = kReprobeNs;  // doubles (to kReprobeMaxNs) while looks find nothing
    uint64_t seen = 0;
    uint64_t id = 0;        // ProcSample::kfd_id
  };
  static constexpr int kCommTries = 3;
  static constexpr uint64_t kReprobeNs = 1000000000ull;
  static constexpr uint64_t kReprobeMaxNs = 8000000000ull;
  // Appends the entry's per-GPU samples; returns how many vram reads succeeded.
  int emit(Entry& e, int pid, std::vector<std::vector<ProcSample>>* per_dev, uint64_t now_ns);
  std::string root_;
  int self_;
  bool read_cu_;
  bool read_sdma_;
  uint64_t detail_every_ns_;
  uint64_t rescan_ns_ = 0;       // list the KFD proc directory at least this often (0: every scan)
  uint64_t last_list_ns_ = 0;
  bool deferred_ = false;
  bool relist_ = false;          // a tracked process vanished: list at the next scan
  timespec mtime_{};             // the directory's mtime at the last look
  int dir_fd_ = -1;              // the KFD proc directory, kept open: fstat per scan, no path walk
  uint64_t open_tried_ns_ = 0;   // last failed open of it (no KFD): retried at the rescan interval
  uint64_t scan_no_ = 0, lists_ = 0, next_id_ = 0, dir_reopens_ = 0;
  std::unordered_map<int, Entry> pids_;
};

struct CgroupInfo {
  bool kube = false;
  std::string pod_uid;       // dashed form
  std::string container_id;  // 64-hex (or runtime-specific)
  std::string runtime;       // containerd | crio | docker | unknown
  std::string qos;           // guaranteed | burstable | besteffort
  std::string path;          // the cgroup path the info came from
};

// Parses one cgroup path (e.g. "/kubepods.slice/kubepods-burstable.slice/
// kubepods-burstable-pod<uid_>.slice/cri-containerd-<id>.scope" or
// "/kubepods/burstable/pod<uid>/<id>").  Returns false if no pod UID is found.
bool parse_kube_cgroup_path(const std::string& path, CgroupInfo* out);
// Parses a whole /proc/<pid>/cgroup file (v2 "0::" line preferred; v1 fallbacks).
bool parse_proc_cgroup(const std::string& content, CgroupInfo* out);

// Caches pid -> CgroupInfo keyed on (pid, starttime) so PID reuse is detected.
// The reuse check costs one cheap read per PID per tick: a cached fd of /proc/<pid>/comm
// (reads of a /proc/<pid> file fail with ESRCH once that process is gone, so a new process
// under the same PID cannot pass it), and the starttime in /proc/<pid>/stat at most once a
// second (generating stat sums over every thread of the process: 4 us for one thread,
// tens of us for a framework process with hundreds).  Called at most once per PID per tick
// whatever the number of callers.
class PidResolver {
 public:
  explicit PidResolver(std::string host_root);
  // Starts a tick at (engine) time now_ns: every PID is re-checked once in it.
  void begin_tick(uint64_t now_ns) {
    ++epoch_;
    now_ns_ = now_ns;
  }
  // Returns nullptr if the PID cannot be read (other PID namespace, exited).  A failure is
  // remembered: the PID is not looked up again within the tick nor for kRetryFailedNs.
  // `kfd_id` (ProcSample::kfd_id, 0 = none): the KFD reader read this very process this tick.
  // A cached entry checked under the same id needs no liveness read: the id outlives neither
  // the process nor a reuse of its PID (KfdProcReader re-creates the entry for either).
  const CgroupInfo* resolve(int pid, uint64_t kfd_id = 0);
  // Test/bench hook: pretend /proc/<pid>/cgroup contains `cgroup_path`.
  void set_override(int pid, const std::string& cgroup_path);
  void clear_overrides();
  void gc(const std::vector<int>& live_pids);

 private:
  struct Entry {
    uint64_t starttime = 0;
    bool ok = false;
    CgroupInfo info;
    std::shared_ptr<CachedFile> comm;  // /proc/<pid>/comm, kept open (liveness)
    uint64_t epoch = 0;                // tick it was last checked in
    uint64_t st_checked_ns = 0;        // engine time of the last starttime check
    uint64_t failed_ns = 0;            // !ok: engine time of the failed lookup
    uint64_t kfd_id = 0;               // KFD identity it was last checked under (0 = none)
  };
  bool read_starttime(int pid, uint64_t* st);
  static constexpr uint64_t kStarttimeEveryNs = 1000000000ull;
  // An unreadable PID (a host PID from inside a PID namespace, hidepid, a process gone) was
  // looked up again on every call: 2 failed opens per call, 2 calls per process per tick.
  static constexpr uint64_t kRetryFailedNs = 1000000000ull;
  uint64_t epoch_ = 1, now_ns_ = 0;
  std::string root_;
  std::unordered_map<int, Entry> cache_;
  std::vector<int> gc_live_;  // gc() scratch
  std::unordered_map<int, std::string> overrides_;
};

}  // namespace gpuexp
