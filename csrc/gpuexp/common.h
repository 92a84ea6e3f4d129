// Common types for the gpuexp telemetry core.
//
// The reference exporter is a single Go main() (/root/reference/main.go:38-158) that
// polls NVML every 30 s and pushes two GaugeVecs.  This core replaces that with a
// timerfd-driven native sampler that writes into a pre-rendered exposition snapshot,
// so the scrape path never touches GPU I/O.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <ctime>
#include <limits>
#include <string>
#include <atomic>
#include <vector>

namespace gpuexp {

constexpr double kNaN = std::numeric_limits<double>::quiet_NaN();

inline uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

inline uint64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

// Tests / projections only: thread CPU burnt so far by the fake sources' stand-ins for silicon
// costs (a fresh SMU fetch, a PMC read round, a sentinel run; fake_metrics_cost_us and
// fake_{pmc,sentinel}_cost_us), so a projection can tell the exporter's own work from them.
std::atomic<uint64_t>& fake_cpu_burnt_ns();

// Names the calling thread (/proc/<pid>/task/<tid>/comm, 15 chars): the exporter's threads
// are gpuexp-sampler, gpuexp-dev (per-GPU read pool), gpuexp-http, gpuexp-pmc, so their CPU
// can be told apart from outside (tests/test_fakehost.py checks the sampler's own account
// against them).
void set_thread_name(const char* name);

// Leveled logging to stderr in logfmt.  The reference printed every pod every cycle to
// stdout (main.go:81,89,108); here nothing is logged per tick at info level.
enum class LogLevel : int { kDebug = 0, kInfo = 1, kWarn = 2, kError = 3, kOff = 4 };
void set_log_level(LogLevel lvl);
LogLevel log_level();
void set_log_json(bool json);  // records as JSON objects instead of logfmt
void log_msg(LogLevel lvl, const char* component, const std::string& msg);

#define GPUEXP_LOG(lvl, comp, msg)                                    \
  do {                                                                \
    if (static_cast<int>(lvl) >= static_cast<int>(::gpuexp::log_level())) \
      ::gpuexp::log_msg(lvl, comp, msg);                              \
  } while (0)

// Small helpers shared by the sysfs/procfs readers.  All file access goes through a
// host-root prefix so tests can point the exporter at a fake /sys + /proc tree.
bool read_small_file(const std::string& path, std::string* out, size_t max_bytes = 65536);
bool read_u64_file(const std::string& path, uint64_t* v);
// pread() an already-open fd from offset 0.  Returns bytes read or -1.
long pread_all(int fd, char* buf, size_t cap);
// ONE pread() at offset 0.  For sysfs attributes: the kernel renders the whole value
// (<= PAGE_SIZE) per read, and a second read at EOF renders it AGAIN — for gpu_metrics
// that is a second SMU table transfer (measured: 410 us/GPU/tick with two reads).
long pread_once(int fd, char* buf, size_t cap);
bool parse_u64(const char* s, size_t n, uint64_t* v);
std::string trim(const std::string& s);
std::vector<std::string> list_dir(const std::string& path);

}  // namespace gpuexp
