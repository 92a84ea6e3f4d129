#include "gpuexp/common.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/prctl.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstring>
#include <mutex>

namespace gpuexp {

void set_thread_name(const char* name) { ::prctl(PR_SET_NAME, name, 0, 0, 0); }

std::atomic<uint64_t>& fake_cpu_burnt_ns() {
  static std::atomic<uint64_t> total{0};
  return total;
}

static std::atomic<int> g_log_level{static_cast<int>(LogLevel::kWarn)};
static std::atomic<bool> g_log_json{false};
static std::mutex g_log_mu;

void set_log_level(LogLevel lvl) { g_log_level.store(static_cast<int>(lvl)); }
LogLevel log_level() { return static_cast<LogLevel>(g_log_level.load(std::memory_order_relaxed)); }
void set_log_json(bool json) { g_log_json.store(json); }

// One record per line on stderr, logfmt (default) or JSON (log_format), with the same keys
// as the Python control plane's records (utils/logfmt.py), so both halves of the exporter
// interleave into one parseable stream.
void log_msg(LogLevel lvl, const char* component, const std::string& msg) {
  static const char* names[] = {"debug", "info", "warn", "error", "off"};
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  const bool json = g_log_json.load(std::memory_order_relaxed);
  std::lock_guard<std::mutex> lk(g_log_mu);
  if (json)
    std::fprintf(stderr, "{\"ts\":%ld.%03ld,\"level\":\"%s\",\"component\":\"%s\",\"msg\":\"", long(ts.tv_sec),
                 long(ts.tv_nsec / 1000000), names[static_cast<int>(lvl)], component);
  else
    std::fprintf(stderr, "ts=%ld.%03ld level=%s component=%s msg=\"", long(ts.tv_sec),
                 long(ts.tv_nsec / 1000000), names[static_cast<int>(lvl)], component);
  for (char c : msg) {
    const unsigned char u = static_cast<unsigned char>(c);
    if (c == '"' || c == '\\') {
      std::fputc('\\', stderr);
      std::fputc(c, stderr);
    } else if (c == '\n') {
      std::fputc(' ', stderr);
    } else if (json && u < 0x20) {
      std::fprintf(stderr, "\\u%04x", u);  // JSON forbids raw control characters
    } else {
      std::fputc(c, stderr);
    }
  }
  std::fputs(json ? "\"}\n" : "\"\n", stderr);
}

bool read_small_file(const std::string& path, std::string* out, size_t max_bytes) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  out->clear();
  char buf[4096];
  while (out->size() < max_bytes) {
    ssize_t n = ::read(fd, buf, sizeof(buf));
    if (n < 0) {
      if (errno == EINTR) continue;
      ::close(fd);
      return false;
    }
    if (n == 0) break;
    out->append(buf, size_t(n));
  }
  ::close(fd);
  return true;
}

bool parse_u64(const char* s, size_t n, uint64_t* v) {
  size_t i = 0;
  while (i < n && (s[i] == ' ' || s[i] == '\t')) ++i;
  if (i == n || s[i] < '0' || s[i] > '9') return false;
  uint64_t x = 0;
  for (; i < n && s[i] >= '0' && s[i] <= '9'; ++i) x = x * 10 + uint64_t(s[i] - '0');
  *v = x;
  return true;
}

bool read_u64_file(const std::string& path, uint64_t* v) {
  char buf[64];
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  ssize_t n = ::read(fd, buf, sizeof(buf) - 1);
  ::close(fd);
  if (n <= 0) return false;
  return parse_u64(buf, size_t(n), v);
}

long pread_all(int fd, char* buf, size_t cap) {
  size_t got = 0;
  while (got < cap) {
    ssize_t n = ::pread(fd, buf + got, cap - got, off_t(got));
    if (n < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    if (n == 0) break;
    got += size_t(n);
  }
  return long(got);
}

long pread_once(int fd, char* buf, size_t cap) {
  for (;;) {
    ssize_t n = ::pread(fd, buf, cap, 0);
    if (n < 0 && errno == EINTR) continue;
    return long(n);
  }
}

std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && (s[b] == ' ' || s[b] == '\n' || s[b] == '\t' || s[b] == '\r')) ++b;
  while (e > b && (s[e - 1] == ' ' || s[e - 1] == '\n' || s[e - 1] == '\t' || s[e - 1] == '\r')) --e;
  return s.substr(b, e - b);
}

std::vector<std::string> list_dir(const std::string& path) {
  std::vector<std::string> out;
  DIR* d = ::opendir(path.c_str());
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    if (e->d_name[0] == '.') continue;
    out.emplace_back(e->d_name);
  }
  ::closedir(d);
  return out;
}

}  // namespace gpuexp
