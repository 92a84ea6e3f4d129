// A tiny in-process sampling profiler for CPU-side hot-path work (no perf in the image).
// Build: g++ -O2 -shared -fPIC -o /tmp/libsigprof.so tools/sigprof.cc
// Use from Python (tools/sigprof.py): start(hz) arms ITIMER_PROF; every signal records the
// interrupted thread's stack (backtrace(), frames after the handler's own); stop(path) writes
// one line per sample (hex PCs) followed by a copy of /proc/self/maps for symbolisation.
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>

namespace {
constexpr int kDepth = 24;
constexpr int kMax = 200000;
void* g_pcs[kMax][kDepth];
int g_n[kMax];
std::atomic<int> g_next{0};

void on_prof(int, siginfo_t*, void*) {
  const int i = g_next.fetch_add(1, std::memory_order_relaxed);
  if (i >= kMax) return;
  g_n[i] = backtrace(g_pcs[i], kDepth);
}
}  // namespace

timer_t g_timer;

// A CLOCK_MONOTONIC high-resolution timer aimed at the calling thread (ITIMER_PROF only
// fires at the scheduler tick: too few samples for a ~100 us tick).  It samples wall time:
// the caller drops samples whose leaf is a sleep.
extern "C" int sigprof_start(int hz) {
  void* warm[4];
  backtrace(warm, 4);  // loads libgcc_s outside the handler
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGPROF, &sa, nullptr);
  sigevent sev{};
  sev.sigev_notify = SIGEV_THREAD_ID;
  sev.sigev_signo = SIGPROF;
  sev._sigev_un._tid = pid_t(syscall(SYS_gettid));
  if (timer_create(CLOCK_MONOTONIC, &sev, &g_timer) != 0) return -1;
  itimerspec its{};
  its.it_interval.tv_nsec = 1000000000L / hz;
  its.it_value = its.it_interval;
  return timer_settime(g_timer, 0, &its, nullptr);
}

extern "C" int sigprof_stop(const char* path) {
  timer_delete(g_timer);
  FILE* f = std::fopen(path, "w");
  if (!f) return -1;
  const int n = std::min(g_next.load(), kMax);
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < g_n[i]; ++k) std::fprintf(f, "%p ", g_pcs[i][k]);
    std::fputc('\n', f);
  }
  std::fputs("MAPS\n", f);
  if (FILE* m = std::fopen("/proc/self/maps", "r")) {
    char buf[4096];
    size_t r;
    while ((r = std::fread(buf, 1, sizeof(buf), m)) > 0) std::fwrite(buf, 1, r, f);
    std::fclose(m);
  }
  std::fclose(f);
  g_next = 0;
  return n;
}
