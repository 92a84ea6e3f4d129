// Concurrency stress for the telemetry core (run under TSAN / ASAN+UBSAN via CMake presets):
//   - sampler thread at 100 Hz over 8 mock GPUs
//   - HTTP server with 2 SO_REUSEPORT loops
//   - N scraper threads on keep-alive connections (plus one gzip scraper)
//   - a control-plane thread swapping pods / cgroup overrides / process lists / faults
//   - an RCCL-tracer stand-in that rewrites, truncates and replaces its counters file
//     (the exporter's writer proof maps the file itself, see optional_sources.cc)
//   - then a steady phase: one scraper at a fixed 40 ms period alone, so the sampler skips the
//     ticks no scrape reads (render_when_due: no table writes, no render) while the
//     control-plane and tracer threads keep going
// Every response must be a complete exposition whose tick counter never goes backwards.
// SURVEY.md §5 "Race detection / sanitizers": sampler vs HTTP vs attribution updates.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <zlib.h>
#include <sys/stat.h>
#include <unistd.h>

#include "gpuexp/client.h"
#include "gpuexp/engine.h"
#include "gpuexp/rccl_shm.h"

using namespace gpuexp;

// Walks a varint-length-delimited protobuf stream; true if the frames tile it exactly.
static bool delimited_ok(const std::string& b) {
  size_t pos = 0;
  while (pos < b.size()) {
    uint64_t len = 0;
    int shift = 0;
    while (true) {
      if (pos >= b.size() || shift > 63) return false;
      const uint8_t c = uint8_t(b[pos++]);
      len |= uint64_t(c & 0x7f) << shift;
      if (!(c & 0x80)) break;
      shift += 7;
    }
    if (len == 0 || pos + len > b.size()) return false;
    pos += size_t(len);
  }
  return true;
}

// Inflates a gzip member (zlib's inflater, independent of the exporter's encoder); false if it
// is not one complete, valid member.
static bool gunzip(const std::string& in, std::string* out) {
  z_stream zs{};
  if (inflateInit2(&zs, 16 + 15) != Z_OK) return false;
  out->clear();
  zs.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data()));
  zs.avail_in = uInt(in.size());
  char buf[65536];
  int rc;
  do {
    zs.next_out = reinterpret_cast<Bytef*>(buf);
    zs.avail_out = sizeof(buf);
    rc = inflate(&zs, Z_NO_FLUSH);
    out->append(buf, sizeof(buf) - zs.avail_out);
  } while (rc == Z_OK);
  const bool ok = rc == Z_STREAM_END && zs.avail_in == 0;
  inflateEnd(&zs);
  return ok;
}

static double ticks_in(const std::string& body) {
  size_t p = body.find("\ngpuexp_ticks_total ");
  if (p == std::string::npos) return -1;
  return std::atof(body.c_str() + p + 20);
}

int main(int argc, char** argv) {
  double seconds = argc > 1 ? std::atof(argv[1]) : 3.0;
  int scrapers = argc > 2 ? std::atoi(argv[2]) : 4;
  EngineConfig cfg;
  cfg.backend = "mock";
  cfg.mock_devices = 8;
  cfg.device_threads = 4;  // exercise the fork-join device pool under the sanitizers
  cfg.interval_s = 0.01;
  cfg.enable_sentinel = true;
  cfg.enable_counters = true;
  cfg.series_profile = "full";  // every family, KFD events and per-pod energy included
  cfg.state_file = "/tmp/gpuexp-stress-state-" + std::to_string(::getpid());  // checkpoint every 50 ms
  cfg.state_interval_s = 0.05;
  char rccl_tmpl[] = "/tmp/gpuexp-stress-rccl-XXXXXX";
  const std::string rccl_dir = ::mkdtemp(rccl_tmpl) ? rccl_tmpl : "";
  cfg.enable_rccl = !rccl_dir.empty();
  cfg.rccl_dir = rccl_dir;
  cfg.http.host = "127.0.0.1";
  cfg.http.port = 0;
  cfg.http.threads = 2;
  Engine e(cfg);
  std::string err;
  if (!e.start(&err)) {
    std::fprintf(stderr, "start failed: %s\n", err.c_str());
    return 2;
  }
  int port = e.http_port();
  std::atomic<bool> stop{false}, stop_busy{false};
  std::atomic<long> scrapes{0}, bad{0}, rccl_seen{0};

  std::vector<std::thread> th, busy;
  for (int s = 0; s < scrapers; ++s) {
    busy.emplace_back([&, s] {
      // scraper 0: gzip; scraper 1: protobuf exposition; the rest: plain text
      ScrapeClient c("127.0.0.1", port, "/metrics", s == 0, 2000,
                     s == 1 ? "application/vnd.google.protobuf;proto=io.prometheus.client.MetricFamily;"
                              "encoding=delimited"
                            : "");
      double last = -1;
      while (!stop_busy.load()) {
        double ns = c.scrape();
        if (ns < 0 || c.last_status() == 503) continue;
        scrapes.fetch_add(1);
        if (s == 1 && !c.last_body().empty() && c.last_body()[0] != '#') {
          if (!delimited_ok(c.last_body())) bad.fetch_add(1);  // protobuf: framing must be exact
          continue;
        }
        std::string inflated;
        if (s == 0 && !gunzip(c.last_body(), &inflated)) {  // gzip: a valid member of a valid body
          bad.fetch_add(1);
          continue;
        }
        const std::string& b = s == 0 ? inflated : c.last_body();
        double t = ticks_in(b);
        if (b.find("\namd_rccl_collective_calls_total{") != std::string::npos) rccl_seen.fetch_add(1);
        if (b.compare(0, 7, "# HELP ") != 0 || b.back() != '\n' || t < last) bad.fetch_add(1);
        last = t;
      }
    });
  }
  th.emplace_back([&] {
    unsigned k = 0;
    while (!stop.load()) {
      ++k;
      std::vector<PodMeta> pods(2);
      pods[0] = {"12345678-1234-1234-1234-1234567890a" + std::to_string(k % 10), "ns", "pod-" + std::to_string(k % 7),
                 {{std::string(64, 'a'), "main"}}};
      pods[1] = {"22345678-1234-1234-1234-1234567890ab", "ns2", "pod-b", {}};
      e.set_pods(pods, k % 3 != 0);  // every third refresh "incomplete" (a source failed)
      if (k % 4 == 0) (void)e.source_status();  // races save_state()'s status updates
      e.set_pid_cgroup(int(100 + k % 5), "/kubepods/burstable/pod12345678-1234-1234-1234-1234567890a" +
                                              std::to_string(k % 10) + "/" + std::string(64, 'a'));
      if (k % 50 == 0) e.clear_pid_cgroups();
      std::vector<ProcSample> procs;
      for (int p = 0; p < int(k % 6); ++p) {
        ProcSample ps;
        ps.pid = 100 + p;
        ps.vram_bytes = 1e9 * p;
        ps.cu_occupancy = 10;
        procs.push_back(ps);
      }
      e.mock()->set_processes(int(k % 8), procs);
      e.mock()->set_fault(int(k % 8), k % 13 == 0 ? "error" : "none");
      e.set_device_owners({{"0000:10:00.0", DeviceOwner{"ns", "owner-" + std::to_string(k % 3), "c"}}});
      // KFD events for the sampler to count and attribute (split lines exercise the
      // per-device tail buffer)
      e.inject_kfd_events(int(k % 8), "9 " + std::to_string(k) + " -" + std::to_string(100 + k % 5) + " 0 2\n1 6");
      e.inject_kfd_events(int(k % 8), "5:python3\n2 0:1\n");
      std::this_thread::sleep_for(std::chrono::milliseconds(3));
    }
  });
  struct stat ns_st {};
  const bool have_ns = ::stat("/proc/self/ns/pid", &ns_st) == 0;
  const std::string rccl_path = rccl_dir + "/gpuexp-rccl-" + std::to_string(uint64_t(ns_st.st_ino)) + "-" +
                                std::to_string(::getpid());
  if (cfg.enable_rccl && have_ns) {
    th.emplace_back([&] {
      // The tracer's life cycle, compressed: create + map + publish, count, then either
      // truncate the file under the reader or unlink it and start over with a new inode.
      for (unsigned k = 0; !stop.load(); ++k) {
        int fd = ::open(rccl_path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
        if (fd < 0) return;
        if (::ftruncate(fd, sizeof(RcclShmFile)) != 0) {
          ::close(fd);
          return;
        }
        void* p = ::mmap(nullptr, sizeof(RcclShmFile), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        ::close(fd);
        if (p == MAP_FAILED) return;
        auto* f = static_cast<RcclShmFile*>(p);
        f->version = 1;
        f->ns_pid = int32_t(::getpid());
        f->pidns_ino = uint64_t(ns_st.st_ino);
        f->rank = 0;
        f->nranks = 2;
        __atomic_store_n(&f->magic, kRcclShmMagic, __ATOMIC_RELEASE);
        for (int i = 0; i < 100 && !stop.load(); ++i) {
          f->ops[0].calls.fetch_add(1, std::memory_order_relaxed);
          f->ops[0].bytes.fetch_add(1u << 20, std::memory_order_relaxed);
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
        ::munmap(p, sizeof(RcclShmFile));
        if (k % 2 == 0) {
          if (::truncate(rccl_path.c_str(), 8) != 0) return;  // short file: must be skipped, not fault
        } else {
          ::unlink(rccl_path.c_str());  // replaced by a new inode next round
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(15));
      }
    });
  }
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  stop_busy.store(true);
  for (auto& t : busy) t.join();
  // steady phase: one keep-alive scraper at a fixed period, everything else still churning
  long steady_scrapes = 0;
  const uint64_t skipped0 = e.stats().renders_skipped;
  {
    ScrapeClient c("127.0.0.1", port, "/metrics", true, 2000, "");
    double last = -1;
    auto next = std::chrono::steady_clock::now();
    const auto end = next + std::chrono::duration<double>(std::max(1.0, seconds / 2));
    while (next < end) {
      double ns = c.scrape();
      std::string inflated;
      if (ns >= 0 && c.last_status() == 200) {
        ++steady_scrapes;
        const double t = gunzip(c.last_body(), &inflated) ? ticks_in(inflated) : -2;
        if (t < last) bad.fetch_add(1);  // (a skipped tick serves the last render: never older than it)
        last = t;
      }
      next += std::chrono::milliseconds(40);
      std::this_thread::sleep_until(next);
    }
  }
  const uint64_t skipped = e.stats().renders_skipped - skipped0;
  stop.store(true);
  for (auto& t : th) t.join();
  EngineStats st = e.stats();
  e.stop();
  std::remove(cfg.state_file.c_str());
  if (!rccl_dir.empty()) {
    ::unlink(rccl_path.c_str());
    ::rmdir(rccl_dir.c_str());
  }
  std::printf("ticks=%llu scrapes=%ld bad=%ld series=%llu render_bytes=%llu rccl_scrapes=%ld steady_scrapes=%ld "
              "renders_skipped=%llu\n",
              (unsigned long long)st.ticks, scrapes.load(), bad.load(), (unsigned long long)st.series,
              (unsigned long long)st.render_bytes, rccl_seen.load(), steady_scrapes, (unsigned long long)skipped);
  // (a sanitizer build on a loaded host ticks slowly: the point is the races, not the rate)
  return (bad.load() == 0 && scrapes.load() > 100 && st.ticks >= 5) ? 0 : 1;
}
