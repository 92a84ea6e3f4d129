#include "gpuexp/http.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sched.h>
#include <sys/prctl.h>
#include <sys/timerfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>
#include <immintrin.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

#include "gpuexp/common.h"

namespace gpuexp {

uint64_t ArrivalPredictor::period() const {
  if (n_iv < 4) return 0;
  uint64_t v[16];
  std::copy(iv, iv + n_iv, v);
  std::nth_element(v, v + n_iv / 2, v + n_iv);
  return v[n_iv / 2];
}

void ArrivalPredictor::observe(uint64_t arrival, bool steady) {
  if (!steady || !last || arrival <= last) {  // (re)start: no schedule to predict from
    if (!steady) n = n_iv = 0;
    phase = last = arrival;
    return;
  }
  const uint64_t p = period();
  if (p) {
    const uint64_t e_rel = last + p, e_abs = phase + p;
    err_rel[pos] = int64_t(arrival) - int64_t(e_rel);
    err_abs[pos] = int64_t(arrival) - int64_t(e_abs);
    pos = (pos + 1) & 15;
    if (n < 16) ++n;
    const int64_t d = err_abs[(pos + 15) & 15];
    // follow the schedule a quarter of each error; a jump beyond 1/8 period re-anchors it
    phase = (d > int64_t(p / 8) || -d > int64_t(p / 8)) ? arrival : uint64_t(int64_t(e_abs) + d / 4);
  } else {
    phase = arrival;
  }
  iv[iv_pos] = arrival - last;
  iv_pos = (iv_pos + 1) & 15;
  if (n_iv < 16) ++n_iv;
  last = arrival;
}

static int64_t spread_of(const int64_t* e, int n, int64_t* sorted) {
  std::copy(e, e + n, sorted);
  std::sort(sorted, sorted + n);
  return sorted[n - 2] - sorted[1];  // one outlier each side ignored
}

int ArrivalPredictor::window(uint64_t max_ns, uint64_t margin, uint64_t* from, uint64_t* until) const {
  const uint64_t p = period();
  if (!p || !last) return 0;
  if (n < 8) {  // too few errors: max_ns centred on the relative prediction
    *from = last + p - max_ns / 2;
    *until = last + p + max_ns / 2;
    return 1;
  }
  int64_t vr[16], va[16];
  const int64_t sr = spread_of(err_rel, n, vr), sa = spread_of(err_abs, n, va);
  const bool abs_wins = sa < sr;
  const int64_t* v = abs_wins ? va : vr;
  const uint64_t e = (abs_wins ? phase : last) + p;
  const int64_t lo = v[1] - int64_t(margin), hi = v[n - 2] + int64_t(margin);
  const int64_t med = v[n / 2];
  int64_t a = lo, b = hi;
  if (b - a > int64_t(max_ns)) {  // keep max_ns around the median arrival
    a = std::max(lo, med - int64_t(max_ns) / 2);
    b = a + int64_t(max_ns);
    if (b > hi) {
      b = hi;
      a = b - int64_t(max_ns);
    }
  }
  *from = uint64_t(int64_t(e) + a);
  *until = uint64_t(int64_t(e) + b);
  return abs_wins ? 2 : 1;
}

uint64_t learnt_scrape_period_ns(const uint64_t* newest_first, int n) {
  for (int k = 0; k < n; ++k) {
    const uint64_t a = newest_first[k];
    if (a < 20000000ull) continue;  // < 20 ms: not a scrape period the pre-wake follows
    uint64_t set[8];
    int m = 0;
    set[m++] = a;
    for (int j = 0; j < n && m < 8; ++j) {
      if (j == k) continue;
      const uint64_t b = newest_first[j];
      const uint64_t lo = std::min(a, b), hi = std::max(a, b);
      if (hi <= lo + lo / 8) set[m++] = b;  // within 12 %
    }
    if (m < 2) continue;
    // the median of the agreeing intervals, not their mean: a scrape 8 ms late (a pause between
    // a benchmark's warm-up and its timed window) agrees within 12 %, and averaged in it moved
    // the next four expected arrivals 2 ms late -- past the pre-wake lead, so the driver's
    // 20-scrape runs lost their first 5 pre-wakes (profiles/r06/session3: "00000111...")
    std::sort(set, set + m);
    return m % 2 ? set[m / 2] : (set[m / 2 - 1] + set[m / 2]) / 2;
  }
  return 0;
}

const char* prewake_mode_name(int mode) {
  switch (mode) {
    case kPrewakeSlices: return "slices";
    case kPrewakeSpin: return "spin";
    default: return "off";
  }
}

int parse_prewake_mode(const std::string& s) {
  std::string v;
  for (char ch : s) v.push_back(char(::tolower(static_cast<unsigned char>(ch))));
  if (v == "off" || v == "false" || v == "0" || v == "no" || v.empty()) return kPrewakeOff;
  if (v == "slices" || v == "true" || v == "on" || v == "1" || v == "yes") return kPrewakeSlices;
  if (v == "spin") return kPrewakeSpin;
  return -1;
}

const std::vector<double>& scrape_latency_bounds() {
  // fine where scrapes sit (server side: a few to a few tens of microseconds), coarse above
  static const std::vector<double> b = {1e-6,   2e-6,   3e-6,   5e-6,   7.5e-6, 10e-6,  15e-6, 20e-6,
                                        25e-6,  35e-6,  50e-6,  75e-6,  100e-6, 250e-6, 500e-6, 1e-3,
                                        2.5e-3, 5e-3,   10e-3,  25e-3,  100e-3, 250e-3, 1.0};
  static_assert(HttpStats::kBuckets == 23, "bucket count");
  return b;
}

void HttpStats::record_latency(uint64_t ns) {
  const auto& b = scrape_latency_bounds();
  double s = double(ns) * 1e-9;
  int i = 0;
  while (i < kBuckets && s > b[size_t(i)]) ++i;
  lat_buckets[i].fetch_add(1, std::memory_order_relaxed);
  lat_sum_ns.fetch_add(ns, std::memory_order_relaxed);
  lat_count.fetch_add(1, std::memory_order_relaxed);
}

namespace {

struct Conn {
  int fd = -1;
  std::string in;
  std::string head;
  SnapshotStore::Pin pin;
  const char* body = nullptr;
  size_t body_len = 0;
  std::string owned_body;  // small non-snapshot bodies
  size_t sent = 0;         // bytes of head+body already written
  bool pending = false;
  bool close_after = false;
  bool is_metrics = false;
  bool gzip_client = false;  // its last /metrics request accepted gzip
  uint64_t last_active_ns = 0;
  uint64_t req_start_ns = 0;
  // Every socket carries kernel receive timestamps (SO_TIMESTAMPNS): rx_mono_ns is when the
  // kernel queued the last bytes read (CLOCK_MONOTONIC) -- the request's arrival for the
  // learnt scrape schedule, and (X-Gpuexp-Timing) the split of "request sent -> parsed" into
  // loopback delivery and this server's wake-up + read.
  bool rx_ts = false;
  uint64_t rx_mono_ns = 0;
  // arrival times of this connection's /metrics requests: the scrape period, learnt
  uint64_t last_metrics_ns = 0;
  uint64_t intervals[4] = {0, 0, 0, 0};
  int n_intervals = 0, iv_pos = 0;
  // Expected next /metrics arrival, or 0 when the scrape period is not steady.  The period is
  // the newest of the last (up to 4) intervals that another of them agrees with within 12 %
  // (>= 20 ms), averaged with its partners: two steady periods arm it (a scraper's third
  // request is already pre-woken), and one odd interval (a late scrape, a pause between a
  // benchmark's warm-up and its timed window) no longer disarms it -- with "the two newest
  // must agree" it cost the next two requests their pre-wake (18 of 20 timed scrapes
  // pre-woken in every round-4 driver-form run).  A real period change is learnt after two
  // intervals at the new period.
  uint64_t period_ns() const {
    uint64_t newest_first[4];
    const int n = std::min(n_intervals, 4);
    for (int k = 0; k < n; ++k) newest_first[k] = intervals[(iv_pos + 3 - k) & 3];
    return learnt_scrape_period_ns(newest_first, n);
  }
  uint64_t expected_next() const {
    if (n_intervals < 2) return 0;
    const uint64_t p = period_ns();
    return p ? last_metrics_ns + p : 0;
  }
  // How early the next request may come: twice the largest deviation from the period among
  // the intervals that agree with it (a scraper whose requests wander by 1 ms needs the
  // worker awake 1-2 ms ahead; a steady one keeps the minimum lead; an outlier interval that
  // does not agree with the period does not widen it).
  uint64_t jitter_lead(uint64_t min_lead, uint64_t max_lead) const {
    const uint64_t p = n_intervals >= 2 ? period_ns() : 0;
    if (!p) return min_lead;
    uint64_t dev = 0;
    for (int j = 0; j < std::min(n_intervals, 4); ++j) {
      const uint64_t b = intervals[(iv_pos + 3 - j) & 3];
      const uint64_t d = b > p ? b - p : p - b;
      if (d <= p / 8) dev = std::max(dev, d);
    }
    return std::clamp<uint64_t>(2 * dev, min_lead, max_lead);
  }
  ArrivalPredictor pred;  // spin pre-wake: where the next request lands
};

bool ieq_prefix(const char* a, size_t alen, const char* b) {
  size_t bl = std::strlen(b);
  if (alen < bl) return false;
  for (size_t i = 0; i < bl; ++i) {
    char x = a[i], y = b[i];
    if (x >= 'A' && x <= 'Z') x = char(x - 'A' + 'a');
    if (y >= 'A' && y <= 'Z') y = char(y - 'A' + 'a');
    if (x != y) return false;
  }
  return true;
}

bool contains_token(const char* s, size_t n, const char* tok) {
  size_t tl = std::strlen(tok);
  for (size_t i = 0; i + tl <= n; ++i)
    if (ieq_prefix(s + i, n - i, tok)) return true;
  return false;
}

// Accept-header negotiation between the text 0.0.4 exposition and client_golang's
// delimited protobuf (expfmt.Negotiate): protobuf wins only when the client lists
// `application/vnd.google.protobuf` with proto=io.prometheus.client.MetricFamily and
// encoding=delimited at a q no lower than the best text/plain (or wildcard) entry.
bool prefers_protobuf(const char* s, size_t n) {
  double q_pb = -1, q_text = -1;
  std::string h(s, n);
  size_t pos = 0;
  while (pos <= h.size()) {
    size_t comma = h.find(',', pos);
    if (comma == std::string::npos) comma = h.size();
    std::string e = h.substr(pos, comma - pos);
    pos = comma + 1;
    for (auto& ch : e) ch = char(::tolower(static_cast<unsigned char>(ch)));
    double q = 1.0;
    size_t qp = e.find(";q=");
    if (qp == std::string::npos) qp = e.find("; q=");
    if (qp != std::string::npos) q = std::atof(e.c_str() + e.find('=', qp) + 1);
    if (e.find("application/vnd.google.protobuf") != std::string::npos) {
      if (e.find("proto=io.prometheus.client.metricfamily") != std::string::npos &&
          e.find("encoding=delimited") != std::string::npos)
        q_pb = std::max(q_pb, q);
    } else if (e.find("text/plain") != std::string::npos || e.find("*/*") != std::string::npos) {
      q_text = std::max(q_text, q);
    }
  }
  return q_pb > 0 && q_pb >= q_text;
}

}  // namespace

struct HttpServer::Worker {
  int index = 0;
  int listen_fd = -1;
  int epfd = -1;
  int stopfd = -1;
  int timerfd = -1;  // scrape pre-wake
  int kickfd = -1;   // set_prewake_mode: re-arm now
  uint64_t armed_at = 0;  // absolute expiry the timer is armed for (0 = disarmed)
  std::thread th;
  std::unordered_map<int, Conn> conns;
  int pinned_cpu = -1;  // follow_rx_cpu: the CPU this worker is pinned to (-1: its own mask)
  cpu_set_t own_mask;   // the thread's affinity at start
  bool have_mask = false;
};

HttpServer::HttpServer(SnapshotStore* store, const HttpConfig& cfg) : store_(store), cfg_(cfg) {}

HttpServer::~HttpServer() { stop(); }

// host "" = every interface: an IPv6 socket with IPV6_V6ONLY off accepts IPv4 too (what
// Go's ListenAndServe(":8000") does, main.go:71), falling back to IPv4 0.0.0.0 when the
// node has IPv6 disabled.  A literal with ':' binds that IPv6 address; otherwise IPv4.
static int make_listener(const std::string& host, int port, bool reuseport, std::string* err) {
  const bool any = host.empty();
  const bool v6 = any || host.find(':') != std::string::npos;
  int fd = ::socket(v6 ? AF_INET6 : AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0 && any) return make_listener("0.0.0.0", port, reuseport, err);
  if (fd < 0) {
    *err = std::string("socket: ") + std::strerror(errno);
    return -1;
  }
  int one = 1, zero = 0;
  ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (reuseport) ::setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
  sockaddr_storage ss{};
  socklen_t len = 0;
  if (v6) {
    ::setsockopt(fd, IPPROTO_IPV6, IPV6_V6ONLY, &zero, sizeof(zero));
    auto* a6 = reinterpret_cast<sockaddr_in6*>(&ss);
    a6->sin6_family = AF_INET6;
    a6->sin6_port = htons(uint16_t(port));
    a6->sin6_addr = in6addr_any;
    if (!any && ::inet_pton(AF_INET6, host.c_str(), &a6->sin6_addr) != 1) {
      *err = "bad listen host: " + host;
      ::close(fd);
      return -1;
    }
    len = sizeof(sockaddr_in6);
  } else {
    auto* a4 = reinterpret_cast<sockaddr_in*>(&ss);
    a4->sin_family = AF_INET;
    a4->sin_port = htons(uint16_t(port));
    if (::inet_pton(AF_INET, host.c_str(), &a4->sin_addr) != 1) {
      *err = "bad listen host: " + host;
      ::close(fd);
      return -1;
    }
    len = sizeof(sockaddr_in);
  }
  if (::bind(fd, reinterpret_cast<sockaddr*>(&ss), len) < 0) {
    const int e = errno;
    ::close(fd);
    if (any && (e == EAFNOSUPPORT || e == EADDRNOTAVAIL)) return make_listener("0.0.0.0", port, reuseport, err);
    *err = "bind " + (any ? std::string("[::]") : host) + ":" + std::to_string(port) + ": " + std::strerror(e);
    return -1;
  }
  if (::listen(fd, 1024) < 0) {
    *err = std::string("listen: ") + std::strerror(errno);
    ::close(fd);
    return -1;
  }
  return fd;
}

bool HttpServer::start(std::string* err) {
  if (running_.load()) return true;
  int nthreads = std::min(kMaxWorkers, std::max(1, cfg_.threads));
  int port = cfg_.port;
  for (int t = 0; t < nthreads; ++t) {
    auto w = std::make_unique<Worker>();
    w->index = t;
    w->listen_fd = make_listener(cfg_.host, port, nthreads > 1, err);
    if (w->listen_fd < 0) {
      stop();
      return false;
    }
    if (t == 0) {
      sockaddr_storage a{};
      socklen_t al = sizeof(a);
      ::getsockname(w->listen_fd, reinterpret_cast<sockaddr*>(&a), &al);
      bound_port_ = a.ss_family == AF_INET6 ? ntohs(reinterpret_cast<sockaddr_in6*>(&a)->sin6_port)
                                            : ntohs(reinterpret_cast<sockaddr_in*>(&a)->sin_port);
      port = bound_port_;
    }
    w->epfd = ::epoll_create1(EPOLL_CLOEXEC);
    w->stopfd = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = w->listen_fd;
    ::epoll_ctl(w->epfd, EPOLL_CTL_ADD, w->listen_fd, &ev);
    ev.data.fd = w->stopfd;
    ::epoll_ctl(w->epfd, EPOLL_CTL_ADD, w->stopfd, &ev);
    // the pre-wake timer and the kick exist in every mode: the mode is switched at run time
    w->timerfd = ::timerfd_create(CLOCK_MONOTONIC, TFD_NONBLOCK | TFD_CLOEXEC);
    if (w->timerfd >= 0) {
      ev.data.fd = w->timerfd;
      ::epoll_ctl(w->epfd, EPOLL_CTL_ADD, w->timerfd, &ev);
    }
    w->kickfd = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (w->kickfd >= 0) {
      ev.data.fd = w->kickfd;
      ::epoll_ctl(w->epfd, EPOLL_CTL_ADD, w->kickfd, &ev);
    }
    workers_.push_back(std::move(w));
  }
  prewake_mode_.store(cfg_.prewake_mode, std::memory_order_relaxed);
  running_.store(true);
  for (auto& w : workers_) {
    Worker* wp = w.get();
    wp->th = std::thread([this, wp] { run(wp); });
  }
  return true;
}

void HttpServer::stop() {
  for (auto& w : workers_) {
    if (w->stopfd >= 0) {
      uint64_t one = 1;
      ssize_t r = ::write(w->stopfd, &one, sizeof(one));
      (void)r;
    }
  }
  for (auto& w : workers_) {
    if (w->th.joinable()) w->th.join();
    for (auto& kv : w->conns) ::close(kv.first);
    w->conns.clear();
    if (w->listen_fd >= 0) ::close(w->listen_fd);
    if (w->epfd >= 0) ::close(w->epfd);
    if (w->stopfd >= 0) ::close(w->stopfd);
    if (w->timerfd >= 0) ::close(w->timerfd);
    if (w->kickfd >= 0) ::close(w->kickfd);
  }
  workers_.clear();
  running_.store(false);
}

void HttpServer::set_prewake_mode(int mode) {
  if (mode < kPrewakeOff || mode > kPrewakeSpin) return;
  prewake_mode_.store(mode, std::memory_order_relaxed);
  for (auto& w : workers_) {
    if (w->kickfd < 0) continue;
    uint64_t one = 1;
    ssize_t r = ::write(w->kickfd, &one, sizeof(one));
    (void)r;
  }
}

bool HttpServer::gzip_due(uint64_t now_ns, uint64_t horizon_ns) const {
  const uint64_t u = gzip_unsteady_ns_.load(std::memory_order_relaxed);
  if (u && now_ns < u + cfg_.gzip_unsteady_hold_ns) return true;
  for (const auto& g : gzip_next_ns_) {
    const uint64_t e = g.load(std::memory_order_relaxed);
    if (e && e <= now_ns + horizon_ns) return true;
  }
  return false;
}

bool HttpServer::render_due(uint64_t now_ns, uint64_t horizon_ns) const {
  if (!metrics_seen_ns_.load(std::memory_order_relaxed)) return true;
  for (const auto& a : unsteady_ns_) {
    const uint64_t u = a.load(std::memory_order_relaxed);
    if (u && now_ns < u + cfg_.gzip_unsteady_hold_ns) return true;
  }
  bool steady = false;
  for (const auto& g : scrape_next_ns_) {
    const uint64_t e = g.load(std::memory_order_relaxed);
    if (!e) continue;
    steady = true;
    if (e <= now_ns + horizon_ns) return true;
  }
  return !steady;
}

void HttpServer::run(Worker* w) {
  set_thread_name("gpuexp-http");
  if (cfg_.follow_rx_cpu) {
    CPU_ZERO(&w->own_mask);
    w->have_mask = ::sched_getaffinity(0, sizeof(w->own_mask), &w->own_mask) == 0;
  }
  // follow_rx_cpu: after a steady connection's /metrics response, move to the CPU its
  // requests arrive on; with no (or several) steady connections, back to the own mask
  auto follow_rx = [&](const Conn* steady) {
    if (!w->have_mask) return;
    int cpu = -1;
    if (steady) {
      socklen_t len = sizeof(cpu);
      if (::getsockopt(steady->fd, SOL_SOCKET, SO_INCOMING_CPU, &cpu, &len) != 0 || cpu < 0 ||
          cpu >= CPU_SETSIZE || !CPU_ISSET(cpu, &w->own_mask))
        cpu = -1;
    }
    if (cpu == w->pinned_cpu) return;
    if (cpu >= 0) {
      cpu_set_t one;
      CPU_ZERO(&one);
      CPU_SET(cpu, &one);
      if (::sched_setaffinity(0, sizeof(one), &one) != 0) return;
      stats_.rx_cpu_moves.fetch_add(1, std::memory_order_relaxed);
    } else if (::sched_setaffinity(0, sizeof(w->own_mask), &w->own_mask) != 0) {
      return;
    }
    w->pinned_cpu = cpu;
  };
  auto follow_steady = [&]() {
    const Conn* steady = nullptr;
    int n_steady = 0;
    for (auto& kv : w->conns)
      if (kv.second.expected_next()) {
        steady = &kv.second;
        ++n_steady;
      }
    follow_rx(n_steady == 1 ? steady : nullptr);
  };
  constexpr int kMaxEvents = 256;
  epoll_event events[kMaxEvents];
  char rbuf[16384];
  uint64_t last_sweep = mono_ns();
  uint64_t last_prewake_ns = 0;  // this worker's last pre-wake timer expiry
  bool spin_poll = false;        // the events being handled came from a spin poll
  uint64_t spin_until = 0, spin_started = 0;  // spin mode: the window being polled (0 = none)
  bool metrics_seen = false;     // a /metrics request was parsed in this batch of events

  bool refollow = false;  // follow_rx_cpu: a connection closed, re-check the pinning
  auto close_conn = [&](int fd) {
    ::epoll_ctl(w->epfd, EPOLL_CTL_DEL, fd, nullptr);
    ::close(fd);
    w->conns.erase(fd);
    stats_.open_conns.fetch_sub(1, std::memory_order_relaxed);
    refollow = cfg_.follow_rx_cpu;
  };

  // Writes as much of the pending response as the socket takes.  Returns false if the
  // connection must be closed.
  auto flush = [&](Conn& c) -> bool {
    while (c.pending) {
      size_t hl = c.head.size();
      iovec iov[2];
      int n = 0;
      if (c.sent < hl) {
        iov[n].iov_base = const_cast<char*>(c.head.data() + c.sent);
        iov[n].iov_len = hl - c.sent;
        ++n;
        if (c.body_len) {
          iov[n].iov_base = const_cast<char*>(c.body);
          iov[n].iov_len = c.body_len;
          ++n;
        }
      } else {
        size_t off = c.sent - hl;
        iov[n].iov_base = const_cast<char*>(c.body + off);
        iov[n].iov_len = c.body_len - off;
        ++n;
      }
      const uint64_t tw = mono_ns();
      ssize_t wr = ::writev(c.fd, iov, n);
      stats_.writev_ns.fetch_add(mono_ns() - tw, std::memory_order_relaxed);
      stats_.writev_calls.fetch_add(1, std::memory_order_relaxed);
      if (wr < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
          stats_.partial_writes.fetch_add(1, std::memory_order_relaxed);
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLOUT;
          ev.data.fd = c.fd;
          ::epoll_ctl(w->epfd, EPOLL_CTL_MOD, c.fd, &ev);
          return true;
        }
        stats_.errors.fetch_add(1, std::memory_order_relaxed);
        return false;
      }
      c.sent += size_t(wr);
      stats_.bytes_sent.fetch_add(uint64_t(wr), std::memory_order_relaxed);
      if (c.sent >= hl + c.body_len) {
        c.pending = false;
        if (c.is_metrics) stats_.record_latency(mono_ns() - c.req_start_ns);
        c.pin.release();
        c.owned_body.clear();
        c.body = nullptr;
        c.body_len = 0;
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.fd = c.fd;
        ::epoll_ctl(w->epfd, EPOLL_CTL_MOD, c.fd, &ev);
        if (c.close_after) return false;
      }
    }
    return true;
  };

  auto respond_simple = [&](Conn& c, int code, const char* reason, const std::string& ctype,
                            std::string body, bool head_only) {
    c.owned_body = std::move(body);
    c.head = "HTTP/1.1 " + std::to_string(code) + " " + reason + "\r\nContent-Type: " + ctype +
             "\r\nContent-Length: " + std::to_string(c.owned_body.size()) + "\r\n" +
             (c.close_after ? "Connection: close\r\n" : "") + "\r\n";
    c.body = head_only ? nullptr : c.owned_body.data();
    c.body_len = head_only ? 0 : c.owned_body.size();
    c.sent = 0;
    c.pending = true;
    c.is_metrics = false;
  };

  // Parses and answers every complete request in the input buffer (in order; a
  // pipelined request waits until the previous response is fully written).
  auto handle_input = [&](Conn& c) -> bool {
    while (!c.pending) {
      size_t end = c.in.find("\r\n\r\n");
      if (end == std::string::npos) {
        if (c.in.size() > 16384) return false;  // header too large
        return true;
      }
      uint64_t t0 = mono_ns();
      const char* p = c.in.data();
      size_t hdr_len = end + 4;
      size_t le = c.in.find("\r\n");
      std::string line(p, le);
      size_t s1 = line.find(' ');
      size_t s2 = line.find(' ', s1 == std::string::npos ? 0 : s1 + 1);
      std::string method, target, version;
      if (s1 != std::string::npos && s2 != std::string::npos) {
        method = line.substr(0, s1);
        target = line.substr(s1 + 1, s2 - s1 - 1);
        version = line.substr(s2 + 1);
      }
      bool http10 = version == "HTTP/1.0";
      bool want_gzip = false, want_proto = false, conn_close = http10, conn_keep = false, want_timing = false;
      uint64_t content_len = 0;
      size_t pos = le + 2;
      while (pos < end) {
        size_t nl = c.in.find("\r\n", pos);
        if (nl == std::string::npos || nl > end) nl = end;
        const char* h = p + pos;
        size_t hn = nl - pos;
        if (ieq_prefix(h, hn, "accept-encoding:")) {
          want_gzip = contains_token(h + 16, hn - 16, "gzip");
        } else if (ieq_prefix(h, hn, "accept:")) {
          want_proto = prefers_protobuf(h + 7, hn - 7);
        } else if (ieq_prefix(h, hn, "connection:")) {
          if (contains_token(h + 11, hn - 11, "close")) conn_close = true;
          if (contains_token(h + 11, hn - 11, "keep-alive")) conn_keep = true;
        } else if (ieq_prefix(h, hn, "content-length:")) {
          parse_u64(h + 15, hn - 15, &content_len);
        } else if (ieq_prefix(h, hn, "x-gpuexp-timing:")) {
          want_timing = true;  // benchmark breakdown: echo the server's own timestamps
        }
        pos = nl + 2;
      }
      if (content_len > 1 << 20) return false;
      if (c.in.size() < hdr_len + content_len) return true;  // wait for body
      c.in.erase(0, hdr_len + size_t(content_len));
      stats_.requests.fetch_add(1, std::memory_order_relaxed);
      c.close_after = conn_close && !(http10 && conn_keep);
      c.req_start_ns = t0;

      size_t q = target.find('?');
      std::string path = q == std::string::npos ? target : target.substr(0, q);
      bool is_head = method == "HEAD";
      if (method.empty()) {
        c.close_after = true;
        respond_simple(c, 400, "Bad Request", "text/plain", "bad request\n", false);
      } else if (method != "GET" && !is_head) {
        respond_simple(c, 405, "Method Not Allowed", "text/plain", "method not allowed\n", false);
      } else if (path == cfg_.metrics_path) {
        stats_.metrics_requests.fetch_add(1, std::memory_order_relaxed);
        // pre-woken: picked up by a spin poll, or (slices) its timer fired shortly before
        const bool timer_woken = last_prewake_ns && t0 >= last_prewake_ns &&
                                 t0 - last_prewake_ns <= cfg_.prewake_max_lead_ns + cfg_.prewake_step_ns;
        const bool prewoken = spin_poll || (timer_woken && prewake_mode_.load(std::memory_order_relaxed) !=
                                                               kPrewakeOff);
        if (prewoken) stats_.prewake_hits.fetch_add(1, std::memory_order_relaxed);
        if (prewoken && (spin_poll || t0 - last_prewake_ns <= cfg_.prewake_lead_ns + cfg_.prewake_step_ns))
          stats_.prewake_hits_narrow.fetch_add(1, std::memory_order_relaxed);
        metrics_seen = true;
        // The scrape schedule is learnt from ARRIVAL times (the kernel's receive timestamp):
        // parse times would carry this worker's own wake-up delay, which differs per mode and
        // would bias the spin window late, where it then misses and stays biased.
        const uint64_t arrival = c.rx_ts && c.rx_mono_ns && c.rx_mono_ns <= t0 && t0 - c.rx_mono_ns < 100000000ull
                                     ? c.rx_mono_ns : t0;
        c.pred.observe(arrival, c.n_intervals < 2 || c.period_ns() != 0);
        if (c.last_metrics_ns && arrival > c.last_metrics_ns) {
          c.intervals[c.iv_pos] = arrival - c.last_metrics_ns;
          c.iv_pos = (c.iv_pos + 1) & 3;
          if (c.n_intervals < 4) ++c.n_intervals;
        }
        c.last_metrics_ns = arrival;
        c.gzip_client = want_gzip && cfg_.enable_gzip;
        if (c.gzip_client && !c.expected_next()) gzip_unsteady_ns_.store(t0, std::memory_order_relaxed);
        metrics_seen_ns_.store(t0, std::memory_order_relaxed);
        if (!c.expected_next()) unsteady_ns_[w->index].store(t0, std::memory_order_relaxed);  // (at once)
        SnapshotStore::Pin pin = store_->acquire();
        if (!pin) {
          respond_simple(c, 503, "Service Unavailable", "text/plain", "no sample yet\n", is_head);
        } else {
          if (want_gzip && cfg_.enable_gzip) gzip_wanted_ns_.store(t0, std::memory_order_relaxed);
          if (want_proto) proto_wanted_ns_.store(t0, std::memory_order_relaxed);
          // Protobuf once the sampler has rendered it (from the tick after the first ask).
          const bool pb = want_proto && !pin->pb.empty();
          const std::string& plain = pb ? pin->pb : pin->body;
          const std::string& zipped = pb ? pin->pb_gz : pin->gz;
          const bool gz = want_gzip && cfg_.enable_gzip;
          bool own = false;
          if (gz && zipped.empty() && !is_head) {
            // off schedule (or the first ask): compress here, for this response only
            c.owned_body.clear();
            own = gzip_compress(plain, &c.owned_body, cfg_.gzip_level) && !c.owned_body.empty();
            stats_.gzip_on_demand.fetch_add(1, std::memory_order_relaxed);
          }
          const bool use_gz = gz && (own || !zipped.empty());
          const std::string& b = own ? c.owned_body : (use_gz ? zipped : plain);
          c.head.clear();
          if (pb) {
            c.head.append("HTTP/1.1 200 OK\r\nContent-Type: application/vnd.google.protobuf; "
                          "proto=io.prometheus.client.MetricFamily; encoding=delimited\r\n");
            stats_.proto_responses.fetch_add(1, std::memory_order_relaxed);
          } else {
            c.head.append("HTTP/1.1 200 OK\r\nContent-Type: text/plain; version=0.0.4; charset=utf-8\r\n");
          }
          if (use_gz) {
            c.head.append("Content-Encoding: gzip\r\n");
            stats_.gzip_responses.fetch_add(1, std::memory_order_relaxed);
          }
          if (want_timing) {
            // CLOCK_MONOTONIC ns of: request parsed (after this thread woke for it), and
            // response about to be written — a same-host client splits its latency with them —
            // then the pre-woken flag and the kernel's receive time of the request (0 = none)
            c.head.append("X-Gpuexp-Timing: ");
            c.head.append(std::to_string(t0));
            c.head.append(" ");
            c.head.append(std::to_string(mono_ns()));
            c.head.append(prewoken ? " 1 " : " 0 ");
            c.head.append(std::to_string(c.rx_ts ? c.rx_mono_ns : 0));
            c.head.append("\r\n");
          }
          c.head.append("Content-Length: ");
          c.head.append(std::to_string(b.size()));
          c.head.append(c.close_after ? "\r\nConnection: close\r\n\r\n" : "\r\n\r\n");
          c.body = is_head ? nullptr : b.data();
          c.body_len = is_head ? 0 : b.size();
          c.pin = std::move(pin);
          c.sent = 0;
          c.pending = true;
          c.is_metrics = true;
        }
      } else if (path == "/healthz") {
        respond_simple(c, 200, "OK", "text/plain", "ok\n", is_head);
      } else if (path == "/readyz") {
        uint64_t age_ns = 0;
        if (cfg_.stale_after_ns) {
          SnapshotStore::Pin pin = store_->acquire();
          if (pin && pin->published_mono_ns && t0 > pin->published_mono_ns) age_ns = t0 - pin->published_mono_ns;
        }
        if (!ready_.load())
          respond_simple(c, 503, "Service Unavailable", "text/plain", "not ready\n", is_head);
        else if (cfg_.stale_after_ns && age_ns > cfg_.stale_after_ns)
          respond_simple(c, 503, "Service Unavailable", "text/plain",
                         "stale: last sample " + std::to_string(age_ns / 1000000) + " ms ago\n", is_head);
        else
          respond_simple(c, 200, "OK", "text/plain", "ready\n", is_head);
      } else if (path == "/") {
        respond_simple(c, 200, "OK", "text/html",
                       "<html><head><title>MI355X GPU exporter</title></head><body>"
                       "<h1>MI355X per-pod GPU exporter</h1><p><a href=\"" + cfg_.metrics_path +
                           "\">Metrics</a></p></body></html>\n",
                       is_head);
      } else {
        respond_simple(c, 404, "Not Found", "text/plain", "not found\n", is_head);
      }
      const bool was_metrics = c.is_metrics;
      if (!flush(c)) return false;
      if (cfg_.follow_rx_cpu && was_metrics && !c.pending) follow_steady();
    }
    return true;
  };

  ::prctl(PR_SET_TIMERSLACK, 10000UL, 0, 0, 0);  // 10 us: pre-wake timers stay punctual
  // spin mode state: the window being polled (0 = not spinning), when it began, and how late
  // the pre-wake timer fires on this host (EWMA; the timer is armed that much early)
  uint64_t timer_late_ns = 30000;
  auto set_timer = [&](uint64_t at) {
    if (w->timerfd < 0 || at == w->armed_at) return;
    itimerspec its{};
    its.it_value.tv_sec = time_t(at / 1000000000ull);
    its.it_value.tv_nsec = long(at % 1000000000ull);
    ::timerfd_settime(w->timerfd, TFD_TIMER_ABSTIME, &its, nullptr);  // zero disarms
    w->armed_at = at;
  };
  // Arms the pre-wake for the earliest expected scrape (see HttpConfig::prewake_mode); in
  // spin mode, starts spinning when its window is (about to be) open.
  auto arm_prewake = [&]() {
    const uint64_t now = mono_ns();
    const int mode = prewake_mode_.load(std::memory_order_relaxed);
    uint64_t next = 0, gz_next = 0, any_next = 0, unsteady = 0, lead = cfg_.prewake_lead_ns;
    uint64_t sp_from = 0, sp_until = 0;
    for (auto& kv : w->conns) {
      const uint64_t e = kv.second.expected_next();
      uint64_t f, u;
      if (e && mode == kPrewakeSpin &&
          kv.second.pred.window(cfg_.prewake_spin_max_ns, cfg_.prewake_spin_margin_ns, &f, &u)) {
        if (u > now && (!sp_from || f < sp_from)) {
          sp_from = f;
          sp_until = u;
        }
      }
      if (e && e + cfg_.prewake_window_ns > now && (!next || e < next)) {
        next = e;
        lead = kv.second.jitter_lead(cfg_.prewake_lead_ns, cfg_.prewake_max_lead_ns);
      }
      // a steady gzip scraper gone quiet for a minute no longer holds the sampler to it
      if (e && kv.second.gzip_client && e + 60000000000ull > now && (!gz_next || e < gz_next)) gz_next = e;
      if (e && e + 60000000000ull > now && (!any_next || e < any_next)) any_next = e;
      if (!e && kv.second.last_metrics_ns) unsteady = std::max(unsteady, kv.second.last_metrics_ns);
    }
    unsteady_ns_[w->index].store(unsteady, std::memory_order_relaxed);
    gzip_next_ns_[w->index].store(gz_next, std::memory_order_relaxed);
    scrape_next_ns_[w->index].store(any_next, std::memory_order_relaxed);
    uint64_t at = 0;
    if ((mode == kPrewakeSlices || mode == kPrewakeSpin) && next) {
      // before the lead: one timer at (expected - lead); inside the window: short slices
      at = now + lead < next ? next - lead : now + cfg_.prewake_step_ns;
    }
    if (mode == kPrewakeSpin && sp_from) {
      // spin = slices + polling inside the predicted arrival window: a request before the
      // window or after it still finds a shallow-idle worker (the slices), one inside it an
      // on-CPU worker
      if (now + timer_late_ns >= sp_from) {  // the window is open (or opens before a timer could fire)
        spin_until = sp_until;
        spin_started = now;
        stats_.prewake_spins.fetch_add(1, std::memory_order_relaxed);
        at = 0;
      } else if (!at || sp_from - timer_late_ns < at) {
        at = sp_from - timer_late_ns;
      }
    }
    set_timer(at);
  };
  auto end_spin = [&](bool hit) {
    stats_.prewake_spin_ns.fetch_add(mono_ns() - spin_started, std::memory_order_relaxed);
    (hit ? stats_.prewake_spin_hits : stats_.prewake_spin_timeouts).fetch_add(1, std::memory_order_relaxed);
    spin_until = 0;
  };

  for (;;) {
    int timeout_ms = 1000;
    if (spin_until) {
      if (mono_ns() >= spin_until || prewake_mode_.load(std::memory_order_relaxed) != kPrewakeSpin) {
        end_spin(false);
        continue;
      }
      timeout_ms = 0;  // poll: the request finds this thread on-CPU
    } else {
      if (refollow) {  // the steady scraper may be gone: unpin (or follow the one left)
        refollow = false;
        follow_steady();
      }
      arm_prewake();
      if (spin_until) continue;
    }
    int n = ::epoll_wait(w->epfd, events, kMaxEvents, timeout_ms);
    if (n < 0 && errno != EINTR) break;
    if (n <= 0 && spin_until) {
      for (int k = 0; k < 32; ++k) _mm_pause();
      continue;
    }
    spin_poll = spin_until != 0;
    metrics_seen = false;
    bool stopping = false;
    for (int i = 0; i < n; ++i) {
      int fd = events[i].data.fd;
      if (fd == w->stopfd) {
        stopping = true;
        continue;
      }
      if (fd == w->kickfd) {  // mode switched: the loop re-arms
        uint64_t v = 0;
        ssize_t r = ::read(w->kickfd, &v, sizeof(v));
        (void)r;
        set_timer(0);
        continue;
      }
      if (fd == w->timerfd) {
        uint64_t expirations = 0;
        ssize_t r = ::read(w->timerfd, &expirations, sizeof(expirations));
        (void)r;
        stats_.prewake_timer_wakeups.fetch_add(1, std::memory_order_relaxed);
        last_prewake_ns = mono_ns();
        if (w->armed_at && prewake_mode_.load(std::memory_order_relaxed) == kPrewakeSpin) {
          const uint64_t late = last_prewake_ns > w->armed_at ? last_prewake_ns - w->armed_at : 0;
          timer_late_ns = std::clamp<uint64_t>((timer_late_ns * 7 + std::min<uint64_t>(late, 200000)) / 8,
                                               2000, 100000);
        }
        w->armed_at = 0;  // fired: a re-arm to the same time must reach the kernel
        continue;
      }
      if (fd == w->listen_fd) {
        for (;;) {
          int cfd = ::accept4(w->listen_fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (cfd < 0) break;
          if (int(w->conns.size()) >= cfg_.max_conns) {
            ::close(cfd);
            stats_.errors.fetch_add(1, std::memory_order_relaxed);
            continue;
          }
          int one = 1;
          ::setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          if (cfg_.socket_sndbuf > 0)
            ::setsockopt(cfd, SOL_SOCKET, SO_SNDBUF, &cfg_.socket_sndbuf, sizeof(cfg_.socket_sndbuf));
          Conn& c = w->conns[cfd];
          c.fd = cfd;
          // kernel receive timestamps on every connection: request arrival times for the
          // scrape schedule (pre-wake) and the benchmark's latency split
          c.rx_ts = ::setsockopt(cfd, SOL_SOCKET, SO_TIMESTAMPNS, &one, sizeof(one)) == 0;
          c.last_active_ns = mono_ns();
          epoll_event ev{};
          ev.events = EPOLLIN;
          ev.data.fd = cfd;
          ::epoll_ctl(w->epfd, EPOLL_CTL_ADD, cfd, &ev);
          stats_.accepted.fetch_add(1, std::memory_order_relaxed);
          stats_.open_conns.fetch_add(1, std::memory_order_relaxed);
        }
        continue;
      }
      auto it = w->conns.find(fd);
      if (it == w->conns.end()) continue;
      Conn& c = it->second;
      c.last_active_ns = mono_ns();
      bool ok = true;
      if (events[i].events & (EPOLLERR | EPOLLHUP)) ok = false;
      if (ok && (events[i].events & EPOLLOUT)) {
        ok = flush(c);
        // A response that completed here may have pipelined requests queued behind it
        // whose bytes were read long ago: no EPOLLIN will come for them.
        if (ok && !c.pending && !c.in.empty() && !(events[i].events & EPOLLIN)) ok = handle_input(c);
      }
      if (ok && (events[i].events & EPOLLIN)) {
        for (;;) {
          ssize_t r;
          if (c.rx_ts) {  // recvmsg for the receive timestamp
            iovec iov{rbuf, sizeof(rbuf)};
            alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(timespec))];
            msghdr mh{};
            mh.msg_iov = &iov;
            mh.msg_iovlen = 1;
            mh.msg_control = cbuf;
            mh.msg_controllen = sizeof(cbuf);
            r = ::recvmsg(fd, &mh, 0);
            for (cmsghdr* cm = r > 0 ? CMSG_FIRSTHDR(&mh) : nullptr; cm; cm = CMSG_NXTHDR(&mh, cm)) {
              if (cm->cmsg_level != SOL_SOCKET || cm->cmsg_type != SCM_TIMESTAMPNS) continue;
              timespec ts;
              std::memcpy(&ts, CMSG_DATA(cm), sizeof(ts));
              timespec rt;
              clock_gettime(CLOCK_REALTIME, &rt);
              const int64_t now_real = int64_t(rt.tv_sec) * 1000000000ll + rt.tv_nsec;
              const int64_t rx_real = int64_t(ts.tv_sec) * 1000000000ll + ts.tv_nsec;
              c.rx_mono_ns = uint64_t(int64_t(mono_ns()) - (now_real - rx_real));  // same instant, other clock
            }
          } else {
            r = ::read(fd, rbuf, sizeof(rbuf));
          }
          if (r > 0) {
            c.in.append(rbuf, size_t(r));
            if (size_t(r) < sizeof(rbuf)) break;
            continue;
          }
          if (r == 0) ok = false;
          else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) ok = false;
          break;
        }
        if (ok || !c.in.empty()) {
          bool hok = handle_input(c);
          ok = ok && hok;
        }
      }
      if (!ok) close_conn(fd);
    }
    if (spin_until && metrics_seen) end_spin(true);
    spin_poll = false;
    if (stopping) break;
    uint64_t now = mono_ns();
    if (now - last_sweep > 1000000000ull) {
      last_sweep = now;
      std::vector<int> idle;
      for (auto& kv : w->conns)
        if (now - kv.second.last_active_ns > uint64_t(cfg_.idle_timeout_ms) * 1000000ull)
          idle.push_back(kv.first);
      for (int fd : idle) close_conn(fd);
    }
  }
}

}  // namespace gpuexp
