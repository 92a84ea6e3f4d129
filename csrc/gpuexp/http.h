// Minimal epoll HTTP/1.1 server for /metrics, /healthz, /readyz.
//
// Reference: `http.Handle("/metrics", promhttp.HandlerFor(reg, ...))` +
// `ListenAndServe(":8000")` in a goroutine (/root/reference/main.go:67-72), fatal on
// bind error.  Here: one (or N, SO_REUSEPORT) event-loop thread(s) that never render —
// a request pins the current snapshot and writev()s pre-built bytes, so scrape latency
// is O(bytes) and independent of GPU I/O.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "gpuexp/snapshot.h"

namespace gpuexp {

enum PrewakeMode : int { kPrewakeOff = 0, kPrewakeSlices = 1, kPrewakeSpin = 2 };
const char* prewake_mode_name(int mode);
int parse_prewake_mode(const std::string& s);  // off|slices|spin (true/on = slices); -1 = invalid

struct HttpConfig {
  std::string host;  // "" = every interface, dual-stack (see make_listener)
  int port = 8000;                     // main.go:71 ":8000"; 0 = ephemeral
  std::string metrics_path = "/metrics";  // main.go:70
  int threads = 1;
  int max_conns = 4096;
  int idle_timeout_ms = 120000;
  bool enable_gzip = true;
  // how long a gzip request from a connection without a steady scrape period keeps the
  // sampler pre-compressing every tick (see gzip_due)
  uint64_t gzip_unsteady_hold_ns = 60000000000ull;
  int gzip_level = 1;  // of responses the worker compresses itself (EngineConfig::gzip_level for the sampler's)
  // Send buffer of accepted sockets.  A fresh TCP socket starts at tcp_wmem[1] (16 KiB),
  // so a 30-200 KB exposition could not be queued by one writev: the rest waited for the
  // peer's ACK and an EPOLLOUT wake-up — measured +25 us p50 for a 26 KB body on loopback.
  // The kernel clamps this to net.core.wmem_max.
  int socket_sndbuf = 4 << 20;
  // /readyz answers 503 once the newest snapshot is older than this (a sampler stuck in a
  // driver call, e.g. an SMU timeout during a GPU reset): Kubernetes then takes the pod
  // out of the Service instead of Prometheus ingesting frozen values as current.  0 = off.
  uint64_t stale_after_ns = 0;
  // Scrape-phase pre-wake.  Prometheus scrapes a target at a fixed interval, so once a
  // connection's /metrics requests arrive at a steady period (>= 20 ms) the worker can be
  // awake when the next one lands instead of paying a wake-up from an idle epoll_wait on the
  // critical path (the `socket_queue_to_parsed` part of a scrape).  Modes (runtime-switchable,
  // HttpServer::set_prewake_mode):
  //   off     block in epoll_wait until the request arrives;
  //   slices  arm a timer prewake_lead_ns before the expected request, then sleep in
  //           prewake_step_ns slices until it arrives (at most prewake_window_ns late):
  //           shallow idle, but each request still pays a timer-to-epoll wake-up;
  //   spin    slices, plus: from each connection's recent arrival errors (ArrivalPredictor)
  //           a window [expected + lo - margin, expected + hi + margin] no longer than
  //           prewake_spin_max_ns, entered by a timer just before it (the timer's own measured
  //           lateness ahead), in which the worker polls the epoll set with a zero timeout +
  //           pause until the request arrives or the window ends.  A request inside the window
  //           finds the worker on-CPU (no wake-up at all); one before or after it still finds
  //           the slices' shallow-idle worker.  CPU cost = the window actually spun (the
  //           arrival jitter) + the slices' few timer wake-ups.
  //           Round 6 A/B (profiles/r06/): spin alone (no slices around the window) reached
  //           86 % hits; slices 98.8 %.
  // The default, slices, is what an interleaved in-process A/B chose (bench.py --prewake-ab,
  // 400 scrapes per arm, block bootstrap; profiles/r06/prewake_ab.md): socket_queue_to_parsed
  // p50 20.1 -> 5.8 us at +0.023 pt exporter CPU, 98.8 % of scrapes pre-woken; spin's p50 was
  // no better than slices' (CI of the difference spans 0) at twice the extra CPU.
  int prewake_mode = 1;  // PrewakeMode (kPrewakeSlices)
  uint64_t prewake_lead_ns = 400000;       // slices: at least; twice the connection's period jitter,
  uint64_t prewake_max_lead_ns = 1500000;  // ... at most
  uint64_t prewake_step_ns = 150000;
  uint64_t prewake_window_ns = 3000000;
  uint64_t prewake_spin_max_ns = 300000;    // spin: longest window (and the window before 4 errors are known)
  uint64_t prewake_spin_margin_ns = 15000;  // spin: slack on both sides of the observed error range
  // Serve a steady scraper from the CPU its requests arrive on (SO_INCOMING_CPU: where the
  // kernel ran the receive path, the NIC queue's CPU, or the client's own for loopback): the
  // worker is pinned there while exactly one steady /metrics connection is open, so the
  // request's receive wakes it without a cross-CPU wake-up.  Env GPUEXP_HTTP_FOLLOW_RX_CPU.
  bool follow_rx_cpu = false;
};

// The scrape period a connection's pre-wake follows, from its newest (up to 4) request
// intervals, newest first: the newest interval that another one agrees with within 12 % (and
// >= 20 ms), averaged with its partners; 0 = no steady period.
uint64_t learnt_scrape_period_ns(const uint64_t* newest_first, int n);

// Where a steady scraper's next request will arrive (spin pre-wake), predicted two ways from
// the median of the last 16 arrival intervals (one late scrape does not skew it, as it does a
// mean): relative -- the last arrival + the period (a scraper that sleeps a period after each
// scrape, like bench.py) -- and phase-locked -- a schedule phase that follows a quarter of each
// error, + the period (a ticker, like Prometheus' scrape loop, whose late scrape is followed by
// an early one).  Each keeps its last 16 errors (arrival - prediction); the window follows the
// predictor whose errors spread less.
struct ArrivalPredictor {
  int64_t err_rel[16] = {}, err_abs[16] = {};
  int n = 0, pos = 0;
  uint64_t iv[16] = {};
  int n_iv = 0, iv_pos = 0;
  uint64_t phase = 0;  // phase-locked estimate of the last arrival
  uint64_t last = 0;   // last arrival
  // `steady` = the connection's scrape period is steady (else the history restarts)
  void observe(uint64_t arrival, bool steady);
  uint64_t period() const;  // median interval (0 before 4 intervals)
  // [from, until] for the next request: [e + lo - margin, e + hi + margin] with lo / hi the
  // 2nd smallest / largest error of the last 16, trimmed to max_ns around the median; before
  // 8 errors, max_ns centred on the relative prediction.  Returns 0 = no window, 1 = relative,
  // 2 = phase-locked.
  int window(uint64_t max_ns, uint64_t margin, uint64_t* from, uint64_t* until) const;
};

// Fixed latency buckets (seconds) for gpuexp_scrape_duration_seconds.
const std::vector<double>& scrape_latency_bounds();

struct HttpStats {
  static constexpr int kBuckets = 23;
  std::atomic<uint64_t> requests{0};
  std::atomic<uint64_t> metrics_requests{0};
  std::atomic<uint64_t> gzip_responses{0};
  std::atomic<uint64_t> proto_responses{0};
  std::atomic<uint64_t> bytes_sent{0};
  std::atomic<uint64_t> errors{0};
  std::atomic<uint64_t> accepted{0};
  std::atomic<uint64_t> open_conns{0};
  // where a response's time goes: writev() syscalls, and writes the socket only took in
  // part (the rest then waits for EPOLLOUT)
  std::atomic<uint64_t> writev_calls{0};
  std::atomic<uint64_t> writev_ns{0};
  std::atomic<uint64_t> partial_writes{0};
  std::atomic<uint64_t> prewake_timer_wakeups{0};  // timer expiries of the scrape pre-wake
  // /metrics requests parsed while their worker was pre-woken (its pre-wake timer fired
  // within prewake_max_lead_ns + prewake_step_ns before the request): the rest paid a full
  // wake-up from an idle epoll_wait
  std::atomic<uint64_t> prewake_hits{0};
  // the same with round 3's narrower window (timer within prewake_lead_ns + one slice), so hit
  // rates stay comparable across the window change
  std::atomic<uint64_t> prewake_hits_narrow{0};
  // gzip responses the worker compressed itself: the snapshot had no gzip copy because no
  // gzip scrape was expected before the next tick (see HttpServer::gzip_due)
  std::atomic<uint64_t> gzip_on_demand{0};
  std::atomic<uint64_t> rx_cpu_moves{0};  // follow_rx_cpu: worker re-pinned to a new CPU
  // spin pre-wake: windows entered, of which a /metrics request ended them (hit) or the window
  // ran out (timeout), and the wall time spent polling in them (= the CPU the mode costs)
  std::atomic<uint64_t> prewake_spins{0};
  std::atomic<uint64_t> prewake_spin_hits{0};
  std::atomic<uint64_t> prewake_spin_timeouts{0};
  std::atomic<uint64_t> prewake_spin_ns{0};
  std::atomic<uint64_t> lat_buckets[kBuckets + 1]{};  // +Inf last, non-cumulative
  std::atomic<uint64_t> lat_sum_ns{0};
  std::atomic<uint64_t> lat_count{0};
  void record_latency(uint64_t ns);
};

class HttpServer {
 public:
  HttpServer(SnapshotStore* store, const HttpConfig& cfg);
  ~HttpServer();
  HttpServer(const HttpServer&) = delete;
  HttpServer& operator=(const HttpServer&) = delete;

  bool start(std::string* err);
  void stop();
  int port() const { return bound_port_; }
  bool running() const { return running_.load(); }

  void set_ready(bool r) { ready_.store(r); }
  // Last time (mono ns) a client asked for gzip; the sampler pre-compresses while
  // this is recent so gzip scrapes stay O(bytes) too.
  uint64_t gzip_wanted_ns() const { return gzip_wanted_ns_.load(std::memory_order_relaxed); }
  // Whether a snapshot published at `now_ns` should carry a gzip copy: true while a gzip
  // client scrapes without a steady period (within gzip_unsteady_hold_ns), or when a steady
  // gzip client's next request is expected within `horizon_ns` (or is overdue).  Prometheus
  // scraping every 15 s against a 10 Hz sampler thus costs one compression per scrape,
  // not 150; a request that arrives off schedule is compressed by the worker itself.
  bool gzip_due(uint64_t now_ns, uint64_t horizon_ns) const;
  // Whether a snapshot published at `now_ns` will be read: false only while every open /metrics
  // connection that scraped within gzip_unsteady_hold is steady and none is expected within
  // `horizon_ns` (nor overdue).  A process never scraped, an irregular scraper (until its period
  // is learnt), or one that went quiet: true.
  // Prometheus scraping every 15 s against a 10 Hz sampler thus needs a render per scrape, not
  // 150 (the engine still renders at least once a second: EngineConfig::render_when_due).
  bool render_due(uint64_t now_ns, uint64_t horizon_ns) const;
  // Last time a scraper negotiated the protobuf exposition (the sampler renders it then).
  uint64_t proto_wanted_ns() const { return proto_wanted_ns_.load(std::memory_order_relaxed); }
  const HttpStats& stats() const { return stats_; }
  // Switches the pre-wake mode of a running server (PrewakeMode); every worker re-arms at once.
  void set_prewake_mode(int mode);
  int prewake_mode() const { return prewake_mode_.load(std::memory_order_relaxed); }

 private:
  struct Worker;
  void run(Worker* w);

  SnapshotStore* store_;
  HttpConfig cfg_;
  int bound_port_ = -1;
  std::atomic<bool> running_{false};
  std::atomic<bool> ready_{false};
  std::atomic<int> prewake_mode_{1};
  std::atomic<uint64_t> gzip_wanted_ns_{0};
  std::atomic<uint64_t> proto_wanted_ns_{0};
  // last gzip /metrics request from a connection without a steady period
  std::atomic<uint64_t> gzip_unsteady_ns_{0};
  // per worker: earliest expected request of its steady gzip connections (0 = none)
  static constexpr int kMaxWorkers = 64;
  std::atomic<uint64_t> gzip_next_ns_[kMaxWorkers]{};
  // the same for every steady /metrics connection, any encoding (render_due)
  std::atomic<uint64_t> scrape_next_ns_[kMaxWorkers]{};
  std::atomic<uint64_t> metrics_seen_ns_{0};  // last /metrics request (0 = never scraped)
  // per worker: newest /metrics request of its open connections that have no steady period yet
  // (a connection that became steady, or closed, no longer holds renders to every tick)
  std::atomic<uint64_t> unsteady_ns_[kMaxWorkers]{};
  HttpStats stats_;
  std::vector<std::unique_ptr<Worker>> workers_;
};

}  // namespace gpuexp
