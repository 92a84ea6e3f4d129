#include "gpuexp/engine.h"

#include "gpuexp/engine_util.h"

#include <fcntl.h>
#include <sys/eventfd.h>
#include <sys/poll.h>
#include <sys/prctl.h>
#include <sys/timerfd.h>
#include <sys/utsname.h>
#include <unistd.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <set>

namespace gpuexp {

namespace {

// True on an engine's own sampler thread (set in run_sampler): that thread charges its
// whole clock to the sampler account, a manual tick_now() caller only the tick itself.
thread_local bool tl_sampler_thread = false;

}  // namespace

ForkJoinPool::ForkJoinPool(int threads) {
  const size_t n = threads > 1 ? size_t(threads - 1) : 0;
  wcpu_.reset(new std::atomic<uint64_t>[n > 0 ? n : 1]);
  for (size_t t = 0; t < n; ++t) wcpu_[t].store(0);
  for (size_t t = 0; t < n; ++t) workers_.emplace_back([this, t] { worker(t); });
}

uint64_t ForkJoinPool::cpu_ns_total() const {
  uint64_t s = 0;
  for (size_t t = 0; t < workers_.size(); ++t) s += wcpu_[t].load();
  return s;
}

ForkJoinPool::~ForkJoinPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    quit_ = true;
  }
  cv_.notify_all();
  for (auto& w : workers_) w.join();
}

void ForkJoinPool::worker(size_t idx) {
  set_thread_name("gpuexp-dev");
  uint64_t seen = 0;
  for (;;) {
    const std::function<void(int)>* fn;
    int n;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return quit_ || epoch_ != seen; });
      if (quit_) return;
      seen = epoch_;
      fn = fn_;
      n = n_;
    }
    for (int i; (i = next_.fetch_add(1)) < n;) (*fn)(i);
    wcpu_[idx].store(thread_cpu_ns());  // before pending_ drops: run() sees it
    std::lock_guard<std::mutex> lk(mu_);
    pending_ -= 1;
    if (pending_ == 0) done_cv_.notify_all();
  }
}

void ForkJoinPool::run(int n, const std::function<void(int)>& fn) {
  if (workers_.empty() || n <= 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    fn_ = &fn;
    n_ = n;
    next_.store(0);
    pending_ = int(workers_.size());
    ++epoch_;
  }
  cv_.notify_all();
  for (int i; (i = next_.fetch_add(1)) < n;) fn(i);
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return pending_ == 0; });
}

const char* Engine::stage_name(int i) {
  static const char* n[kStages] = {"devices", "processes", "attribution", "sentinel",
                                   "counters", "series", "render", "publish"};
  return n[i];
}

const char* Engine::dev_part_name(int i) {
  static const char* n[kDevParts] = {"counters_kick", "control", "gpu_metrics", "vram", "ras", "gtt"};
  return n[i];
}

Engine::Engine(const EngineConfig& cfg) : cfg_(cfg) { self_pid_ = int(::getpid()); }

Engine::~Engine() { stop(); }

std::vector<std::string> family_labels(const FamilySpec& f) {
  std::vector<std::string> l;
  switch (f.base) {
    case LabelBase::kDevice: l = {"gpu", "bdf", "namespace", "pod", "container"}; break;
    case LabelBase::kProcess: l = {"gpu", "pid", "comm", "namespace", "pod", "container"}; break;
    case LabelBase::kPod: l = {"namespace", "pod"}; break;
    case LabelBase::kNone: break;
  }
  for (const char* e : f.extra) l.emplace_back(e);
  return l;
}

// Continuous counters: the plugin's fallback round interval, two read rounds (a window older than
// two of these is not current): rounds come every tick, or every counters_min_interval_s.
int Engine::counters_interval_ms() const {
  return std::max(10, int(std::max(cfg_.interval_s, cfg_.counters_min_interval_s) * 2000));
}

// counters_cpu_budget: a finished read round's CPU (this thread's kick + sync, and the plugin
// thread's since the last round) goes into a per-round EWMA; the rounds' minimum interval becomes
// EWMA / budget when that is longer than both counters_min_interval_s and a tick, rounded up to
// whole ticks and at most 2 x max(counters_min_interval_s, tick) -- the plugin's fallback interval
// (counters_interval_ms) is twice that, so a window is never taken for stale.  8 MI355X GPUs at
// ~15 us per read: 120 us per round -> 16 ms, no change; a CPX node's 64 partitions at that cost:
// ~0.9 ms per round -> 120 ms, a round every 2nd tick at 10 Hz, every 10th at 100 Hz.
// The EWMA follows the steady cost, not a stall: a late round (its sync ran out: the wait polls,
// up to counters_sync_us of CPU) is left out, and a round counts at most 2x the EWMA -- a GPU
// whose reads queue behind a starved sentinel run for a second must not halve its round rate
// (MI355X: 8 stalled rounds took the EWMA past 750 us and the windows to 200 ms, session 10).
void counters_round_policy(double round_cpu_ns, bool late, double budget, double base_ns, double period_ns,
                           double* ewma_ns, double* iv_ns) {
  if (late) return;
  const double x = *ewma_ns > 0 ? std::min(round_cpu_ns, 2 * *ewma_ns) : round_cpu_ns;
  *ewma_ns = *ewma_ns > 0 ? 0.9 * *ewma_ns + 0.1 * x : x;
  double iv = 0;
  if (budget > 0 && period_ns > 0) {
    const double want = std::min(*ewma_ns / budget, 2 * std::max(base_ns, period_ns));
    if (want > base_ns && want > period_ns) iv = std::max(base_ns, std::ceil(want / period_ns - 1e-6) * period_ns);
  }
  *iv_ns = iv;
}

void Engine::counters_round_done(bool late) {
  uint64_t c = counters_round_acc_ns_;
  counters_round_acc_ns_ = 0;
  const uint64_t p = counters_->cpu_ns();
  const bool first = counter_rounds_++ == 0;  // (the first round carries the plugin's start-up)
  if (p >= counters_round_plugin_seen_) c += p - counters_round_plugin_seen_;
  counters_round_plugin_seen_ = p;
  if (first) return;
  counters_round_policy(double(c), late, cfg_.counters_cpu_budget, cfg_.counters_min_interval_s * 1e9,
                        cfg_.interval_s * 1e9, &counters_round_cpu_ns_, &counters_round_iv_ns_);
}

double Engine::counters_round_interval_s() const {
  if (!counters_) return 0;
  return (counters_round_iv_ns_ > 0 ? counters_round_iv_ns_ : cfg_.counters_min_interval_s * 1e9) * 1e-9;
}

// Registers a source's family table: SeriesTable ids, and handle slots per GPU or global.
void Engine::register_families(const std::vector<FamilySpec>& specs) {
  for (const FamilySpec& f : specs) {
    if (f.needs_legacy && !cfg_.legacy_families) continue;
    fam_ids_[f.id] = table_.add_family(FamilyDef{f.name, f.help, f.type, family_labels(f)});
    if (f.scope == RefScope::kGpu) {
      fam_off_[f.id] = gpu_slots_;
      gpu_slots_ += f.slots;
    } else if (f.scope == RefScope::kGlobal) {
      fam_off_[f.id] = int(grefs_.size());
      grefs_.resize(grefs_.size() + size_t(f.slots));
    }
  }
}

void Engine::define_families() {
  std::fill(std::begin(fam_ids_), std::end(fam_ids_), -1);
  std::fill(std::begin(fam_off_), std::end(fam_off_), -1);
  gpu_slots_ = 0;
  grefs_.clear();
  for (const auto* t : {&device_family_specs(), &process_family_specs(), &pod_family_specs(), &rccl_family_specs(),
                        &kfd_event_family_specs(), &self_family_specs()})
    register_families(*t);
}

namespace {
// Runtime libraries started here (amdsmi, ROCr/HSA, HIP) create threads of their own, which
// inherit the creating thread's name: named "gpuexp-rt" they show apart from the host
// process's threads in per-thread CPU accounting (bench.py exporter_cpu_us_per_step_by_thread).
struct RuntimeThreadsName {
  char saved[17] = {};
  RuntimeThreadsName() {
    ::prctl(PR_GET_NAME, saved, 0, 0, 0);
    set_thread_name("gpuexp-rt");
  }
  ~RuntimeThreadsName() { set_thread_name(saved); }
};
}  // namespace

bool Engine::start(std::string* err) {
  if (running_.load()) return true;
  RuntimeThreadsName rt_name;
  start_mono_ns_ = mono_ns();
  compiled_ = cfg_.exposition != "classic";
  counters_kick_mode_ = cfg_.counters_kick != "auto" ? cfg_.counters_kick
                        : (cfg_.interval_s > 0 && cfg_.interval_s < 0.05 ? "end" : "start");
  define_families();
  // Listen first: a port conflict fails before any GPU-side source (amdsmi, HSA queues,
  // sentinel runs) exists.  Every later failure tears down what was already started.
  if (cfg_.serve_http) {
    HttpConfig hc = cfg_.http;
    hc.gzip_level = cfg_.gzip_level;
    if (const char* e = std::getenv("GPUEXP_HTTP_FOLLOW_RX_CPU")) hc.follow_rx_cpu = e[0] != '0';
    // experiment knobs (A/B on a box): pre-wake slice and minimum lead, microseconds
    if (const char* e = std::getenv("GPUEXP_HTTP_PREWAKE_STEP_US")) hc.prewake_step_ns = uint64_t(std::atoll(e)) * 1000;
    if (const char* e = std::getenv("GPUEXP_HTTP_PREWAKE_LEAD_US")) hc.prewake_lead_ns = uint64_t(std::atoll(e)) * 1000;
    if (const char* e = std::getenv("GPUEXP_HTTP_PREWAKE_SPIN_MAX_US"))
      hc.prewake_spin_max_ns = uint64_t(std::atoll(e)) * 1000;
    http_ = std::make_unique<HttpServer>(&store_, hc);
    if (!http_->start(err)) {
      http_.reset();
      return false;
    }
  }
  bool ok = false;
  struct Undo {
    Engine* e;
    bool* ok;
    ~Undo() {
      if (*ok) return;
      if (e->http_) e->http_->stop();
      e->http_.reset();
      if (e->backend_) e->backend_->shutdown();
      e->backend_.reset();
      e->mock_ = nullptr;
      e->devices_.clear();
    }
  } undo{this, &ok};
  if (cfg_.backend == "mock") {
    auto m = std::make_unique<MockBackend>(cfg_.mock_devices);
    if (!cfg_.mock_xgmi_file.empty()) m->set_traffic_file(cfg_.mock_xgmi_file);
    mock_ = m.get();
    backend_ = std::move(m);
  } else if (cfg_.backend == "sysfs") {
    backend_ = std::make_unique<SysfsBackend>(cfg_.host_root);
  } else if (cfg_.backend == "amdsmi") {
    backend_ = make_amdsmi_backend(cfg_.host_root, cfg_.process_source == "amdsmi", cfg_.force_amdsmi_metrics);
  } else {
    *err = "unknown backend: " + cfg_.backend;
    return false;
  }
  backend_->set_metrics_coalescing(cfg_.metrics_coalesce);
  backend_->set_metrics_min_interval(uint64_t(std::max(0.0, cfg_.metrics_min_interval_s) * 1e9));
  backend_->set_fake_metrics_cost(cfg_.fake_metrics_cost_us * 1000ull);
  std::vector<DeviceInfo> all;
  if (!backend_->init(&all, err)) return false;
  if (!cfg_.device_filter.empty() || !cfg_.device_filter_bdf.empty()) {
    auto lower = [](std::string x) {
      for (auto& ch : x) ch = char(::tolower(static_cast<unsigned char>(ch)));
      return x;
    };
    for (auto& d : all) {
      bool want = std::find(cfg_.device_filter.begin(), cfg_.device_filter.end(), d.index) != cfg_.device_filter.end();
      for (const auto& b : cfg_.device_filter_bdf) want = want || lower(b) == lower(d.bdf);
      if (want) devices_.push_back(d);
    }
    // keep backend indices: DeviceInfo::index addresses the backend's own table
  } else {
    devices_ = all;
  }
  if (!cfg_.queue_devices.empty() || !cfg_.queue_devices_bdf.empty()) {
    for (auto& d : devices_) {
      bool on = std::find(cfg_.queue_devices.begin(), cfg_.queue_devices.end(), d.index) != cfg_.queue_devices.end();
      for (const auto& b : cfg_.queue_devices_bdf) on = on || engine_util::lower(b) == engine_util::lower(d.bdf);
      d.queue_enabled = on;
    }
  }
  const bool any_queue = std::any_of(devices_.begin(), devices_.end(), [](const DeviceInfo& d) {
    return d.queue_enabled;
  });
  dstate_.assign(devices_.size(), DevState());
  {  // SMU fetch groups: a whole GPU, or the partitions of one socket (share_socket_fetches)
    std::vector<int> sockets;
    fetch_groups_ = 0;
    for (const DeviceInfo& d : devices_) {
      if (d.socket_group < 0) {
        ++fetch_groups_;
      } else if (std::find(sockets.begin(), sockets.end(), d.socket_group) == sockets.end()) {
        sockets.push_back(d.socket_group);
        ++fetch_groups_;
      }
    }
  }
  for (DevState& st : dstate_) st.refs.assign(size_t(gpu_slots_), SeriesRef());
  owner_keys_.clear();
  for (const DeviceInfo& d : devices_) owner_keys_.push_back(device_owner_keys(d));
  metrics_fresh_.assign(devices_.size(), 0);
  metrics_coalesced_.assign(devices_.size(), 0);
  if (cfg_.series_profile == "full" && cfg_.backend != "mock") {
    const std::string root = cfg_.host_root.empty() ? "" : cfg_.host_root;
    ras_.resize(devices_.size());
    for (size_t i = 0; i < devices_.size(); ++i) {
      const DeviceInfo& di = devices_[i];
      if (di.render_minor >= 0)
        ras_[i].open(root + "/sys/class/drm/renderD" + std::to_string(di.render_minor) + "/device");
      else if (!di.bdf.empty())
        ras_[i].open(root + "/sys/bus/pci/devices/" + di.bdf);
    }
    ras_cache_.assign(devices_.size(), RasTotals());
    ras_next_ns_.assign(devices_.size(), 0);
    // GTT lives on the PCI function (a partition's amdgpu_xcp node has no mem_info_*)
    gtt_used_f_.resize(devices_.size());
    gtt_total_.assign(devices_.size(), kNaN);
    for (size_t i = 0; i < devices_.size(); ++i) {
      const DeviceInfo& di = devices_[i];
      for (const std::string& dir : {root + "/sys/class/drm/renderD" + std::to_string(di.render_minor) + "/device",
                                     root + "/sys/bus/pci/devices/" + di.bdf}) {
        if (!gtt_used_f_[i].open(dir + "/mem_info_gtt_used")) continue;
        std::string body;
        uint64_t v = 0;
        if (read_small_file(dir + "/mem_info_gtt_total", &body) && parse_u64(body.data(), body.size(), &v))
          gtt_total_[i] = double(v);
        break;
      }
    }
  }
  // auto = serial: a fresh gpu_metrics read is kernel busy-wait (its CPU is the same on any
  // thread) and waking a pool costs more CPU than the parallel reads save wall time
  // (8 fake GPUs at 100 Hz: 9.8 % vs 6.3 % of a core, profiles/r04/devices_split.txt); a
  // pool only shortens the tick's wall time (8 x 0.45 ms at most), so it stays opt-in.
  int nthreads = cfg_.device_threads;
  if (nthreads <= 0) nthreads = 1;
  if (nthreads > 1) pool_ = std::make_unique<ForkJoinPool>(nthreads);
  kfd_ = std::make_unique<KfdProcReader>(cfg_.host_root, cfg_.exclude_self ? self_pid_ : -1, cfg_.kfd_cu_occupancy,
                                         uint64_t(cfg_.kfd_detail_interval_s * 1e9),
                                         uint64_t(cfg_.kfd_rescan_interval_s * 1e9), cfg_.kfd_sdma);
  resolver_ = std::make_unique<PidResolver>(cfg_.host_root);

  // Counters first: the rocprofiler tool must register before the HSA runtime loads,
  // which the sentinel's first HIP call does.
  if (cfg_.enable_counters && cfg_.fake_pmc_cost_us >= 0 && cfg_.backend != "amdsmi") {
    const bool inline_rounds = cfg_.interval_s > 0 && cfg_.counters_inline;
    counters_ = make_fake_counters(uint64_t(cfg_.fake_pmc_cost_us), counters_interval_ms(), inline_rounds,
                                   cfg_.fake_pmc_stalls_us);
    std::string e;
    if (!counters_->start(devices_, &e)) {
      counters_status_ = "unavailable: " + e;
      counters_.reset();
    } else {
      counters_status_ = counters_->status();
    }
  } else if (cfg_.enable_counters && cfg_.backend != "mock" && !any_queue) {
    counters_status_ = "disabled: no GPU in queue_devices";
  } else if (cfg_.enable_counters && cfg_.backend != "mock") {
    const bool continuous = cfg_.counters_mode == "continuous";
    // continuous: every tick kicks a read; the plugin's own timer (2 ticks) only covers
    // engines without a sampler thread
    const int interval_ms = continuous && cfg_.interval_s > 0 ? counters_interval_ms() : cfg_.counters_interval_ms;
    // a periodic sampler runs each tick's read round itself (kick / sync): no wake-ups of the
    // plugin's counting thread per tick (~30-55 us of CPU per tick on MI355X, profiles/r04)
    const bool inline_rounds = continuous && cfg_.interval_s > 0 && cfg_.counters_inline;
    counters_ = make_rocprof_counters(cfg_.counters_plugin, cfg_.counters_window_ms, interval_ms, continuous,
                                      inline_rounds);
    std::string e;
    if (!counters_ || !counters_->start(devices_, &e)) {
      counters_status_ = "unavailable: " + e;
      GPUEXP_LOG(LogLevel::kWarn, "counters", counters_status_);
      counters_.reset();
    } else {
      counters_status_ = counters_->status();
    }
  } else if (cfg_.enable_counters) {
    counters_status_ = "mock";
  }
  if (cfg_.enable_sentinel && cfg_.fake_sentinel_cost_us >= 0 && cfg_.backend != "amdsmi") {
    sentinel_ = make_fake_sentinel(uint64_t(cfg_.fake_sentinel_cost_us));
    std::string e;
    sentinel_->start(devices_, &e);
    sentinel_status_ = sentinel_->status();
  } else if (cfg_.enable_sentinel && cfg_.backend != "mock" && !any_queue) {
    sentinel_status_ = "disabled: no GPU in queue_devices";
  } else if (cfg_.enable_sentinel && cfg_.backend != "mock") {
    std::string e;
    // Prefer the counters plugin's queue (one GPU queue, and its ~173 MiB context save
    // area, per GPU instead of two); the HIP plugin's own stream otherwise.
    if (cfg_.sentinel_impl != "hip" && counters_) {
      sentinel_ = make_queue_sentinel(cfg_.counters_plugin, cfg_.sentinel_ring, cfg_.sentinel_spin);
      if (sentinel_ && !sentinel_->start(devices_, &e)) {
        GPUEXP_LOG(LogLevel::kInfo, "sentinel", "queue sentinel unavailable (" + e + "), using HIP");
        sentinel_.reset();
      }
    }
    if (!sentinel_ && cfg_.sentinel_impl != "queue") {
      sentinel_ = make_hip_sentinel(cfg_.sentinel_ring, cfg_.sentinel_spin);
      e = "libgpuexp_hip.so not loadable";
      if (sentinel_ && !sentinel_->start(devices_, &e)) sentinel_.reset();
    }
    if (!sentinel_) {
      sentinel_status_ = "unavailable: " + e;
      GPUEXP_LOG(LogLevel::kWarn, "sentinel", sentinel_status_);
      sentinel_.reset();
    } else {
      sentinel_status_ = sentinel_->status();
    }
  } else if (cfg_.enable_sentinel) {
    sentinel_status_ = "mock";
  }
  if (cfg_.enable_rccl) rccl_ = make_rccl_source(cfg_.rccl_dir, cfg_.rccl_verify, cfg_.rccl_scan_interval_s);
  {
    std::string v;
    driver_version_ = read_small_file((cfg_.host_root.empty() ? "" : cfg_.host_root) + "/sys/module/amdgpu/version", &v, 128)
                          ? trim(v)
                          : (mock_ ? "mock" : "in-kernel");  // DKMS builds carry a version file
    struct utsname u{};
    kernel_release_ = ::uname(&u) == 0 ? u.release : "";
  }
  if (!cfg_.state_file.empty()) load_state();
  if (cfg_.enable_kfd_events && cfg_.series_profile == "full") {
    kfd_events_ = std::make_unique<KfdEventSource>();
    if (mock_) {
      kfd_events_->set_devices(devices_.size());  // events arrive through inject_kfd_events only
      kfd_events_status_ = "mock (injected events)";
    } else {
      std::string e;
      const int n = kfd_events_->open(devices_, cfg_.kfd_path, &e);
      if (n == 0) {
        kfd_events_status_ = "unavailable: " + e;
        GPUEXP_LOG(LogLevel::kWarn, "kfd_events", kfd_events_status_);
        kfd_events_.reset();
      } else {
        kfd_events_status_ = "on " + std::to_string(n) + " GPU(s), " +
                             (kfd_events_->all_processes() ? "every process's events"
                                                           : "device-wide events + own process (no CAP_SYS_ADMIN)");
      }
    }
  }

  if (!cfg_.trace_path.empty()) {
    trace_ = std::fopen(cfg_.trace_path.c_str(), "w");
    if (trace_) {
      std::fputs("[\n", trace_);
      trace_t0_ = mono_ns();
    }
  }
  ok = true;
  running_.store(true);
  if (cfg_.interval_s > 0 && cfg_.sampler_thread) {
    stop_fd_ = ::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
    sampler_ = std::thread([this] { run_sampler(); });
  }
  return true;
}

void Engine::stop() {
  if (!running_.exchange(false)) return;
  if (stop_fd_ >= 0) {
    uint64_t one = 1;
    ssize_t r = ::write(stop_fd_, &one, sizeof(one));
    (void)r;
  }
  if (sampler_.joinable()) sampler_.join();
  if (stop_fd_ >= 0) ::close(stop_fd_);
  stop_fd_ = -1;
  if (!cfg_.state_file.empty()) {
    std::lock_guard<std::mutex> lk(tick_mu_);
    save_state();
  }
  if (http_) http_->stop();
  if (sentinel_) sentinel_->stop();
  if (counters_) counters_->stop();
  if (backend_) backend_->shutdown();
  if (trace_) {
    std::fputs("{}]\n", trace_);
    std::fclose(trace_);
    trace_ = nullptr;
  }
}

void Engine::run_sampler() {
  set_thread_name("gpuexp-sampler");
  tl_sampler_thread = true;
  int tfd = ::timerfd_create(CLOCK_MONOTONIC, TFD_CLOEXEC);
  uint64_t period = uint64_t(cfg_.interval_s * 1e9);
  if (period < 1000000) period = 1000000;  // 1 kHz cap
  itimerspec its{};
  its.it_interval.tv_sec = time_t(period / 1000000000ull);
  its.it_interval.tv_nsec = long(period % 1000000000ull);
  its.it_value.tv_nsec = 1;  // first tick immediately
  ::timerfd_settime(tfd, 0, &its, nullptr);
  pollfd fds[2] = {{tfd, POLLIN, 0}, {stop_fd_, POLLIN, 0}};
  while (running_.load()) {
    int n = ::poll(fds, 2, -1);
    if (n < 0) continue;
    if (fds[1].revents & POLLIN) break;
    if (fds[0].revents & POLLIN) {
      uint64_t expirations = 0;
      ssize_t r = ::read(tfd, &expirations, sizeof(expirations));
      if (r != sizeof(expirations)) continue;
      if (expirations > 1) {
        std::lock_guard<std::mutex> lk(stats_mu_);
        stats_.overruns += expirations - 1;
      }
      std::lock_guard<std::mutex> lk(tick_mu_);
      tick_locked(mono_ns());
    }
  }
  ::close(tfd);
}

void timer_wakeup_cost(uint64_t period_ns, int n, uint64_t* cpu_ns, uint64_t* late_ns) {
  *cpu_ns = *late_ns = 0;
  int tfd = ::timerfd_create(CLOCK_MONOTONIC, TFD_CLOEXEC);
  if (tfd < 0 || n <= 0) {
    if (tfd >= 0) ::close(tfd);
    return;
  }
  itimerspec its{};
  its.it_interval.tv_sec = time_t(period_ns / 1000000000ull);
  its.it_interval.tv_nsec = long(period_ns % 1000000000ull);
  its.it_value = its.it_interval;
  uint64_t due = mono_ns() + period_ns;
  ::timerfd_settime(tfd, 0, &its, nullptr);
  pollfd fd{tfd, POLLIN, 0};
  const uint64_t c0 = thread_cpu_ns();
  for (int i = 0; i < n; ++i) {  // the sampler's own wait (run_sampler), with no tick in between
    if (::poll(&fd, 1, -1) < 0) continue;
    uint64_t exp = 0;
    if (::read(tfd, &exp, sizeof(exp)) != sizeof(exp)) continue;
    const uint64_t t = mono_ns();
    *late_ns += t > due ? t - due : 0;
    due += (exp ? exp : 1) * period_ns;
  }
  *cpu_ns = (thread_cpu_ns() - c0) / uint64_t(n);
  *late_ns /= uint64_t(n);
  ::close(tfd);
}

void Engine::tick_now(uint64_t now_ns) {
  std::lock_guard<std::mutex> lk(tick_mu_);
  tick_locked(now_ns);
}

void Engine::set_pods(std::vector<PodMeta> pods, bool complete) {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_pods_ = std::move(pods);
  ctl_dirty_ = true;
  pending_complete_ = complete;
}

void Engine::set_device_owners(std::vector<std::pair<std::string, DeviceOwner>> owners) {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_owners_ = std::move(owners);
  ctl_dirty_ = true;
}

void Engine::inject_kfd_events(int dev, const std::string& bytes) {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_kfd_bytes_.emplace_back(dev, bytes);
}

void Engine::set_pid_cgroup(int pid, const std::string& cgroup_path) {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_overrides_.emplace_back(pid, cgroup_path);
}

void Engine::clear_pid_cgroups() {
  std::lock_guard<std::mutex> lk(ctl_mu_);
  pending_overrides_.clear();
  clear_overrides_ = true;
}

void Engine::trace_event(const char* name, uint64_t start_ns, uint64_t dur_ns) {
  if (!trace_ || trace_events_ >= cfg_.trace_max_events) return;
  ++trace_events_;
  std::fprintf(trace_, "{\"name\":\"%s\",\"ph\":\"X\",\"ts\":%.3f,\"dur\":%.3f,\"pid\":%d,\"tid\":1},\n", name,
               double(start_ns - trace_t0_) * 1e-3, double(dur_ns) * 1e-3, self_pid_);
}

void Engine::tick_locked(uint64_t now) {
  uint64_t cpu0 = thread_cpu_ns();
  uint64_t gen = ++gen_;
  double dt_s = last_tick_now_ && now > last_tick_now_ ? double(now - last_tick_now_) * 1e-9 : 0.0;
  last_tick_now_ = now;
  uint64_t ts[kStages + 1], cs[kStages + 1];  // stage boundaries: wall, sampler-thread CPU
  // The per-stage CPU split is sampled on one tick in kStageCpuEvery (a thread CPU clock read is
  // a system call: 7 of them per tick were ~1 % of an 8-GPU node's tick at 10 Hz); the whole
  // tick's CPU is read every tick.  Which ticks: a hash of the generation, so a periodic stage
  // (a gpu_metrics fetch every 2nd or 4th tick) is not always in or always out of the sample.
  const bool split_cpu = ((gen * 0x9E3779B97F4A7C15ull) >> 61) % kStageCpuEvery == 0;
  auto cpu_mark = [split_cpu]() { return split_cpu ? thread_cpu_ns() : 0; };
  ts[0] = mono_ns();
  cs[0] = cpu0;
  if (!startup_ns_ && start_mono_ns_ && ts[0] > start_mono_ns_) startup_ns_ = ts[0] - start_mono_ns_;
  // continuous counters: this tick's read goes out now (or right after the device reads)
  // and is collected before the series stage, so the exported window is one tick interval
  resolver_->begin_tick(now);
  uint64_t part[kDevParts] = {};
  // "end" (auto below 50 ms ticks): the read for this tick went out at the end of the previous
  // one, so it has completed by the counters stage -- at 100 Hz most ticks have no SMU fetch
  // to hide a ~200 us PM4 read behind, and waiting for it cost 2-3 sleep/wake-ups per tick;
  // the exported window then ends one tick earlier (10 ms at 100 Hz)
  const std::string& kick_mode = counters_kick_mode_;
  const bool kick_late = kick_mode == "after_devices";
  const bool kick_end = kick_mode == "end";
  // (rounds at most every counters_min_interval_s, or longer under counters_cpu_budget: in
  // between a tick exports the last window)
  const uint64_t period_ns = cfg_.interval_s > 0 ? uint64_t(cfg_.interval_s * 1e9) : 0;
  const uint64_t ctr_iv = counters_round_iv_ns_ > 0 ? uint64_t(counters_round_iv_ns_)
                                                    : uint64_t(cfg_.counters_min_interval_s * 1e9);
  // Leveling: a round stretched over several ticks (counters_cpu_budget, e.g. a CPX node) is put
  // off by one tick when that tick is due two or more SMU fetches -- predicted from the tick one
  // fetch pattern (fetch_ticks_) earlier, since the read goes out before the tick's fetches.  A
  // put-off round runs on the next tick whatever it carries; windows stay < 2 fallback intervals.
  auto heavy_ahead = [&](uint64_t tick) {  // `tick`: a tick_index_ value
    const uint64_t k = uint64_t(fetch_ticks_);
    if (k < 2 || k >= uint64_t(kFreshHist) || tick <= k) return false;
    const int f = fresh_hist_[(tick - k) % kFreshHist];
    return f >= 2 && f < fetch_groups_;
  };
  auto counters_due = [&](uint64_t t, uint64_t tick) {
    if (!period_ns || !counters_kick_ns_ || t < counters_kick_ns_) return true;
    if (t - counters_kick_ns_ + period_ns / 2 < ctr_iv) return false;
    if (counters_round_iv_ns_ > 0 && !counters_deferred_ && heavy_ahead(tick)) {
      counters_deferred_ = true;
      leveled_ = true;
      return false;
    }
    counters_deferred_ = false;
    return true;
  };
  // a round's CPU on this thread (kick + sync), for counters_cpu_budget
  auto kick_counters = [&] {
    const uint64_t k0 = thread_cpu_ns();
    counters_->kick();
    counters_round_acc_ns_ += thread_cpu_ns() - k0;
  };
  bool round = kick_end && counters_round_next_;  // kicked at the end of the previous tick
  counters_round_next_ = false;
  leveled_ = false;
  if (counters_ && !kick_late && !kick_end && counters_due(now, tick_index_ + 1)) {
    kick_counters();
    counters_kick_ns_ = now;
    round = true;
    part[0] = mono_ns() - ts[0];
  }
  const uint64_t c0 = mono_ns();

  // Control-plane updates (pushed from Python at low rate).
  {
    std::lock_guard<std::mutex> lk(ctl_mu_);
    if (clear_overrides_) {
      resolver_->clear_overrides();
      clear_overrides_ = false;
      ++ctl_epoch_;
    }
    if (!pending_overrides_.empty()) ++ctl_epoch_;
    for (auto& o : pending_overrides_) resolver_->set_override(o.first, o.second);
    pending_overrides_.clear();
    if (ctl_dirty_) {
      ++ctl_epoch_;
      pods_by_uid_.clear();
      container_names_.clear();
      for (auto& p : pending_pods_) {
        for (auto& c : p.containers) container_names_[engine_util::lower(c.first)] = c.second;
        pods_by_uid_[engine_util::lower(p.uid)] = p;
      }
      owners_.clear();
      for (auto& o : pending_owners_) owners_[engine_util::lower(o.first)] = o.second;
      ctl_dirty_ = false;
      // per-pod totals (energy, xGMI bytes, KFD events; possibly restored from the state
      // file) are garbage-collected against a pod list only if that list is complete: a
      // refresh in which a source failed must not wipe them
      pods_complete_ = pending_complete_;
      const uint64_t applied = mono_ns();
      for (auto& kv : pods_by_uid_) pod_last_known_ns_[{kv.second.ns, kv.second.name}] = applied;
    }
  }
  part[1] = mono_ns() - c0;

  // The memory reads -- per-process VRAM (KFD / amdsmi list) and each GPU's VRAM / GTT used --
  // run at most every process_min_interval_s; a tick in between exports the last values again.
  const bool procs_due = !period_ns || !procs_read_ns_ || now < procs_read_ns_ || per_dev_.size() != devices_.size() ||
                         now - procs_read_ns_ + period_ns / 2 >= uint64_t(cfg_.process_min_interval_s * 1e9);
  if (procs_due) procs_read_ns_ = now;

  // 0: device telemetry (engine_device.cc)
  const uint64_t errs = sample_devices(now, split_cpu, procs_due, part);
  // Tick leveling: with the SMU fetches phased over k ticks (update_fetch_policy), a tick that
  // carries two or more of them defers the periodic extras whose timers came due -- the
  // sentinel run and the KFD rescan listing -- to a lighter tick (at most to twice their
  // interval).  Once run there they stay there: their timers count from the actual run.  At
  // 8 GPUs and 10 Hz the fetches come 2,2,1,2,1 per tick and these extras had a 0.5 s period
  // too, so without it they kept landing on a two-fetch tick (the heaviest tick ~1.5x the mean).
  int fresh_now = 0;
  for (const DevState& st : dstate_) fresh_now += st.cur.ok && !st.cur.metrics_coalesced && !st.cur.metrics_shared;
  // (with the fetches phased over k ticks, "heavy" is relative to the lightest of the last k: a
  // stretched PMC round -- a CPX node's 64 reads -- weighs as two fetches, so the extras do not
  // pile onto the one-fetch ticks the rounds were leveled to)
  const int load_now = fresh_now + (round && counters_round_iv_ns_ > 0 ? 2 : 0);
  bool heavy_tick = fresh_now >= 2 && fresh_now < fetch_groups_;
  if (counters_round_iv_ns_ > 0 && fetch_ticks_ >= 2 && fetch_ticks_ < kFreshHist &&
      tick_index_ >= uint64_t(fetch_ticks_)) {
    int lo = 255;
    for (int j = 1; j <= fetch_ticks_; ++j) lo = std::min<int>(lo, load_hist_[(tick_index_ + 1 - uint64_t(j)) % kFreshHist]);
    heavy_tick = load_now >= 2 && load_now > lo;
  }  // (every group fetched: no lighter tick)
  if (counters_ && kick_late && counters_due(now, tick_index_ + 1)) {
    counters_kick_ns_ = now;
    round = true;
    const uint64_t k0 = mono_ns();
    kick_counters();
    part[0] = mono_ns() - k0;
  }
  ts[1] = mono_ns();
  cs[1] = cpu_mark();
  for (int k = 0; k < kDevParts; ++k) dev_part_total_s_[k] += double(part[k]) * 1e-9;

  // 1: processes
  // (reused across ticks: the lists keep their capacity, no allocation per tick)
  std::vector<std::vector<ProcSample>>& per_dev = per_dev_;
  if (procs_due) {
    per_dev.resize(devices_.size());
    for (auto& l : per_dev) l.clear();
  }
  if (procs_due && cfg_.process_source != "none") {
    bool from_backend = cfg_.process_source != "kfd";
    if (from_backend)
      for (size_t i = 0; i < devices_.size(); ++i)
        if (!backend_->processes(devices_[i], &per_dev[i])) {
          from_backend = false;
          break;
        }
    if (!from_backend) {
      const uint64_t lists0 = kfd_->lists();
      kfd_->scan(devices_, &per_dev, now, heavy_tick);
      if (heavy_tick && kfd_->lists() == lists0 && kfd_->listing_deferred()) leveled_ = true;
    } else if (cfg_.exclude_self) {
      for (auto& l : per_dev)
        l.erase(std::remove_if(l.begin(), l.end(), [this](const ProcSample& p) { return p.pid == self_pid_; }),
                l.end());
    }
  }
  ts[2] = mono_ns();
  cs[2] = cpu_mark();

  // 2: device ownership (device plugin map first, then single-pod inference; engine_pods.cc)
  infer_owners(per_dev);
  ts[3] = mono_ns();
  cs[3] = cpu_mark();

  // 3: sentinel (drain previous run, launch next; never blocks on the GPU)
  const uint64_t sen_iv = uint64_t(cfg_.sentinel_min_interval_s * 1e9);
  if (sentinel_ && (cfg_.interval_s <= 0 || !sentinel_last_ns_ || now < sentinel_last_ns_ ||
                    (now - sentinel_last_ns_ + uint64_t(cfg_.interval_s * 5e8) >= sen_iv &&
                     !(heavy_tick && now - sentinel_last_ns_ < 2 * sen_iv)))) {
    sentinel_->tick(now);  // at most every sentinel_min_interval_s (half a tick of slack)
    sentinel_last_ns_ = now;
    ++sentinel_runs_;
  } else if (sentinel_ && heavy_tick && now - sentinel_last_ns_ + uint64_t(cfg_.interval_s * 5e8) >= sen_iv) {
    leveled_ = true;
  }
  if (kfd_events_) count_kfd_events();
  ts[4] = mono_ns();
  cs[4] = cpu_mark();
  // 4: counters: wait (bounded) for this tick's read round; sampled in collect_device
  if (counters_ && round) {
    const uint64_t s0 = thread_cpu_ns();
    const bool late = !counters_->sync(cfg_.counters_sync_us);
    counters_late_ += late;
    counters_round_acc_ns_ += thread_cpu_ns() - s0;
    counters_round_done(late);
  }
  ts[5] = mono_ns();
  cs[5] = cpu_mark();

  // 6 (decided here): does this tick render -- when a scrape will read it (render_when_due):
  // with only steady scrapers known and none due before the tick after next, the tick neither
  // writes the series table nor renders (at least one render a second); the series stage's
  // computations run all the same
  bool render_now = true;
  ++tick_index_;
  if (cfg_.render_every_ticks > 0) {  // (tests: a scrape schedule without an HTTP server)
    render_now = tick_index_ % uint64_t(cfg_.render_every_ticks) == 0;
  } else if (http_ && cfg_.render_when_due && period_ns) {
    const uint64_t tn = mono_ns();
    render_now = !last_render_mono_ || tn < last_render_mono_ || tn - last_render_mono_ >= 1000000000ull ||
                 http_->render_due(tn, 2 * period_ns + 5000000ull);
  }
  if (!render_now) ++renders_skipped_;
  emit_ = render_now;

  // 5: series
  for (size_t i = 0; i < devices_.size(); ++i) {
    if (cfg_.series_profile != "legacy") collect_device(int(i), gen, dt_s);
  }
  emit_processes(gen, per_dev);
  if (cfg_.series_profile != "legacy") {
    emit_pods(gen, per_dev);
    emit_rccl(gen);
  }
  if (kfd_events_) emit_kfd_events(gen);
  emit_self(gen);
  ts[6] = mono_ns();
  cs[6] = cpu_mark();

  // 6: render into a free snapshot slot (render_now: decided before the series stage)
  emit_ = true;
  int slot = render_now ? store_.begin_write() : -1;
  uint64_t rbytes = 0, nseries = 0;
  if (slot >= 0) {
    last_render_mono_ = mono_ns();
    Snapshot* snap = store_.slot(slot);
    // gzip copy only when a gzip scrape is expected before the tick after next (or its
    // schedule is unknown): a 15 s Prometheus scrape costs one compression, not 150
    const uint64_t period_ns = cfg_.interval_s > 0 ? uint64_t(cfg_.interval_s * 1e9) : 1000000000ull;
    const bool want_gz = http_ && http_->gzip_due(mono_ns(), 2 * period_ns + 5000000ull);
    if (want_gz) ++gzip_eager_;
    snap->gz.clear();
    // (the slot's previous generation: only the fields changed since are copied into it)
    if (compiled_) table_.render_compiled(&snap->body, want_gz ? &snap->gz : nullptr, gen, cfg_.gc_after, snap->gen);
    else table_.render(&snap->body, gen, cfg_.gc_after);
    snap->gen = gen;
    snap->render_ns = now;
    rbytes = snap->body.size();
    nseries = table_.live_series(gen);
    snap->series = nseries;
    ts[7] = mono_ns();
    cs[7] = cpu_mark();
    // 7: gzip (classic; compiled emitted it with the body) + publish
    snap->pb.clear();
    snap->pb_gz.clear();
    const uint64_t tnow = mono_ns();
    if (want_gz && !compiled_) gzip_compress(snap->body, &snap->gz, cfg_.gzip_level);
    if (http_ && http_->proto_wanted_ns() && tnow - http_->proto_wanted_ns() < 60000000000ull) {
      table_.render_proto(&snap->pb, gen);
      if (want_gz) gzip_compress(snap->pb, &snap->pb_gz, cfg_.gzip_level);
    }
    snap->published_mono_ns = mono_ns();
    store_.publish(slot);
    if (http_) http_->set_ready(true);
  } else {
    ts[7] = mono_ns();
    cs[7] = cpu_mark();
  }
  if (!cfg_.state_file.empty() && ts[7] - state_saved_ns_ >= uint64_t(cfg_.state_interval_s * 1e9)) save_state();
  fresh_hist_[tick_index_ % kFreshHist] = uint8_t(std::min(fresh_now, 255));
  load_hist_[tick_index_ % kFreshHist] = uint8_t(std::min(load_now, 255));
  if (counters_ && kick_end && counters_due(now + period_ns, tick_index_ + 1)) {  // next tick's read, completing while we sleep
    kick_counters();
    counters_kick_ns_ = now + period_ns;
    counters_round_next_ = true;
  }
  uint64_t tend = mono_ns();
  cs[kStages] = thread_cpu_ns();
  uint64_t stage_dur[kStages] = {ts[1] - ts[0], ts[2] - ts[1], ts[3] - ts[2], ts[4] - ts[3],
                                 ts[5] - ts[4], ts[6] - ts[5], ts[7] - ts[6], tend - ts[7]};
  for (int k = 0; k < kStages; ++k) {
    last_stage_ns_[k] = stage_dur[k];
    uint64_t start = k == 0 ? ts[0] : (k < kStages - 1 ? ts[k] : ts[7]);
    trace_event(stage_name(k), start, stage_dur[k]);
    if (k == 0 && trace_) {  // the devices stage's parts, inside its span
      trace_event("devices/control", c0, part[1]);
      for (size_t i = 0; i < dstate_.size(); ++i)  // per GPU (they overlap on the read pool)
        if (dstate_[i].cur.metrics_wall_ns) trace_event("devices/gpu_metrics", c0 + part[1], dstate_[i].cur.metrics_wall_ns);
    }
  }
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.ticks += 1;
    stats_.fresh_reads += uint64_t(fresh_now);
    stats_.last_tick_fresh = uint64_t(fresh_now);
    stats_.sentinel_runs = sentinel_runs_;
    stats_.kfd_lists = kfd_ ? kfd_->lists() : 0;
    stats_.leveled_ticks += leveled_ ? 1 : 0;
    if (slot < 0 && render_now) stats_.publish_skipped += 1;
    stats_.renders_skipped = renders_skipped_;
    stats_.counter_rounds = counter_rounds_;
    stats_.counters_round_cpu_ns = counters_round_cpu_ns_;
    stats_.counters_round_interval_s = counters_round_interval_s();
    stats_.last_tick_ns = tend - ts[0];
    stats_.max_tick_ns = std::max(stats_.max_tick_ns, stats_.last_tick_ns);
    stats_.tick_ns_total += stats_.last_tick_ns;
    stats_.max_tick_cpu_ns = std::max(stats_.max_tick_cpu_ns, cs[kStages] - cpu0);
    stats_.tick_cpu_ns_total += cs[kStages] - cpu0;
    if (slot >= 0) {
      stats_.render_bytes = rbytes;
      stats_.series = nseries;
    }
    stats_.device_errors += errs;
    for (int k = 0; k < kStages; ++k) {
      stats_.stage_ns[k] = double(stage_dur[k]);
      if (split_cpu)  // the sampler thread's own CPU per stage, scaled up from the sampled ticks
        stats_.stage_cpu_ns[k] += kStageCpuEvery * (cs[k + 1] - cs[k]);
    }
    // every thread that worked for this tick: the sampler, the per-GPU read pool, and the
    // counter plugin's thread (its PM4 read rounds since the last tick)
    // The sampler thread charges its whole clock since the last tick (timerfd wake-ups
    // included); a manual tick_now() from another thread charges the tick itself.
    const uint64_t own = cs[kStages];
    uint64_t cpu = own - cpu0;
    if (tl_sampler_thread) {
      if (sampler_cpu_seen_ && own >= sampler_cpu_seen_) cpu = own - sampler_cpu_seen_;
      sampler_cpu_seen_ = own;
    }
    if (pool_) {
      const uint64_t p = pool_->cpu_ns_total();
      if (p >= pool_cpu_seen_) cpu += p - pool_cpu_seen_;
      pool_cpu_seen_ = p;
    }
    if (counters_) {
      const uint64_t c = counters_->cpu_ns();
      if (c >= counters_cpu_seen_) cpu += c - counters_cpu_seen_;
      counters_cpu_seen_ = c;
    }
    stats_.sampler_cpu_ns += cpu;
    stats_.gzip_eager = gzip_eager_;
    stats_.relayouts += table_.last_relayouts();
    stats_.families_skipped += table_.last_skipped();
    stats_.families_rendered += table_.last_walked();
    expo_relayouts_ += table_.last_relayouts();
    stats_.code_builds = table_.code_builds();
  }
}

std::string Engine::snapshot_text() {
  auto pin = store_.acquire();
  return pin ? pin->body : std::string();
}

EngineStats Engine::stats() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  return stats_;
}

std::string Engine::source_status() {
  std::string s = std::string("backend=") + (backend_ ? backend_->name() : "none") + " sentinel=" + sentinel_status_ +
                  " counters=" + counters_status_ + " rccl=" + (rccl_ ? cfg_.rccl_dir : "disabled") +
                  " kfd_events=" + kfd_events_status_ + " state=" + state_status();
  if (backend_)
    for (const auto& d : devices_) s += " gpu" + std::to_string(d.index) + "=[" + backend_->describe(d) + "]";
  return s;
}

}  // namespace gpuexp
