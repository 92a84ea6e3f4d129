// RoundMachine: see pmc_rounds.h.  No HSA in here: every GPU access goes through ReadPort.
#include "gpuexp/pmc_rounds.h"

#include <sys/prctl.h>
#include <time.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace gpuexp_pmc {

using namespace gpuexp_ctr;

const char* read_mode_name(ReadMode m) {
  return m == kCumulative ? "cumulative" : m == kResets ? "resets at read" : m == kStops ? "stops at read" : "?";
}

namespace {
uint64_t own_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

// Timed condition-variable wait on the steady clock.  gcc 11's TSan runtime does not intercept
// pthread_cond_clockwait (what a steady_clock wait compiles to), so it misses the unlock inside
// the wait and reports a double lock: the TSan build (csrc/tests/pmc_harness_main.cc under the
// tsan preset) waits on the system clock instead, which goes through pthread_cond_timedwait.
template <class Pred>
bool wait_until(std::condition_variable& cv, std::unique_lock<std::mutex>& lk, Clock::time_point deadline, Pred p) {
#if defined(__SANITIZE_THREAD__)
  return cv.wait_until(lk, std::chrono::system_clock::now() + (deadline - Clock::now()), p);
#else
  return cv.wait_until(lk, deadline, p);
#endif
}
}  // namespace

constexpr double kMaxTimeUncFrac = 0.05;  // a window is published when its ends are this well-timed
constexpr double kAnchorUncS = 250e-6;     // a read timed this well can start a window
constexpr std::chrono::microseconds kPromptRead{300};  // a read not held up completes within this
constexpr std::chrono::microseconds kSlowRead{1000};   // on a slow queue: a read done later than this was held
constexpr std::chrono::microseconds kSlowQueue{800};   // reads seen pending this long after their post, as a rule
                                                       // (prompt reads take 50-600 us on MI355X)

struct RoundMachine::Slot {
  ReadPort* port = nullptr;
  bool ready = false;  // armed at init (arm_sync)
  // ---- read state: round_mu_ ----
  bool inflight = false;  // a packet with a completion signal is pending on queue q
  int q = 0;
  bool arming = false;    // ... and it is a (re-)arm: start program + baseline read
  bool was_pending = false;  // the pending packet predates this round: one look
  Clock::time_point t_checked{};  // last time the pending packet was seen not complete
  bool seen_pending = false;      // ... by a look after it was posted (its execution time is then
                                  // known only to within [t_checked, the look that saw it done])
  Clock::time_point t_post{};     // when the pending packet was posted
  double pending_seen_s = 0;      // EWMA of how long after its post a read was last seen pending
  uint64_t pending_seen_n = 0;    // reads in that average
  double cum[kNumCtr] = {}, cum_xm[kMaxXcc] = {}, cum_xg[kMaxXcc] = {};
  bool have_cum = false;
  Clock::time_point t_last{};  // when the last read executed (the start of the next window)
  double t_last_unc = 0;       // half-width of t_last's uncertainty (s); 0 for a prompt read
  int zero_grbm = 0;
  int stuck_rounds = 0;
  bool rq_open = false;   // the rescue queue exists
  bool rescued = false;   // reads go to the rescue queue
  bool orphan = false;    // the read abandoned on queue 0 has not completed yet
  int probation = 0;      // back on queue 0 with the rescue queue alive: completed reads to go
  RearmState rs;
  // ---- health: atomics (readers on any thread) ----
  std::atomic<uint64_t> stalls{0}, resets{0}, rearms{0}, rescues{0}, releases{0}, conflicts{0};
  std::atomic<uint64_t> merged{0};  // reads whose time was too uncertain: merged into the next window
  std::atomic<bool> rescue_active{false}, waiting_rearm{false};
  // ---- published window: m_mu ----
  mutable std::mutex m_mu;
  Derived m;
  double last_raw[kNumCtr] = {};
  int last_inst[kNumCtr] = {};
  uint64_t last_samples = 0;
  double last_window_s = 0;
  double pub_cum[kNumCtr] = {};
  Clock::time_point t_window_end{};
};

RoundMachine::RoundMachine(const MachineConfig& c) : cfg_(c), epoch_(Clock::now()) {}

RoundMachine::~RoundMachine() { stop(); }

int64_t RoundMachine::ns(Clock::time_point t) const {
  return int64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(t - epoch_).count()) + 1;
}

void RoundMachine::add(ReadPort* port, const Derived& model) {
  auto s = std::make_unique<Slot>();
  s->port = port;
  s->m = model;
  slots_.push_back(std::move(s));
}

bool RoundMachine::usable(int dev) const {
  if (dev < 0 || size_t(dev) >= slots_.size()) return false;
  const Slot& s = *slots_[size_t(dev)];
  return s.port && s.ready && !s.port->broken.load();
}

bool RoundMachine::arm_sync(int dev) {
  if (dev < 0 || size_t(dev) >= slots_.size() || !slots_[size_t(dev)]->port) return false;
  Slot& s = *slots_[size_t(dev)];
  std::lock_guard<std::mutex> lk(round_mu_);
  if (s.port->broken.load()) return false;
  const auto t0 = Clock::now();
  const auto deadline = t0 + std::chrono::milliseconds(cfg_.arm_timeout_ms);
  s.port->post_arm(cfg_.mode == kCumulative);
  auto pending = t0;  // last seen not complete: the baseline read ran between then and `now`
  for (int i = 0; !s.port->done(0); ++i) {
    pending = Clock::now();
    if (s.port->failed() || pending >= deadline) {
      s.port->broken = true;  // the GPU may still run the packets: it owns the buffers
      return false;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(i == 0 ? cfg_.first_slice_us : cfg_.slice_us));
  }
  const auto now = Clock::now();
  s.t_last = pending + (now - pending) / 2;
  s.t_last_unc = std::chrono::duration<double>(now - pending).count() / 2;
  s.have_cum = false;
  if (cfg_.mode == kCumulative) {
    Sample smp;
    if (!s.port->collect(0, &smp)) return false;
    std::memcpy(s.cum, smp.v, sizeof(s.cum));
    std::memcpy(s.cum_xm, smp.xm, sizeof(s.cum_xm));
    std::memcpy(s.cum_xg, smp.xg, sizeof(s.cum_xg));
    s.have_cum = true;
  }
  rearm_done(s.rs, ns(now));
  s.ready = true;
  return true;
}

void RoundMachine::start() {
  if (cfg_.mode == kReadUnknown) return;  // duty windows: nothing runs here
  {
    std::lock_guard<std::mutex> lk(cv_mu_);
    quit_ = false;
    kick_seq_ = done_seq_ = 0;
    leftover_ = false;
  }
  kick_seq_a_.store(0);
  {
    std::lock_guard<std::mutex> rl(round_mu_);
    round_ = Round{};
    live_ = true;
  }
  thread_ = std::thread([this] { loop(); });
}

void RoundMachine::stop() {
  {
    std::lock_guard<std::mutex> rl(round_mu_);  // no round from here on
    if (!live_ && !thread_.joinable()) return;
    live_ = false;
  }
  {
    std::lock_guard<std::mutex> lk(cv_mu_);
    quit_ = true;
  }
  cv_.notify_all();
  done_cv_.notify_all();
  if (thread_.joinable()) thread_.join();
  std::lock_guard<std::mutex> rl(round_mu_);
  for (size_t i = 0; i < slots_.size(); ++i) {
    Slot& s = *slots_[i];
    if (!usable(int(i))) continue;
    // a packet still pending: its queue is stuck; the GPU may write the buffers later
    if (s.inflight || (s.orphan && !s.port->done(0))) {
      s.port->broken = true;
      continue;
    }
    const int q = s.rescued ? 1 : 0;  // a rescued GPU's first queue may still be stuck
    s.port->post_stop(q);
    const auto deadline = Clock::now() + std::chrono::seconds(1);
    while (!s.port->done(q) && !s.port->failed() && Clock::now() < deadline)
      std::this_thread::sleep_for(std::chrono::microseconds(cfg_.slice_us));
    if (!s.port->done(q)) {
      s.port->broken = true;
      continue;
    }
    if (s.rq_open) {
      s.port->close_rescue();
      s.rq_open = false;
      s.rescue_active = false;
    }
  }
}

// ---------------------------------------------------------------------------------------
// One round: a packet in flight on every GPU at once.  A GPU whose packet is still pending
// from an earlier round gets no new one (it gets one look in this round).
// ---------------------------------------------------------------------------------------
void RoundMachine::post_round_locked(Clock::time_point now) {
  const uint64_t c0 = own_cpu_ns();
  round_.gen += 1;
  round_.waiting.clear();
  const int64_t tn = ns(now);
  for (size_t i = 0; i < slots_.size(); ++i) {
    Slot& s = *slots_[i];
    if (!usable(int(i))) continue;
    if (s.rescued && s.orphan && s.port->done(0)) {
      // the read abandoned on the first queue ran: that queue moves again; reads go back there
      // (the rescue queue stays until probation_rounds reads there complete; a rescue read
      // still in flight is collected first, from its own buffer)
      s.orphan = false;
      s.rescued = false;
      s.probation = cfg_.probation_rounds;
      s.rescue_active = false;
    }
    s.was_pending = s.inflight;
    if (!s.inflight) {
      if (!s.rescued && !s.orphan && rearm_due(s.rs, cfg_.rearm, tn)) {
        s.port->post_arm(cfg_.mode == kCumulative);
        s.q = 0;
        s.arming = true;
        s.seen_pending = false;
      } else {
        s.q = s.rescued ? 1 : 0;
        s.port->post_read(s.q);
        s.arming = false;
        s.seen_pending = false;
      }
      s.inflight = true;
      s.t_checked = now;
      s.t_post = now;
    }
    round_.waiting.push_back(int(i));
  }
  cpu_post_ += own_cpu_ns() - c0;
}

void RoundMachine::round_stuck(Slot& s, int dev, Clock::time_point now) {
  s.t_checked = now;
  s.seen_pending = true;
  ++s.stalls;
  // rescue reads and (re-)arms are never rescued; nor are reads outside cumulative mode (a
  // second queue's read would reset / stop the counters the abandoned one still reads)
  if (s.q == 1 || s.arming || cfg_.mode != kCumulative) return;
  // stuck again while on probation (the rescue queue still exists): back to it at once
  if (++s.stuck_rounds < (s.rq_open ? 1 : cfg_.rescue_rounds)) return;
  if (!s.rq_open) {
    if (!cfg_.rescue || !s.port->open_rescue()) return;
    s.rq_open = true;
    ++s.rescues;
    if (cfg_.log)
      std::fprintf(stderr, "[aqlpmc] gpu %s: counter reads stuck behind a sentinel run the workload leaves no wave "
                   "slot for; reads moved to a queue of their own\n", s.port->label().c_str());
  }
  s.rescued = true;
  s.orphan = true;
  s.probation = 0;
  s.inflight = false;  // abandoned on queue 0 (it still runs, harmlessly, once the queue moves)
  s.stuck_rounds = 0;
  s.rescue_active = true;
}

void RoundMachine::round_done(Slot& s, int dev, Clock::time_point now) {
  s.inflight = false;
  s.stuck_rounds = 0;
  const bool arming = s.arming;
  s.arming = false;
  // The packet executed between the last time it was seen pending and now.  A read never seen
  // pending ran promptly after it was posted (t_checked): reads complete in 50-600 us unless a
  // sentinel run holds the queue, and then a look finds them pending.  Its time is taken from the
  // post, not from how late the look came (a look delayed by scheduling would otherwise move the
  // window's end by half the delay).
  // (A look within kPromptRead of the post that finds it pending says nothing more: it is still
  // a prompt read.  Held reads are those still pending later than that.  A queue whose reads
  // are still pending kSlowQueue after their post as a rule -- its EWMA says so -- is slow: a read first
  // seen done more than kSlowRead after its post may have run anywhere since the last look that
  // found it pending (or since its post), and is held too.  Without that, a sampler descheduled
  // between two looks on a loaded host took a slow queue's read for a prompt one and published
  // a wrong rate; on a prompt queue the same gap says nothing about the read, which ran within
  // its usual time.)
  const auto since = now - s.t_checked;
  const bool slow_queue = s.pending_seen_s > std::chrono::duration<double>(kSlowQueue).count();
  const bool held = (s.seen_pending && s.t_checked - s.t_post > kPromptRead) || (slow_queue && now - s.t_post > kSlowRead);
  if (s.seen_pending) {  // (the first observation seeds the average: a slow queue is slow from its first reads)
    const double v = std::chrono::duration<double>(s.t_checked - s.t_post).count();
    s.pending_seen_s = s.pending_seen_n++ ? 0.8 * s.pending_seen_s + 0.2 * v : v;
  }
  const auto t = held ? s.t_checked + since / 2 : s.t_checked + std::min<Clock::duration>(since, kPromptRead) / 2;
  const double unc = held ? std::chrono::duration<double>(since).count() / 2 : 0.0;
  Sample smp;
  const uint64_t k0 = own_cpu_ns();
  const bool got = s.port->collect(s.q, &smp);
  cpu_collect_ += own_cpu_ns() - k0;
  if (s.q == 0 && s.probation > 0 && --s.probation == 0 && s.rq_open) {
    s.port->close_rescue();
    s.rq_open = false;
    ++s.releases;
    if (cfg_.log)
      std::fprintf(stderr, "[aqlpmc] gpu %s: counter reads complete on the first queue again; rescue queue "
                   "released\n", s.port->label().c_str());
  }
  if (arming) {
    if (!got) return;  // the re-arm stays due: posted again next round
    s.t_last = t;
    s.t_last_unc = unc;
    s.zero_grbm = 0;
    s.have_cum = false;
    if (cfg_.mode == kCumulative) {
      std::memcpy(s.cum, smp.v, sizeof(s.cum));
      std::memcpy(s.cum_xm, smp.xm, sizeof(s.cum_xm));
      std::memcpy(s.cum_xg, smp.xg, sizeof(s.cum_xg));
      s.have_cum = true;
    }
    rearm_done(s.rs, ns(now));
    s.waiting_rearm = false;
    ++s.rearms;
    if (cfg_.log)
      std::fprintf(stderr, "[aqlpmc] gpu %s: counters re-armed after someone else reset or stopped them\n",
                   s.port->label().c_str());
    return;
  }
  if (!got) return;
  const double wall = std::chrono::duration<double>(t - s.t_last).count();
  if (cfg_.mode == kCumulative) {
    double d[kNumCtr], xm[kMaxXcc] = {}, xg[kMaxXcc] = {};
    bool backwards = false;
    for (int k = 0; k < kNumCtr; ++k) {
      d[k] = smp.v[k] - s.cum[k];
      backwards = backwards || d[k] < 0;
    }
    for (int x = 0; x < smp.nxcc && x < kMaxXcc; ++x) {
      xm[x] = std::max(0.0, smp.xm[x] - s.cum_xm[x]);
      xg[x] = std::max(0.0, smp.xg[x] - s.cum_xg[x]);
    }
    const bool first = !s.have_cum;
    // A read that stalled behind a sentinel run is seen complete only at the next round's look:
    // its execution time is uncertain by up to half a tick, and a window ending (or starting) there
    // would carry that error into every rate (a 23 % FLOP/s error on silicon).  Its counts are
    // not lost -- the baseline stays at the last well-timed read, so the next window spans both
    // intervals with well-known ends.  (The error shrinks with the window: a long merged window
    // is accepted once both uncertainties are under 5 % of it.)  A badly-timed read that ends an
    // accepted long window leaves the next window's start uncertain; the next well-timed read
    // then drops that short window and starts a fresh one (below), so one window is lost, not ten.
    if (!first && !backwards && unc + s.t_last_unc > kMaxTimeUncFrac * wall) {
      ++s.merged;
      if (unc <= kAnchorUncS) {
        // this read's own time is good (the bad one was the window's start): the window's counts
        // are dropped unpublished and the next window starts here, well-timed
        std::memcpy(s.cum, smp.v, sizeof(s.cum));
        std::memcpy(s.cum_xm, smp.xm, sizeof(s.cum_xm));
        std::memcpy(s.cum_xg, smp.xg, sizeof(s.cum_xg));
        s.t_last = t;
        s.t_last_unc = unc;
      }
      return;
    }
    std::memcpy(s.cum, smp.v, sizeof(s.cum));
    std::memcpy(s.cum_xm, smp.xm, sizeof(s.cum_xm));
    std::memcpy(s.cum_xg, smp.xg, sizeof(s.cum_xg));
    s.have_cum = true;
    s.t_last = t;
    s.t_last_unc = unc;
    const WindowAction act = window_action(d, first, wall, &s.zero_grbm);
    if (act == kRearm) {
      // reset / re-programmed / stopped under us: this window is unknown
      const bool was_waiting = s.rs.waiting;
      if (!was_waiting || backwards) ++s.resets;
      const uint64_t c0 = s.rs.conflicts;
      rearm_on_reset(s.rs, cfg_.rearm, ns(now), backwards);
      s.conflicts += s.rs.conflicts - c0;
      s.waiting_rearm = true;
      if (cfg_.log && !was_waiting)
        std::fprintf(stderr, "[aqlpmc] gpu %s: counters %s by someone else; windows withheld, re-arm %s\n",
                     s.port->label().c_str(), backwards ? "reset" : "stopped",
                     cfg_.rearm.mode == kRearmOff ? "disabled (GPUEXP_PMC_REARM=off)" : "after a back-off");
      return;
    }
    if (act == kPublish && !s.rs.waiting) publish(s, d, smp, wall, t, smp.v, xm, xg);
  } else {
    // each read restarts the counts: a badly-timed window cannot be merged, only withheld
    if (unc + s.t_last_unc <= kMaxTimeUncFrac * wall) publish(s, smp.v, smp, wall, t, nullptr, nullptr, nullptr);
    else ++s.merged;
    s.t_last = t;
    s.t_last_unc = unc;
    if (cfg_.mode == kStops) {
      // counting stopped at the read: again (one PM4 gap).  The next window counts from the start
      // packet, posted now -- not from the read, which may have been collected late.
      s.port->post_start();
      s.t_last = Clock::now();
      s.t_last_unc = 0;
    }
  }
}

void RoundMachine::look_locked(Clock::time_point now, bool at_deadline, bool final) {
  auto& w = round_.waiting;
  for (auto it = w.begin(); it != w.end();) {
    Slot& s = *slots_[size_t(*it)];
    if (!s.inflight) {  // taken over (rescue) or collected by another pass
      it = w.erase(it);
    } else if (s.port->failed()) {
      s.port->broken = true;
      s.inflight = false;
      it = w.erase(it);
    } else if (s.port->done(s.q)) {
      round_done(s, *it, now);
      it = w.erase(it);
    } else if (s.was_pending || (at_deadline && final)) {  // one look for an old packet
      round_stuck(s, *it, now);
      s.was_pending = false;
      it = w.erase(it);
    } else {
      s.t_checked = now;
      s.seen_pending = true;
      ++it;
    }
  }
}

bool RoundMachine::work(uint64_t gen, Clock::time_point deadline, bool final, const std::atomic<uint64_t>* stop_seq,
                        uint64_t seen_seq) {
  for (int i = 0;; ++i) {
    const uint64_t w0 = own_cpu_ns();
    Clock::time_point now;
    {
      std::lock_guard<std::mutex> lk(round_mu_);
      if (!live_ || round_.gen != gen) return true;  // superseded: the newer round owns the reads
      now = Clock::now();
      const bool at_deadline = now >= deadline;
      const uint64_t k0 = cpu_collect_.load();
      look_locked(now, at_deadline, final);
      cpu_wait_ += own_cpu_ns() - w0 - (cpu_collect_.load() - k0);
      if (round_.waiting.empty()) {
        ++rounds_;
        return true;
      }
      if (at_deadline || (stop_seq && stop_seq->load() != seen_seq)) return false;
    }
    const auto slice = std::chrono::microseconds(i == 0 ? cfg_.first_slice_us : cfg_.slice_us);
    const uint64_t s0 = own_cpu_ns();
    std::this_thread::sleep_for(std::min<Clock::duration>(slice, deadline - now));
    cpu_wait_ += own_cpu_ns() - s0;
  }
}

void RoundMachine::kick() {
  if (cfg_.mode == kReadUnknown) return;
  if (cfg_.inline_rounds) {  // post the round's reads from the caller (no wake-up)
    const auto now = Clock::now();
    last_kick_ns_.store(ns(now));
    std::lock_guard<std::mutex> rl(round_mu_);
    if (live_) post_round_locked(now);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(cv_mu_);
    ++kick_seq_;
    kick_seq_a_.store(kick_seq_);
  }
  cv_.notify_all();
}

int RoundMachine::sync(int timeout_us) {
  if (cfg_.mode == kReadUnknown) return 0;  // duty windows: nothing per tick to wait for
  const auto deadline = Clock::now() + std::chrono::microseconds(std::max(0, timeout_us));
  if (cfg_.inline_rounds) {  // collect the reads posted at the kick (normally complete by now)
    uint64_t gen;
    {
      std::lock_guard<std::mutex> rl(round_mu_);
      if (!live_ || round_.waiting.empty()) return 0;
      gen = round_.gen;
    }
    if (work(gen, deadline, /*final=*/false, nullptr, 0)) return 0;
    {
      std::lock_guard<std::mutex> lk(cv_mu_);
      leftover_ = true;
      leftover_gen_ = gen;
    }
    cv_.notify_all();
    return 1;
  }
  std::unique_lock<std::mutex> lk(cv_mu_);
  const uint64_t want = kick_seq_;
  return wait_until(done_cv_, lk, deadline, [&] { return done_seq_ >= want || quit_; }) ? 0 : 1;
}

void RoundMachine::loop() {
  ::prctl(PR_SET_NAME, "gpuexp-pmc", 0, 0, 0);
  ::prctl(PR_SET_TIMERSLACK, 10000UL, 0, 0, 0);  // 10 us: the polling slices stay short
  const auto interval = std::chrono::milliseconds(cfg_.interval_ms);
  // a stalled GPU costs a thread-run round at most this long (the others' reads are in flight)
  const auto round_limit = std::chrono::milliseconds(std::min(1000, cfg_.interval_ms));
  if (cfg_.inline_rounds) {
    // the engine runs the rounds (kick / sync); this thread follows reads that outlived a
    // sync, and runs rounds itself only when nothing has kicked for a second
    bool idle = false;
    for (;;) {
      bool left = false;
      uint64_t gen = 0;
      {
        std::unique_lock<std::mutex> lk(cv_mu_);
        wait_until(cv_, lk,
                   Clock::now() + (idle ? interval : std::max<Clock::duration>(2 * interval, std::chrono::seconds(1))),
                   [&] { return quit_ || leftover_; });
        if (quit_) break;
        left = leftover_;
        gen = leftover_gen_;
        leftover_ = false;
      }
      if (left) {
        // until each read completed, the next kick took the round over, or an interval passed
        // (then the next round's one look decides)
        work(gen, Clock::now() + interval, /*final=*/false, nullptr, 0);
        thread_cpu_ns_.store(own_cpu_ns());
        continue;
      }
      const int64_t last = last_kick_ns_.load();
      const auto now = Clock::now();
      const int64_t quiet = std::max<int64_t>(1000000000ll, 2000000ll * cfg_.interval_ms);
      idle = !last || ns(now) - last > quiet;
      if (!idle) continue;
      {
        std::lock_guard<std::mutex> rl(round_mu_);
        if (!live_) break;
        post_round_locked(now);
        gen = round_.gen;
      }
      work(gen, now + round_limit, /*final=*/true, nullptr, 0);
      thread_cpu_ns_.store(own_cpu_ns());
    }
    return;
  }
  uint64_t served = 0;
  for (;;) {
    uint64_t target;
    {
      std::unique_lock<std::mutex> lk(cv_mu_);
      // a tick's kick, or on our own every interval when nothing kicks (manual engines)
      wait_until(cv_, lk, Clock::now() + interval, [&] { return quit_ || kick_seq_ != served; });
      if (quit_) break;
      target = kick_seq_;
    }
    const auto begin = Clock::now();
    uint64_t gen;
    {
      std::lock_guard<std::mutex> rl(round_mu_);
      if (!live_) break;
      post_round_locked(begin);
      gen = round_.gen;
    }
    // final at the limit; a newer kick ends the round early (its pending reads get their one
    // look in the next round), so a stuck GPU never delays the next round of the others
    work(gen, begin + round_limit, /*final=*/true, &kick_seq_a_, target);
    thread_cpu_ns_.store(own_cpu_ns());
    served = target;
    {
      std::lock_guard<std::mutex> lk(cv_mu_);
      done_seq_ = target;
    }
    done_cv_.notify_all();
  }
}

// ---------------------------------------------------------------------------------------
// Publication and readers
// ---------------------------------------------------------------------------------------
void RoundMachine::publish(Slot& s, const double* d, const Sample& smp, double wall, Clock::time_point end,
                           const double* cum, const double* xm, const double* xg) {
  std::lock_guard<std::mutex> lk(s.m_mu);
  s.t_window_end = end;
  if (cum) std::memcpy(s.pub_cum, cum, sizeof(s.pub_cum));
  std::memcpy(s.last_raw, d, sizeof(s.last_raw));
  std::memcpy(s.last_inst, smp.inst, sizeof(s.last_inst));
  s.last_samples = smp.samples;
  s.last_window_s = wall;
  if (wall > 0) {
    derive(s.m, d, smp.inst, wall);
    derive_xcc(s.m, xm ? xm : smp.xm, xg ? xg : smp.xg, smp.nxcc);
  }
}

void RoundMachine::publish_window(int dev, const double* d, const Sample& smp, double wall_s) {
  if (dev < 0 || size_t(dev) >= slots_.size()) return;
  publish(*slots_[size_t(dev)], d, smp, wall_s, Clock::now(), nullptr, nullptr, nullptr);
}

int RoundMachine::sample(int dev, double* out) {
  if (dev < 0 || size_t(dev) >= slots_.size() || !slots_[size_t(dev)]->port) return -1;
  Slot& s = *slots_[size_t(dev)];
  std::lock_guard<std::mutex> lk(s.m_mu);
  if (!s.m.valid || s.port->broken.load()) return -1;
  // continuous: a GPU whose reads have been stuck (or withheld) for 2 fallback intervals has no
  // current window; exporting the last one as current would be wrong
  if (cfg_.mode != kReadUnknown && Clock::now() - s.t_window_end > std::chrono::milliseconds(2 * cfg_.interval_ms))
    return -1;
  std::memcpy(out, s.m.latest, sizeof(s.m.latest));
  return 0;
}

int RoundMachine::sample_xcc(int dev, double* out, int max) {
  if (dev < 0 || size_t(dev) >= slots_.size() || !slots_[size_t(dev)]->port || max <= 0) return 0;
  Slot& s = *slots_[size_t(dev)];
  std::lock_guard<std::mutex> lk(s.m_mu);
  if (!s.m.valid || s.port->broken.load()) return 0;
  if (cfg_.mode != kReadUnknown && Clock::now() - s.t_window_end > std::chrono::milliseconds(2 * cfg_.interval_ms))
    return 0;
  const int n = std::min(max, s.m.nxcc);
  for (int x = 0; x < n; ++x) out[x] = s.m.xcc_busy[x];
  return n;
}

int RoundMachine::scope(int dev) {
  if (dev < 0 || size_t(dev) >= slots_.size()) return -1;
  Slot& s = *slots_[size_t(dev)];
  std::lock_guard<std::mutex> lk(s.m_mu);
  return s.m.scope;
}

bool RoundMachine::health(int dev, Health* out) const {
  if (dev < 0 || size_t(dev) >= slots_.size() || !slots_[size_t(dev)]->port) return false;
  const Slot& s = *slots_[size_t(dev)];
  out->stalls = s.stalls.load();
  out->resets = s.resets.load();
  out->rearms = s.rearms.load();
  out->rescues = s.rescues.load();
  out->releases = s.releases.load();
  out->rescue_active = s.rescue_active.load();
  out->waiting_rearm = s.waiting_rearm.load();
  out->conflicts = s.conflicts.load();
  out->broken = s.port->broken.load();
  return true;
}

uint64_t RoundMachine::windows(int dev) const {
  if (dev < 0 || size_t(dev) >= slots_.size()) return 0;
  const Slot& s = *slots_[size_t(dev)];
  std::lock_guard<std::mutex> lk(s.m_mu);
  return s.m.windows;
}

std::string RoundMachine::debug(int dev) {
  if (dev < 0 || size_t(dev) >= slots_.size() || !slots_[size_t(dev)]->port) return "";
  Slot& s = *slots_[size_t(dev)];
  std::lock_guard<std::mutex> lk(s.m_mu);
  char win[64];
  std::snprintf(win, sizeof(win), "%.6f", s.last_window_s);
  std::string out = "samples=" + std::to_string(s.last_samples) + ";windows=" + std::to_string(s.m.windows) + ";merged=" + std::to_string(s.merged.load()) +
                    ";simd=" + std::to_string(s.m.simd) + ";cu=" + std::to_string(s.m.cu) +
                    ";mode=" + (cfg_.mode != kReadUnknown ? read_mode_name(cfg_.mode) : "duty") + ";window_s=" + win +
                    ";resets=" + std::to_string(s.resets.load()) + ";stalls=" + std::to_string(s.stalls.load()) +
                    ";rescued=" + (s.rescues.load() ? "1" : "0") +
                    ";rescue_active=" + (s.rescue_active.load() ? "1" : "0") +
                    ";rescues=" + std::to_string(s.rescues.load()) +
                    ";rescue_releases=" + std::to_string(s.releases.load()) +
                    ";rearms=" + std::to_string(s.rearms.load()) +
                    ";rearm_waiting=" + (s.waiting_rearm.load() ? "1" : "0") + ";";
  if (const uint64_t r = rounds_.load()) {
    char c[200];
    std::snprintf(c, sizeof(c), "rounds=%llu;round_cpu_us_post=%.2f;round_cpu_us_wait=%.2f;round_cpu_us_collect=%.2f;",
                  (unsigned long long)r, cpu_post_.load() / 1e3 / r, cpu_wait_.load() / 1e3 / r,
                  cpu_collect_.load() / 1e3 / r);
    out += c;
  }
  if (cfg_.mode == kCumulative) {
    char c[160];
    std::snprintf(c, sizeof(c), "cum_MFMA=%.0f;cum_GRBM_COUNT=%.0f;cum_GUI=%.0f;", s.pub_cum[kMfma],
                  s.pub_cum[kGrbmCount], s.pub_cum[kGuiActive]);
    out += c;
  }
  for (int k = 0; k < kNumCtr; ++k) {
    char t[128];
    std::snprintf(t, sizeof(t), "%s=%.0f/%d;", name(k), s.last_raw[k], s.last_inst[k]);
    out += t;
  }
  out += "nxcc=" + std::to_string(s.m.nxcc) + ";xcc_busy=";
  for (int x = 0; x < s.m.nxcc; ++x) {
    char t[32];
    std::snprintf(t, sizeof(t), "%s%.2f", x ? "," : "", s.m.xcc_busy[x]);
    out += t;
  }
  return out + ";";
}

}  // namespace gpuexp_pmc
