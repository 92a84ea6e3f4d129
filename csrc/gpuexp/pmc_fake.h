// Scripted fake GPUs for the PMC read machine (pmc_rounds.h): the CPU stand-in of aql_pmc.cc's
// HSA queues, so the round / rescue / probation / re-arm / leftover logic runs in the CPU tests
// (tests/test_pmc_rounds.py) and under TSan / ASan (csrc/tests/pmc_harness_main.cc).
//
// Model.  Each queue executes its packets in order, one `latency_us` each once the queue
// reaches them; queue 0 does not advance inside a stall window (a sentinel dispatch the
// workload leaves no wave slot for).  The counters are chip state shared by both queues: they
// count `rate` per second (times a fixed multiple per counter) since the last start program --
// the exporter's own (an arm) or someone else's (a foreign reset) -- and stand still while
// someone else has stopped them.  A read's output is the counters at the moment it executes.
// Every packet records when it completed, when the machine first looked at it and when it was
// first seen complete, and how often its output was collected, so a test can check that no
// GPU's window is held by another's and that every read is collected exactly once.
#pragma once

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "gpuexp/pmc_rounds.h"

namespace gpuexp_pmc {

struct FakeScript {
  int64_t latency_us = 40;                            // execution time of one packet
  std::vector<std::pair<int64_t, int64_t>> stalls;    // queue 0 stands still in [a, b) (us)
  std::vector<int64_t> resets;                        // someone else's start program at t (us)
  std::vector<std::pair<int64_t, int64_t>> stops;     // someone else stops counting at a; starts again at b (b < 0: never)
  int64_t queue_error_at = -1;                        // the queue fails at t (us); -1 never
  bool rescue_fails = false;                          // open_rescue cannot create a second queue
  double rate = 1.0e9;                                // GRBM_COUNT per second
  int read_mode = 0;                                  // what a read does: 0 nothing (cumulative), 1 resets, 2 stops
};

class FakePort : public ReadPort {
 public:
  enum Kind { kRead = 0, kArm = 1, kStart = 2, kStop = 3 };
  struct Packet {
    int q = 0;
    Kind kind = kRead;
    bool signaled = true;
    bool reads = true;      // writes the output buffer
    int64_t post = 0, complete = 0;
    int64_t first_look = -1, seen = -1;  // done() calls on this packet (its signal's last packet)
    int collected = 0;
  };

  FakePort(const FakeScript& s, Clock::time_point t0, int index) : s_(s), t0_(t0), index_(index) {
    for (int64_t t : s.resets) events_.push_back({t, true});
    for (auto& st : s.stops) {
      events_.push_back({st.first, false});
      if (st.second >= 0) events_.push_back({st.second, true});
    }
  }

  // ---- ReadPort ----
  void post_read(int q) override { push(q, kRead, true, true); }
  void post_arm(bool baseline) override {
    if (baseline) {
      push(0, kStart, false, false);
      push(0, kArm, true, true);
    } else {
      push(0, kStart, true, false);
    }
  }
  void post_start() override { push(0, kStart, false, false); }
  void post_stop(int q) override { push(q, kStop, true, false); }
  bool done(int q) override {
    std::lock_guard<std::mutex> lk(mu_);
    Packet* p = last_signaled(q);
    if (!p) return true;
    const int64_t t = now();
    if (p->first_look < 0) p->first_look = t;
    const bool d = t >= p->complete;
    if (d && p->seen < 0) p->seen = t;
    return d;
  }
  bool failed() override { return s_.queue_error_at >= 0 && now() >= s_.queue_error_at; }
  bool collect(int q, Sample* out) override {
    std::lock_guard<std::mutex> lk(mu_);
    const int64_t t = now();
    Packet* best = nullptr;
    for (auto& p : packets_)
      if (p.q == q && p.reads && p.complete <= t && (!best || p.complete > best->complete)) best = &p;
    if (!best) return false;
    best->collected += 1;
    fill(best->complete, out);
    return true;
  }
  bool open_rescue() override {
    std::lock_guard<std::mutex> lk(mu_);
    if (s_.rescue_fails) return false;
    if (rq_open_) double_open_ += 1;
    rq_open_ = true;
    opened_ += 1;
    q1_tail_ = 0;
    return true;
  }
  void close_rescue() override {
    std::lock_guard<std::mutex> lk(mu_);
    if (!rq_open_) double_close_ += 1;
    rq_open_ = false;
    closed_ += 1;
  }
  std::string label() const override { return "fake:" + std::to_string(index_); }

  // ---- inspection (after the machine stopped) ----
  std::vector<Packet> packets() {
    std::lock_guard<std::mutex> lk(mu_);
    return packets_;
  }
  int opened() const { return opened_; }
  int closed() const { return closed_; }
  int misuse() const { return double_open_ + double_close_ + post_on_closed_; }
  bool rescue_open() const { return rq_open_; }
  int64_t now() const {
    return int64_t(std::chrono::duration_cast<std::chrono::microseconds>(Clock::now() - t0_).count());
  }
  // Counter multiples per GRBM_COUNT (so a test knows what a correct window derives to).
  static double mult(int k) {
    using namespace gpuexp_ctr;
    switch (k) {
      case kGrbmCount: return 1.0;
      case kGuiActive: return 0.5;       // GPU busy 50 %
      case kMfma: return 0.25 * 1024;    // MFMA busy 25 % of 1024 SIMDs
      case kDramRd32: return 0.01;       // HBM read = 0.32 B per GRBM clock
      default: return 0.001 * (k + 1);
    }
  }

 private:
  struct Ev {
    int64_t t;
    bool start;  // start (reset + counting) / stop
  };

  void push(int q, Kind k, bool signaled, bool reads) {
    std::lock_guard<std::mutex> lk(mu_);
    if (q == 1 && !rq_open_) {
      post_on_closed_ += 1;
      return;
    }
    const int64_t t = now();
    int64_t& tail = q == 1 ? q1_tail_ : q0_tail_;
    int64_t ready = std::max(t, tail);
    for (bool moved = true; q == 0 && moved;) {
      moved = false;
      for (auto& st : s_.stalls)
        if (ready >= st.first && ready < st.second) {
          ready = st.second;
          moved = true;
        }
    }
    Packet p;
    p.q = q;
    p.kind = k;
    p.signaled = signaled;
    p.reads = reads;
    p.post = t;
    p.complete = ready + s_.latency_us;
    tail = p.complete;
    packets_.push_back(p);
    if (k == kStart) events_.push_back({p.complete, true});
    if (k == kStop) events_.push_back({p.complete, false});
    if (k == kRead && s_.read_mode == 1) events_.push_back({p.complete, true});   // the read resets
    if (k == kRead && s_.read_mode == 2) events_.push_back({p.complete, false});  // the read stops counting
  }

  Packet* last_signaled(int q) {
    for (auto it = packets_.rbegin(); it != packets_.rend(); ++it)
      if (it->q == q && it->signaled) return &*it;
    return nullptr;
  }

  // Counting seconds just before time t (a read at t sees the counters before its own effect):
  // since the last start event, minus stopped time.
  double counting_s(int64_t t) {
    std::vector<Ev> ev;
    for (auto& e : events_)
      if (e.t < t) ev.push_back(e);
    std::stable_sort(ev.begin(), ev.end(), [](const Ev& a, const Ev& b) { return a.t < b.t; });
    bool on = false;
    int64_t last = 0, acc = 0;
    for (auto& e : ev) {
      if (on) acc += e.t - last;
      last = e.t;
      if (e.start) {
        acc = 0;
        on = true;
      } else {
        on = false;
      }
    }
    if (on) acc += t - last;
    return double(acc) * 1e-6;
  }

  void fill(int64_t t, Sample* out) {
    const double c = counting_s(t) * s_.rate;
    *out = Sample{};
    for (int k = 0; k < kNumCtr; ++k) {
      out->v[k] = c * mult(k);
      out->inst[k] = 1;
    }
    out->samples = kNumCtr;
    out->nxcc = 8;
    for (int x = 0; x < 8; ++x) {
      out->xm[x] = out->v[gpuexp_ctr::kMfma] / 8;
      out->xg[x] = out->v[gpuexp_ctr::kGrbmCount];
    }
  }

  FakeScript s_;
  Clock::time_point t0_;
  int index_;
  std::mutex mu_;
  std::vector<Packet> packets_;
  std::vector<Ev> events_;
  int64_t q0_tail_ = 0, q1_tail_ = 0;
  bool rq_open_ = false;
  int opened_ = 0, closed_ = 0, double_open_ = 0, double_close_ = 0, post_on_closed_ = 0;
};

// A scenario: `gpus` fake GPUs driven the way the engine drives the plugin -- per tick a kick,
// `work_us` of device reads, a sync of up to `sync_us`, then every GPU's sample -- while a
// reader thread calls the machine's readers concurrently (the engine's HTTP / series paths).
struct HarnessConfig {
  int gpus = 8;
  int ticks = 60;
  int tick_us = 10000;
  int work_us = 300;
  int sync_us = 2000;
  bool inline_rounds = true;
  bool kick_at_end = false;  // the engine's counters_kick=end: kick after the tick, sync in the next
  bool reader = true;
  MachineConfig machine;     // mode / interval / rescue / re-arm (inline_rounds is taken from above)
  std::vector<FakeScript> scripts;  // one per GPU (missing: defaults)
};

struct GpuOutcome {
  Health health;
  uint64_t windows = 0;        // published windows (Derived.windows)
  int fresh_ticks = 0;         // ticks whose sample() after sync returned a window
  int bad_windows = 0;         // fresh samples whose derived rates were off by > rate_tolerance
  double worst_rate_err = 0;   // |HBM read B/s / expected - 1|, worst fresh sample
  int packets = 0, reads_completed = 0, uncollected = 0, double_collected = 0;
  int arms = 0;                // arm packets posted after init
  int64_t max_lateness_us = 0; // seen - max(complete, first look), over collected packets
  int rescue_opened = 0, rescue_closed = 0, misuse = 0;
  bool rescue_open_at_end = false;
};

struct HarnessOutcome {
  std::vector<GpuOutcome> gpus;
  int ticks = 0;
  int late_syncs = 0;          // syncs that returned 1 (reads left over)
  int64_t max_sync_us = 0;     // longest sync call
  int64_t max_kick_us = 0;     // longest kick call
  uint64_t reader_calls = 0;
  bool armed_all = false;
  std::string error;
};

HarnessOutcome run_pmc_harness(const HarnessConfig& cfg, double rate_tolerance = 0.1);

}  // namespace gpuexp_pmc
