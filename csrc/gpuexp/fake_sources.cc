// In-process stand-ins of the GPU-side optional sources for the fake-host engine (tests and
// tools/project_cpu.py): the real PMC read machine (pmc_rounds.cc) over scripted fake GPUs
// (pmc_fake.h), and a sentinel, each burning the per-GPU host CPU measured on MI355X for the
// work they stand for.  The 8-GPU CPU projection then carries the sentinel and counters
// stages that scale with the GPU count (VERDICT r05 Next #2: round 5's fake host had neither,
// 0.4 us/tick for 8 GPUs against 2.2-6.2 / 11.3-16.9 us per GPU per tick on silicon).
#include <cmath>

#include "gpuexp/common.h"
#include "gpuexp/pmc_fake.h"
#include "gpuexp/sources.h"

namespace gpuexp {

namespace {

void burn_cpu_us(uint64_t us) {
  if (!us) return;
  const uint64_t c0 = thread_cpu_ns();
  uint64_t c = c0;
  while ((c = thread_cpu_ns()) - c0 < us * 1000) {
  }
  fake_cpu_burnt_ns().fetch_add(c - c0, std::memory_order_relaxed);
}

// A fake GPU's read path that costs host CPU like an HSA queue's: writing the AQL packet and
// ringing the doorbell at post (a quarter), reducing the output buffer at collect (the rest).
class CostPort : public gpuexp_pmc::ReadPort {
 public:
  CostPort(std::unique_ptr<gpuexp_pmc::FakePort> p, uint64_t cost_us) : p_(std::move(p)), cost_us_(cost_us) {}
  void post_read(int q) override {
    burn_cpu_us(cost_us_ / 4);
    p_->post_read(q);
  }
  void post_arm(bool baseline_read) override { p_->post_arm(baseline_read); }
  void post_start() override { p_->post_start(); }
  void post_stop(int q) override { p_->post_stop(q); }
  bool done(int q) override { return p_->done(q); }
  bool failed() override { return p_->failed(); }
  bool collect(int q, gpuexp_pmc::Sample* out) override {
    const bool ok = p_->collect(q, out);
    burn_cpu_us(cost_us_ - cost_us_ / 4);
    return ok;
  }
  bool open_rescue() override { return p_->open_rescue(); }
  void close_rescue() override { p_->close_rescue(); }
  std::string label() const override { return p_->label(); }

 private:
  std::unique_ptr<gpuexp_pmc::FakePort> p_;
  uint64_t cost_us_;
};

class FakeCounters : public CounterSource {
 public:
  FakeCounters(uint64_t cost_us, int interval_ms, bool inline_rounds,
               std::vector<std::pair<int64_t, int64_t>> stalls_us)
      : cost_us_(cost_us), stalls_us_(std::move(stalls_us)) {
    mc_.interval_ms = interval_ms;
    mc_.inline_rounds = inline_rounds;
    mc_.log = false;
  }
  ~FakeCounters() override { stop(); }

  bool start(const std::vector<DeviceInfo>& devs, std::string* err) override {
    m_ = std::make_unique<gpuexp_pmc::RoundMachine>(mc_);
    const auto t0 = gpuexp_pmc::Clock::now();
    gpuexp_ctr::Derived model;
    model.simd = 1024;
    model.cu = 256;
    model.privileged = true;
    for (size_t i = 0; i < devs.size(); ++i) {
      gpuexp_pmc::FakeScript s;
      s.latency_us = 20;  // a PM4 counter read on MI355X: tens of microseconds
      s.stalls = stalls_us_;
      ports_.push_back(std::make_unique<CostPort>(std::make_unique<gpuexp_pmc::FakePort>(s, t0, int(i)), cost_us_));
      m_->add(devs[i].queue_enabled ? ports_.back().get() : nullptr, model);
    }
    for (size_t i = 0; i < devs.size(); ++i)
      if (devs[i].queue_enabled && !m_->arm_sync(int(i))) {
        *err = "fake PMC arm failed";
        return false;
      }
    m_->start();
    started_ = true;
    return true;
  }
  void kick() override {
    if (started_) m_->kick();
  }
  bool sync(int timeout_us) override { return !started_ || m_->sync(timeout_us) == 0; }
  uint64_t cpu_ns() override { return started_ ? m_->thread_cpu_ns() : 0; }
  bool sample(int dev, double dt_s, CounterReading* out) override {
    double v[kCounterOutputs];
    if (!started_ || m_->sample(dev, v) != 0) return false;
    fill_counter_reading(v, out);
    out->nxcc = std::max(0, m_->sample_xcc(dev, out->xcc_mfma_busy_pct, kMaxXcc));
    return true;
  }
  int scope(int dev) override { return started_ ? m_->scope(dev) : -1; }
  bool health(int dev, CounterHealth* out) override {
    gpuexp_pmc::Health h;
    if (!started_ || !m_->health(dev, &h)) return false;
    out->stalls = h.stalls;
    out->resets = h.resets;
    out->rearms = h.rearms;
    out->rescues = h.rescues;
    out->releases = h.releases;
    out->rescue_active = h.rescue_active;
    return true;
  }
  void stop() override {
    if (started_) m_->stop();
    started_ = false;
  }
  std::string status() const override {
    return "fake PMC read machine (" + std::to_string(cost_us_) + " us CPU per GPU read)";
  }

 private:
  uint64_t cost_us_;
  std::vector<std::pair<int64_t, int64_t>> stalls_us_;
  gpuexp_pmc::MachineConfig mc_;
  std::unique_ptr<gpuexp_pmc::RoundMachine> m_;
  std::vector<std::unique_ptr<CostPort>> ports_;
  bool started_ = false;
};

// Drain + dispatch of one sentinel run per GPU per tick(), each burning `cost_us` of CPU (the
// raw-AQL dispatch on the PMC queue and the pinned-ring drain, profiles/r05 c5*.json).
class FakeSentinel : public SentinelSource {
 public:
  explicit FakeSentinel(uint64_t cost_us) : cost_us_(cost_us) {}
  bool start(const std::vector<DeviceInfo>& devs, std::string*) override {
    runs_.assign(devs.size(), 0);
    return true;
  }
  void tick(uint64_t) override {
    for (auto& r : runs_) {
      burn_cpu_us(cost_us_);
      r += 1;
    }
  }
  bool read(int dev, SentinelReading* out) override {
    if (dev < 0 || size_t(dev) >= runs_.size() || !runs_[size_t(dev)]) return false;
    out->ok = true;
    out->sclk_hz = 2.4e9;
    out->dispatch_latency_s = 13e-6;
    out->xcc_id = dev % kMaxXcc;
    out->runs = runs_[size_t(dev)];
    out->pending_s = 0;
    out->mem_latency_s = 1.2e-6;
    for (int x = 0; x < kMaxXcc; ++x) {
      out->xcc_latency_s[x] = 13e-6;
      out->xcc_mem_latency_s[x] = 1.2e-6;
    }
    return true;
  }
  void stop() override {}
  std::string status() const override {
    return "fake sentinel (" + std::to_string(cost_us_) + " us CPU per GPU run)";
  }

 private:
  uint64_t cost_us_;
  std::vector<uint64_t> runs_;
};

}  // namespace

std::unique_ptr<CounterSource> make_fake_counters(uint64_t cost_us, int interval_ms, bool inline_rounds,
                                                  const std::vector<std::pair<int64_t, int64_t>>& stalls_us) {
  return std::make_unique<FakeCounters>(cost_us, interval_ms, inline_rounds, stalls_us);
}

std::unique_ptr<SentinelSource> make_fake_sentinel(uint64_t cost_us) {
  return std::make_unique<FakeSentinel>(cost_us);
}

}  // namespace gpuexp
