// run_pmc_harness: the PMC read machine on scripted fake GPUs (pmc_fake.h), driven the way the
// engine drives the aqlprofile plugin, with a concurrent reader.  Used by tests/test_pmc_rounds.py
// (through the _gpuexp module) and by the sanitizer driver csrc/tests/pmc_harness_main.cc.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include "gpuexp/pmc_fake.h"

namespace gpuexp_pmc {

HarnessOutcome run_pmc_harness(const HarnessConfig& cfg, double rate_tolerance) {
  HarnessOutcome out;
  const auto t0 = Clock::now();
  std::vector<std::unique_ptr<FakePort>> ports;
  for (int i = 0; i < cfg.gpus; ++i)
    ports.push_back(std::make_unique<FakePort>(size_t(i) < cfg.scripts.size() ? cfg.scripts[size_t(i)] : FakeScript{},
                                               t0, i));
  MachineConfig mc = cfg.machine;
  mc.inline_rounds = cfg.inline_rounds;
  RoundMachine m(mc);
  gpuexp_ctr::Derived model;
  model.simd = 1024;
  model.cu = 256;
  model.privileged = true;
  for (auto& p : ports) m.add(p.get(), model);
  out.armed_all = true;
  for (int i = 0; i < cfg.gpus; ++i) out.armed_all = m.arm_sync(i) && out.armed_all;
  std::vector<int> init_arms(size_t(cfg.gpus), 0);
  for (int i = 0; i < cfg.gpus; ++i)
    for (auto& p : ports[size_t(i)]->packets()) init_arms[size_t(i)] += p.kind == FakePort::kArm || (p.kind == FakePort::kStart && p.signaled);
  m.start();

  std::atomic<bool> stop{false};
  std::atomic<uint64_t> reader_calls{0};
  std::thread reader;
  if (cfg.reader)
    reader = std::thread([&] {
      double v[gpuexp_ctr::kNumOut], x[gpuexp_ctr::kMaxXcc];
      Health h;
      while (!stop.load()) {
        for (int i = 0; i < cfg.gpus; ++i) {
          m.sample(i, v);
          m.sample_xcc(i, x, gpuexp_ctr::kMaxXcc);
          m.health(i, &h);
          m.scope(i);
          if ((reader_calls.load() & 63) == 0) (void)m.debug(i);
          reader_calls += 1;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      }
    });

  out.gpus.resize(size_t(cfg.gpus));
  std::vector<uint64_t> last_windows(size_t(cfg.gpus), 0);
  // expected HBM read rate of a correct window: rate x mult(DRAM) x 32 B
  auto tick_start = Clock::now();
  for (int t = 0; t < cfg.ticks; ++t) {
    if (!cfg.kick_at_end || t == 0) {
      const auto k0 = Clock::now();
      m.kick();
      out.max_kick_us = std::max<int64_t>(out.max_kick_us, std::chrono::duration_cast<std::chrono::microseconds>(
                                                                Clock::now() - k0).count());
    }
    std::this_thread::sleep_for(std::chrono::microseconds(cfg.work_us));  // the tick's device reads
    const auto s0 = Clock::now();
    if (m.sync(cfg.sync_us) != 0) out.late_syncs += 1;
    out.max_sync_us = std::max<int64_t>(out.max_sync_us, std::chrono::duration_cast<std::chrono::microseconds>(
                                                              Clock::now() - s0).count());
    for (int i = 0; i < cfg.gpus; ++i) {
      GpuOutcome& g = out.gpus[size_t(i)];
      const uint64_t w = m.windows(i);
      const bool fresh = w > last_windows[size_t(i)];
      last_windows[size_t(i)] = w;
      double v[gpuexp_ctr::kNumOut];
      if (m.sample(i, v) != 0 || !fresh) continue;
      g.fresh_ticks += 1;
      const FakeScript s = size_t(i) < cfg.scripts.size() ? cfg.scripts[size_t(i)] : FakeScript{};
      // a window over a foreign stop publishes zero rates once (window_action); the first window
      // after init is too short for the rate check
      if (!s.stops.empty() || t == 0) continue;
      const double want = s.rate * FakePort::mult(gpuexp_ctr::kDramRd32) * 32.0;
      const double err = std::fabs(v[6] / want - 1.0);
      g.worst_rate_err = std::max(g.worst_rate_err, err);
      if (!(err <= rate_tolerance) || std::fabs(v[2] - 50.0) > 100 * rate_tolerance) g.bad_windows += 1;
    }
    if (cfg.kick_at_end) m.kick();
    tick_start += std::chrono::microseconds(cfg.tick_us);
    std::this_thread::sleep_until(tick_start);
    out.ticks += 1;
  }
  stop.store(true);
  if (reader.joinable()) reader.join();
  out.reader_calls = reader_calls.load();
  for (int i = 0; i < cfg.gpus; ++i) m.health(i, &out.gpus[size_t(i)].health);
  // windows published (through debug: "windows=N;")
  for (int i = 0; i < cfg.gpus; ++i) {
    const std::string d = m.debug(i);
    const size_t p = d.find("windows=");
    out.gpus[size_t(i)].windows = p == std::string::npos ? 0 : std::strtoull(d.c_str() + p + 8, nullptr, 10);
  }
  // reads that completed before the machine stopped must all have been collected (those that
  // completed within the last two ticks may still have been waiting for a look: a counting
  // thread descheduled on a loaded host looks late, and stop() does not wait for it)
  const int64_t end = (ports.empty() ? 0 : ports[0]->now()) - 2 * int64_t(cfg.tick_us);
  m.stop();
  for (int i = 0; i < cfg.gpus; ++i) {
    GpuOutcome& g = out.gpus[size_t(i)];
    FakePort& p = *ports[size_t(i)];
    int arms = 0;
    for (auto& k : p.packets()) {
      g.packets += 1;
      arms += k.kind == FakePort::kArm || (k.kind == FakePort::kStart && k.signaled);
      if (!k.reads) continue;
      if (k.complete <= end) g.reads_completed += 1;
      if (k.collected > 1) g.double_collected += 1;
      if (k.collected == 0 && k.complete <= end) g.uncollected += 1;
      if (k.collected >= 1 && k.seen >= 0) {
        const int64_t from = std::max(k.complete, k.first_look);
        g.max_lateness_us = std::max<int64_t>(g.max_lateness_us, k.seen - from);
        if (std::getenv("PMC_HARNESS_DEBUG") && k.seen - from > 400)
          std::fprintf(stderr, "gpu %d q%d kind %d post %lld complete %lld first_look %lld seen %lld\n", i, k.q, int(k.kind),
                       (long long)k.post, (long long)k.complete, (long long)k.first_look, (long long)k.seen);
      }
    }
    g.arms = arms - init_arms[size_t(i)];
    g.rescue_opened = p.opened();
    g.rescue_closed = p.closed();
    g.misuse = p.misuse();
    g.rescue_open_at_end = p.rescue_open();
  }
  return out;
}

}  // namespace gpuexp_pmc
