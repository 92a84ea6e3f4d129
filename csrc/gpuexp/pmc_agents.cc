// match_agents (shared with aql_pmc.cc) and the stub-GPU lifecycle test of pmc_agents.h.
#include "gpuexp/pmc_agents.h"

#include <cctype>
#include <memory>
#include <mutex>
#include <set>
#include <thread>

#include "gpuexp/pmc_fake.h"

namespace gpuexp_pmc {

namespace {
std::string lower(std::string s) {
  for (auto& c : s) c = char(::tolower(static_cast<unsigned char>(c)));
  return s;
}
}  // namespace

AgentMatch match_agents(int ndev, const char* const* bdfs, const std::vector<std::string>& gpu_bdfs) {
  AgentMatch m;
  m.gpu_of.assign(size_t(std::max(0, ndev)), -1);
  m.reserved.assign(size_t(std::max(0, ndev)), false);
  std::vector<bool> taken(gpu_bdfs.size(), false);
  for (int d = 0; d < ndev; ++d) {
    const bool off = bdfs[d][0] == '-';  // reserve the agent, no queue (queue_devices)
    const std::string want = lower(bdfs[d] + (off ? 1 : 0));
    for (size_t gi = 0; gi < gpu_bdfs.size(); ++gi) {
      if (taken[gi] || want != lower(gpu_bdfs[gi])) continue;
      taken[gi] = true;  // the k-th device with a BDF gets the k-th agent with it (partitions)
      if (off) {
        m.reserved[size_t(d)] = true;
        m.n_reserved += 1;
      } else {
        m.gpu_of[size_t(d)] = int(gi);
      }
      break;
    }
  }
  return m;
}

namespace {

// The stub runtime: hands out queue / signal ids and heap buffers and keeps track of them.
struct StubRuntime {
  std::mutex mu;
  int next = 1;
  std::set<int> queues, signals;
  std::set<void*> buffers;
  int queues_created = 0, signals_created = 0, buffers_allocated = 0;
  int double_release = 0, foreign_release = 0;
  int fail_queue_gpu = -1;  // create_queue fails for this GPU (its setup fails)
  ~StubRuntime() {
    for (void* b : buffers) delete[] static_cast<char*>(b);  // the runtime's own shutdown
  }
};

struct StubOps {
  StubRuntime* rt;
  int gpu;
  bool create_queue(int* q) {
    std::lock_guard<std::mutex> lk(rt->mu);
    if (gpu == rt->fail_queue_gpu) return false;
    *q = rt->next++;
    rt->queues.insert(*q);
    rt->queues_created += 1;
    return true;
  }
  void destroy_queue(int q) {
    std::lock_guard<std::mutex> lk(rt->mu);
    if (!rt->queues.erase(q)) rt->double_release += 1;
  }
  bool valid(int h) const { return h != 0; }
  bool create_signal(int* s) {
    std::lock_guard<std::mutex> lk(rt->mu);
    *s = rt->next++;
    rt->signals.insert(*s);
    rt->signals_created += 1;
    return true;
  }
  void destroy_signal(int s) {
    std::lock_guard<std::mutex> lk(rt->mu);
    if (!rt->signals.erase(s)) rt->double_release += 1;
  }
  void* alloc(size_t n) {
    auto* p = new char[n];
    std::lock_guard<std::mutex> lk(rt->mu);
    rt->buffers.insert(p);
    rt->buffers_allocated += 1;
    return p;
  }
  void release(void* p) {
    std::lock_guard<std::mutex> lk(rt->mu);
    if (!rt->buffers.erase(p)) {
      rt->foreign_release += 1;
      return;
    }
    delete[] static_cast<char*>(p);
  }
};

// aql_pmc.cc's Agent on a stub runtime: the lifecycle through pmc_agents.h, the packets through a
// scripted fake GPU (pmc_fake.h).
struct StubAgent : ReadPort, AgentResources<int, int> {
  StubAgent(StubRuntime* rt, int gpu, const FakeScript& s, Clock::time_point t0)
      : ops{rt, gpu}, fake(s, t0, gpu) {}
  bool setup() {  // aql_pmc.cc setup_agent: buffers, then queue + signal
    cmd_buf = ops.alloc(4096);
    out_buf = ops.alloc(4096);
    return cmd_buf && out_buf && ops.create_queue(&queue) && ops.create_signal(&sig);
  }
  void post_read(int q) override { fake.post_read(q); }
  void post_arm(bool b) override { fake.post_arm(b); }
  void post_start() override { fake.post_start(); }
  void post_stop(int q) override { fake.post_stop(q); }
  bool done(int q) override { return fake.done(q); }
  bool failed() override { return fake.failed(); }
  bool collect(int q, Sample* out) override { return fake.collect(q, out); }
  bool open_rescue() override {
    return gpuexp_pmc::open_rescue(ops, *this, 4096, 4096, [this] { return fake.open_rescue(); });
  }
  void close_rescue() override {
    if (ops.valid(rq)) fake.close_rescue();
    gpuexp_pmc::close_rescue(ops, *this);
  }
  std::string label() const override { return fake.label(); }
  StubOps ops;
  FakePort fake;
  bool ready = false;
};

}  // namespace

LifecycleOutcome run_agent_lifecycle(int gpus, int failing_gpu, int starved_gpu, int broken_gpu, int ticks) {
  LifecycleOutcome out;
  StubRuntime rt;
  rt.fail_queue_gpu = failing_gpu;
  // gpus runtime agents plus one more the engine reserves without a queue ('-', queue_devices);
  // engine devices list them in reverse, so matching is by BDF, not position
  std::vector<std::string> gpu_bdfs;
  for (int g = 0; g <= gpus; ++g) {
    char b[32];
    std::snprintf(b, sizeof(b), "0000:%02X:00.0", 0x10 + 0x10 * g);
    gpu_bdfs.push_back(b);
  }
  std::vector<std::string> names;
  for (int g = gpus; g >= 0; --g) names.push_back((g == gpus ? "-" : "") + lower(gpu_bdfs[size_t(g)]));
  std::vector<const char*> bdfs;
  for (auto& n : names) bdfs.push_back(n.c_str());
  const int ndev = int(bdfs.size());
  out.devices = ndev;
  const AgentMatch m = match_agents(ndev, bdfs.data(), gpu_bdfs);

  const auto t0 = Clock::now();
  std::vector<std::unique_ptr<StubAgent>> agents;
  agents.resize(size_t(ndev));
  for (int d = 0; d < ndev; ++d) {
    const int gi = m.gpu_of[size_t(d)];
    if (gi < 0) continue;
    out.matched += 1;
    FakeScript s;
    s.latency_us = 30;
    if (gi == starved_gpu) s.stalls = {{40000, 200000}};  // queue 0 stuck behind a sentinel run
    agents[size_t(d)] = std::make_unique<StubAgent>(&rt, gi, s, t0);
    agents[size_t(d)]->ready = agents[size_t(d)]->setup();
    out.usable += agents[size_t(d)]->ready;
  }

  MachineConfig mc;
  mc.inline_rounds = true;
  mc.interval_ms = 20;
  mc.log = false;
  RoundMachine machine(mc);
  gpuexp_ctr::Derived model;
  model.simd = 1024;
  model.cu = 256;
  model.privileged = true;
  for (auto& a : agents) machine.add(a && a->ready ? a.get() : nullptr, model);
  for (int d = 0; d < ndev; ++d)
    if (agents[size_t(d)] && agents[size_t(d)]->ready) out.armed += machine.arm_sync(d);
  machine.start();
  auto next = Clock::now();
  for (int t = 0; t < ticks; ++t) {
    machine.kick();
    std::this_thread::sleep_for(std::chrono::microseconds(300));
    machine.sync(2000);
    next += std::chrono::milliseconds(10);
    std::this_thread::sleep_until(next);
  }
  machine.stop();
  for (int d = 0; d < ndev; ++d) {
    out.windows.push_back(machine.windows(d));
    const int gi = m.gpu_of[size_t(d)];
    if (gi == failing_gpu) out.windows_on_failed_gpu += int(machine.windows(d));
  }
  // teardown, as aql_pmc.cc teardown_locked: a GPU marked broken keeps its buffers
  for (int d = 0; d < ndev; ++d) {
    StubAgent* a = agents[size_t(d)].get();
    if (!a) continue;
    out.rescues_opened += a->fake.opened();
    out.rescues_closed += a->fake.closed();
    const bool broken = m.gpu_of[size_t(d)] == broken_gpu || a->broken.load();
    out.buffers_left_by_design += release_agent(a->ops, *a, broken);
  }
  {
    std::lock_guard<std::mutex> lk(rt.mu);
    out.queues_created = rt.queues_created;
    out.queues_live = int(rt.queues.size());
    out.signals_created = rt.signals_created;
    out.signals_live = int(rt.signals.size());
    out.buffers_allocated = rt.buffers_allocated;
    out.buffers_live = int(rt.buffers.size());
    out.double_release = rt.double_release;
    out.foreign_release = rt.foreign_release;
  }
  agents.clear();
  return out;  // rt's destructor frees the buffers left by design (the runtime's shutdown)
}

}  // namespace gpuexp_pmc
