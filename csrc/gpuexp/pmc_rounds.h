// The continuous-counting read machine of the aqlprofile PMC plugin, behind a small
// queue-and-signal interface (ReadPort), so the same code runs on HSA queues in production
// (aql_pmc.cc) and on scripted fake GPUs in the CPU tests (pmc_fake.h, tests/test_pmc_rounds.py,
// the tsan / asan presets).
//
// A read round posts one read packet per GPU at once and collects each GPU as soon as its read
// completes, so one stuck GPU never holds the others' windows.  The rest is per-GPU state:
//   * a read still pending at its round's end gets ONE look in the next round, then counts
//     as a stall; after kRescueRounds stalls its reads move to a rescue queue of their own
//     (the first queue is stuck behind a sentinel dispatch the workload leaves no wave slot
//     for), and back once the abandoned read completes, the rescue queue being released after
//     kProbationRounds completed reads (rescue -> probation -> release);
//   * a window whose counters went backwards or stood still means someone else reset or
//     stopped them: windows are withheld and counting is re-armed asynchronously (start +
//     baseline read as one packet pair, never a blocking wait) after a back-off
//     (counter_model.h rearm_on_reset);
//   * in inline mode (the engine's sampler runs each round: kick at the tick's start, sync
//     before its series stage) reads that outlive the sync wait are followed by the counting
//     thread until they complete or the next kick takes the round over (leftover hand-off).
// The per-device loop this replaces in the reference: /root/reference/main.go:123-138.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gpuexp/counter_model.h"

namespace gpuexp_pmc {

using gpuexp_ctr::kMaxXcc;
using gpuexp_ctr::kNumCtr;
using Clock = std::chrono::steady_clock;

// What a read packet does to running counters (probed on the GPU at init by aql_pmc.cc):
// kCumulative: they keep counting (deltas of successive reads); kResets: each read returns the
// counts since the previous read; kStops: counting stops at a read (re-started after it).
// kReadUnknown: no continuous counting (duty-cycled windows, published from outside).
enum ReadMode { kReadUnknown, kCumulative, kResets, kStops };
const char* read_mode_name(ReadMode m);

// One read's output, reduced per counter (chip totals, plus per-XCC MFMA / GRBM_COUNT).
struct Sample {
  double v[kNumCtr] = {};
  int inst[kNumCtr] = {};
  uint64_t samples = 0;
  double xm[kMaxXcc] = {};  // SQ_VALU_MFMA_BUSY_CYCLES per XCC
  double xg[kMaxXcc] = {};  // GRBM_COUNT per XCC
  int nxcc = 0;             // 0: XCC coordinates unavailable
};

// One GPU's counter read path.  Queue 0 is the GPU's first queue (shared with the sentinel);
// queue 1 is the rescue queue, which exists between open_rescue and close_rescue and only ever
// carries reads.  Each queue has one completion signal, armed by every post_* that names it.
// The machine calls a port only under its round lock, so never from two threads at once.
class ReadPort {
 public:
  virtual ~ReadPort() = default;
  virtual void post_read(int q) = 0;                // a read, no barrier (runs past a stalled dispatch)
  virtual void post_arm(bool baseline_read) = 0;    // queue 0: start program, then (baseline) a read
  virtual void post_start() = 0;                    // queue 0: start program, no completion (kStops)
  virtual void post_stop(int q) = 0;                // stop program (shutdown)
  virtual bool done(int q) = 0;                     // q's signal has completed
  virtual bool failed() = 0;                        // a queue error: the GPU is unusable
  virtual bool collect(int q, Sample* out) = 0;     // the output of q's last completed read
  virtual bool open_rescue() = 0;
  virtual void close_rescue() = 0;
  virtual std::string label() const = 0;            // for log lines (the BDF)
  // A packet timed out or the queue failed: the GPU may still own the port's buffers.  Read by
  // the sentinel and the calibration paths of aql_pmc.cc as well.
  std::atomic<bool> broken{false};
};

struct MachineConfig {
  ReadMode mode = kCumulative;
  int interval_ms = 1000;       // fallback: a round every interval when nothing kicks
  bool inline_rounds = false;   // the kicker runs the rounds (gpuexp_rp_set_inline)
  bool rescue = true;           // GPUEXP_PMC_READ_RESCUE
  int rescue_rounds = 3;
  int probation_rounds = 5;
  int arm_timeout_ms = 1000;    // arm_sync
  int first_slice_us = 60, slice_us = 100;  // polling slices while waiting for reads
  gpuexp_ctr::RearmConfig rearm;
  bool log = true;              // one stderr line per rescue / release / re-arm
};

// Read health of one GPU (gpuexp::CounterHealth order + extras).
struct Health {
  uint64_t stalls = 0, resets = 0, rearms = 0, rescues = 0, releases = 0;
  bool rescue_active = false;
  bool waiting_rearm = false;
  uint64_t conflicts = 0;
  bool broken = false;
};

class RoundMachine {
 public:
  explicit RoundMachine(const MachineConfig& c);
  ~RoundMachine();
  RoundMachine(const RoundMachine&) = delete;
  RoundMachine& operator=(const RoundMachine&) = delete;

  // Set-up (before start): one slot per engine device; port nullptr = no counters there.
  // `model` carries the GPU's SIMD / CU counts and privilege for the derivations.
  void add(ReadPort* port, const gpuexp_ctr::Derived& model);
  // Init only, before start: start counting (+ baseline read), waiting up to arm_timeout_ms.
  bool arm_sync(int dev);
  int size() const { return int(slots_.size()); }
  bool usable(int dev) const;

  // Continuous mode: starts / joins the counting thread.  stop() also stops counting on every
  // GPU that has no read in flight (bounded wait) and releases rescue queues that are idle.
  void start();
  void stop();

  // Engine side, once per tick.  Inline: kick posts the round from the caller and sync collects
  // it (up to timeout_us; 1 = reads left over for the counting thread).  Thread mode: kick wakes
  // the thread, sync waits for its round.  0 = done.
  void kick();
  int sync(int timeout_us);

  // Readers, any thread.
  int sample(int dev, double* out);               // kNumOut doubles; -1 when no current window
  int sample_xcc(int dev, double* out, int max);  // per-XCC MFMA busy; returns n
  int scope(int dev);
  bool health(int dev, Health* out) const;
  std::string debug(int dev);                     // "key=value;..." (gpuexp_rp_debug)
  uint64_t windows(int dev) const;                // windows published so far
  uint64_t thread_cpu_ns() const { return thread_cpu_ns_.load(); }
  uint64_t rounds() const { return rounds_.load(); }

  // Duty-cycled windows (mode kReadUnknown): the caller publishes each window itself.
  void publish_window(int dev, const double* d, const Sample& s, double wall_s);

 private:
  struct Slot;
  struct Round {
    uint64_t gen = 0;            // bumped by every post_round: a newer round takes the old one over
    std::vector<int> waiting;    // devices whose read of this round is not collected yet
  };

  void post_round_locked(Clock::time_point now);
  // Looks at the round `gen` until it is collected, `deadline` passes, or `stop` says so.
  // final: reads still pending at the deadline count as stalls.  Returns true when none is left.
  bool work(uint64_t gen, Clock::time_point deadline, bool final, const std::atomic<uint64_t>* stop_seq,
            uint64_t seen_seq);
  void look_locked(Clock::time_point now, bool at_deadline, bool final);
  void round_done(Slot& s, int dev, Clock::time_point now);
  void round_stuck(Slot& s, int dev, Clock::time_point now);
  void publish(Slot& s, const double* d, const Sample& smp, double wall, Clock::time_point end, const double* cum,
               const double* xm, const double* xg);
  void loop();
  int64_t ns(Clock::time_point t) const;

  MachineConfig cfg_;
  std::vector<std::unique_ptr<Slot>> slots_;
  Clock::time_point epoch_;

  std::mutex round_mu_;  // the round, every slot's read state, every port call
  Round round_;
  bool live_ = false;    // under round_mu_: started and not stopping

  std::thread thread_;
  std::mutex cv_mu_;
  std::condition_variable cv_, done_cv_;
  bool quit_ = false;                     // cv_mu_
  uint64_t kick_seq_ = 0, done_seq_ = 0;  // cv_mu_ (thread mode)
  std::atomic<uint64_t> kick_seq_a_{0};   // kick_seq_ for the round's early-exit check
  bool leftover_ = false;                 // cv_mu_: sync handed the reads of round leftover_gen_
  uint64_t leftover_gen_ = 0;             // to the thread
  std::atomic<int64_t> last_kick_ns_{0};

  std::atomic<uint64_t> thread_cpu_ns_{0}, rounds_{0};
  std::atomic<uint64_t> cpu_post_{0}, cpu_wait_{0}, cpu_collect_{0};
};

}  // namespace gpuexp_pmc
