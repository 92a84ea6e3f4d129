// The telemetry engine: sampler thread + series table + snapshot store + HTTP server.
//
// Reference control loop: `for { list pods; kubectl exec ps; NVML loop; Sleep(30s) }`
// (/root/reference/main.go:74-157), period = 30 s + scan time, crash on any error.
// Here a timerfd drives a fixed-rate tick (1/10/100 Hz) whose stages never block on the
// network, and each source fails in isolation (SURVEY.md §5 failure-detection row).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <initializer_list>
#include <iterator>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "gpuexp/backends.h"
#include "gpuexp/device.h"
#include "gpuexp/exposition.h"
#include "gpuexp/engine_families.h"
#include "gpuexp/http.h"
#include "gpuexp/kfd_events.h"
#include "gpuexp/procs.h"
#include "gpuexp/ras.h"
#include "gpuexp/snapshot.h"
#include "gpuexp/sources.h"

namespace gpuexp {

// Fork-join pool for per-GPU reads: each MI355X gpu_metrics read is an SMU table transfer
// (~0.35-0.42 ms of driver time per GPU per tick, measured), independent per GPU, so an
// 8-GPU tick costs one transfer of latency instead of eight.
class ForkJoinPool {
 public:
  explicit ForkJoinPool(int threads);
  ~ForkJoinPool();
  // Runs fn(i) for i in [0, n) on the pool + the caller; returns when all are done.
  void run(int n, const std::function<void(int)>& fn);
  int threads() const { return int(workers_.size()) + 1; }
  // Cumulative thread CPU of the workers (each publishes its own clock after every run(),
  // before run() returns; so it includes their wake-up and lock costs, not only the items).
  uint64_t cpu_ns_total() const;

 private:
  void worker(size_t idx);
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0;
  std::atomic<int> next_{0};
  std::unique_ptr<std::atomic<uint64_t>[]> wcpu_;
  int pending_ = 0;
  uint64_t epoch_ = 0;
  bool quit_ = false;
};

// Thread CPU (ns) the host charges for one timer wake-up of the sampler's own wait (timerfd +
// poll, no work in between), and the mean lateness of the wake-ups: n periods of period_ns.  A
// host property, not the exporter's: tests/test_fakehost.py charges an MI355X host's figure.
void timer_wakeup_cost(uint64_t period_ns, int n, uint64_t* cpu_ns, uint64_t* late_ns);

// counters_cpu_budget's policy (engine.cc): one finished read round of `round_cpu_ns` moves the
// per-round CPU EWMA and sets the rounds' minimum interval (0 = counters_min_interval); a late
// round leaves both as they are.
void counters_round_policy(double round_cpu_ns, bool late, double budget, double base_ns, double period_ns,
                           double* ewma_ns, double* iv_ns);

struct EngineConfig {
  std::string backend = "mock";        // mock | sysfs | amdsmi
  int device_threads = 0;              // 0 = auto (serial), N > 1 = a pool of N reader threads
  int mock_devices = 1;
  std::string mock_xgmi_file;          // mock only: per-peer traffic matrix (MockBackend::set_traffic_file)
  std::string host_root;               // "" == "/"
  double interval_s = 1.0;             // 0 = manual ticks only (tests)
  // false: no sampler thread although interval_s > 0 -- the caller ticks (tick_now) on its own
  // clock, with every interval-derived policy as the sampler would have it (tools/tickbench.py)
  bool sampler_thread = true;
  // With an HTTP server: render and publish a tick's snapshot only when a scrape will read it
  // (HttpServer::render_due: only steady scrapers known and none due before the tick after next
  // = skip), and at least once a second.  Prometheus at 15 s against a 10 Hz sampler: ~1.1
  // renders a second instead of 10.  A scraper at the tick rate (the bench) reads every tick.
  bool render_when_due = true;
  int render_every_ticks = 0;  // tests only: > 0 renders (and writes the table) on every N-th tick only
  bool serve_http = true;
  HttpConfig http;
  std::string series_profile = "standard";  // standard | full | compact | legacy
  double ras_interval_s = 10.0;        // full profile: RAS/AER sysfs re-read period
  bool metrics_coalesce = true;        // skip gpu_metrics SMU fetches between PMFW refreshes
  // At most one SMU fetch per GPU per this many seconds (0 = no cap).  < 0 = auto: the cap
  // follows the measured CPU of a fresh fetch so that all GPUs' fetches together stay within
  // metrics_cpu_budget of one core (between fetches the cached table is re-decoded; the
  // per-tick activity signals come from the PMC counters, read every tick).
  double metrics_min_interval_s = -1;
  // auto: fraction of one core for SMU fetches (all GPUs).  0.75 %: 8 GPUs under load (~380 us of
  // kernel busy-wait per fetch) fetch every 5th tick at 10 Hz, one GPU every tick
  // (profiles/r06/cpu_projection.txt)
  double metrics_cpu_budget = 0.0075;
  double metrics_max_interval_s = 1.0;  // auto: never staler than this
  uint64_t fake_metrics_cost_us = 0;   // tests only: thread CPU burnt per fresh gpu_metrics read
  // tests / tools/project_cpu.py only (fake_sources.cc): >= 0 runs the real PMC read machine on
  // scripted fake GPUs (counters) or a fake sentinel, burning this much CPU per GPU per read / run
  int fake_pmc_cost_us = -1;
  // tests only: every fake GPU's PMC queue stands still over these [a, b) windows (us since start)
  std::vector<std::pair<int64_t, int64_t>> fake_pmc_stalls_us;
  int fake_sentinel_cost_us = -1;
  bool legacy_families = true;         // pod_gpu_memory_usage / docker_gpu_memory_perc_usage
  bool pod_attribution = true;
  bool infer_device_owner = true;      // single-pod GPU -> device series carry the pod
  std::string process_source = "auto";  // auto | kfd | amdsmi | none
  bool kfd_cu_occupancy = true;
  // KFD's per-process sdma_<gpu_id>: off by default, it is not SDMA time on MI355X
  // (profiles/r04/sdma_units.txt: one jump of 1.24e12 at the first copy, then flat)
  bool kfd_sdma = false;
  double kfd_detail_interval_s = 1.0;  // cu_occupancy / sdma re-read period (0 = every tick)
  // KFD proc directory listed at least this often (and on its mtime moving, or a tracked
  // process vanishing); tracked processes' VRAM is read every tick either way (0 = list every tick)
  double kfd_rescan_interval_s = 0.5;
  // The per-process reads (KFD VRAM per process and GPU, or amdsmi's process list) run at most
  // this often; a tick in between exports the last lists again (0 = every tick).  Per-process
  // VRAM does not need a 100 Hz tick, and at 8 GPUs x 4 processes these reads were the
  // sampler's largest stage after the SMU fetch (tools/tickbench.py).  At <= 20 Hz: every tick.
  double process_min_interval_s = 0.05;
  bool exclude_self = true;
  bool enable_sentinel = false;
  std::string sentinel_impl = "auto";  // auto (PMC queue if the aqlprofile counters run, else HIP) | hip | queue
  int sentinel_ring = 64;
  int sentinel_spin = 500;  // ~15 us window (rocprofv3: spin 2000 ran 61 us/launch)
  // The sentinel runs at most this often (its SCLK / dispatch / memory-latency probes do not need
  // a 100 Hz tick; each run is a dispatch + ring drain per GPU on the sampler).  Manual-tick
  // engines (interval_s = 0) run it every tick.
  double sentinel_min_interval_s = 0.5;
  bool enable_counters = false;
  std::string counters_plugin;         // path to _gpuexp_aqlpmc.so / _gpuexp_rocprof.so
  // continuous: counting never pauses and is read once per tick (aqlprofile plugin);
  // duty: a counters_window_ms window every counters_interval_ms (either plugin)
  std::string counters_mode = "continuous";
  int counters_window_ms = 20;         // duty: counting window...
  int counters_interval_ms = 1000;     // ...once per interval (see rocprof_plugin.cc)
  int counters_sync_us = 2000;         // continuous: longest a tick waits for its own counter read
  // continuous: a PMC read round at most this often (0 = every tick).  Each round costs host CPU
  // per GPU (packet + output reduction); above 20 Hz a tick exports the last window again.
  double counters_min_interval_s = 0.05;
  // continuous + periodic ticks: the read rounds together may use this share of one core (0 = no
  // cap).  A round's CPU grows with the logical GPUs (a CPX node has 64 PMC reads per round); when
  // the measured round CPU / this share exceeds counters_min_interval_s, rounds come that much less
  // often, at most half as often, and a stretched round may go one tick later to stay off a tick
  // with two SMU fetches (a window never gets older than the plugin's two fallback intervals).
  double counters_cpu_budget = 0.0075;
  // continuous: when a tick's PMC read goes out.  "start": before the device reads;
  // "after_devices": once the gpu_metrics SMU fetches are done (a PM4 read in flight while
  // the SMU serves the metrics table slows the fetch, profiles/r04/devices_split.txt).
  // continuous: when a tick's PMC read goes out -- "start" of the tick, "after_devices", "end"
  // of the previous tick, or "auto" (end below 50 ms ticks, else start)
  std::string counters_kick = "auto";
  bool counters_inline = true;  // continuous + periodic ticks: the sampler runs the read rounds
  bool enable_rccl = false;
  std::string rccl_dir = "/dev/shm";
  bool rccl_verify = true;             // attribute a tracer file only to a process that maps it
  double rccl_scan_interval_s = 1.0;   // list the tracer directory at most this often (when it changed)
  bool enable_kfd_events = true;       // full profile: KFD SMI events (VM faults, resets, ...)
  bool firmware_info = true;           // full profile: amd_gpu_firmware_info (one series per loaded firmware)
  // Checkpoint of the exporter's own accumulations (per-pod energy, KFD event counts) so
  // they continue across exporter restarts; "" = off.  Written every state_interval_s and
  // at stop (write + rename), read at start.
  std::string state_file;
  double state_interval_s = 10.0;
  // Per-pod totals of a pod that no applied pod list has had for this long are dropped even
  // while the lists are partial (a metadata source keeps failing); complete lists drop at once.
  double pod_totals_ttl_s = 3600.0;
  std::string kfd_path = "/dev/kfd";   // the device node itself (not under host_root)
  bool force_amdsmi_metrics = false;
  int gzip_level = 1;
  // "compiled": fixed-layout body patched in place, gzip from pre-encoded static bits
  // (SeriesTable::render_compiled); "classic": re-render changed families, compress the body.
  std::string exposition = "compiled";
  uint64_t gc_after = 1;               // stale series vanish this many ticks after last seen
  std::vector<int> device_filter;      // empty = all
  std::vector<std::string> device_filter_bdf;  // also accepted: PCI BDFs ("0000:75:00.0")
  // GPUs that get the exporter's own GPU queue (sentinel + PMC counters), by index or BDF;
  // both empty = every exported GPU.  ~346 MiB of pinned host memory per queue on MI355X.
  std::vector<int> queue_devices;
  std::vector<std::string> queue_devices_bdf;
  std::string trace_path;              // Chrome trace JSON of sampler stages
  size_t trace_max_events = 200000;
  std::string version = "0.1.0";
};

struct PodMeta {
  std::string uid;
  std::string ns;
  std::string name;
  std::vector<std::pair<std::string, std::string>> containers;  // (container_id, name)
};

struct DeviceOwner {
  std::string ns, pod, container;
};

struct EngineStats {
  uint64_t ticks = 0;
  uint64_t overruns = 0;
  uint64_t publish_skipped = 0;
  uint64_t last_tick_ns = 0;
  uint64_t max_tick_ns = 0;   // since start or the last reset_tick_max()
  uint64_t tick_ns_total = 0;  // wall time of every tick so far (mean = tick_ns_total / ticks)
  // the sampler thread's own CPU per tick: the work a tick carries, whatever preempts it
  uint64_t max_tick_cpu_ns = 0;   // since start or the last reset_tick_max()
  uint64_t tick_cpu_ns_total = 0;
  uint64_t render_bytes = 0;
  uint64_t series = 0;
  uint64_t device_errors = 0;
  double stage_ns[8] = {};
  uint64_t stage_cpu_ns[8] = {};  // cumulative sampler-thread CPU per stage (pool / PMC threads not split)
  uint64_t sampler_cpu_ns = 0;
  uint64_t gzip_eager = 0;  // snapshots published with a gzip copy
  uint64_t relayouts = 0;   // compiled exposition: families laid out again (0 per tick in steady state)
  uint64_t code_builds = 0; // compiled exposition: Huffman code builds
  uint64_t families_skipped = 0;  // compiled exposition: families passed over unchanged (cumulative)
  uint64_t families_rendered = 0; // ... and families walked (cumulative)
  // tick leveling (engine.cc): fresh gpu_metrics reads, sentinel runs and KFD listings so far,
  // and ticks that deferred one of the last two because they carried >= 2 SMU fetches
  uint64_t fresh_reads = 0, sentinel_runs = 0, kfd_lists = 0, leveled_ticks = 0;
  uint64_t last_tick_fresh = 0;  // SMU fetches the last tick carried
  uint64_t renders_skipped = 0;  // ticks that published nothing: no scrape due (render_when_due)
  // continuous counters: read rounds so far, their CPU (EWMA per round, the sampler's kick + sync
  // and the plugin thread's), and the current minimum round interval (counters_min_interval_s, or
  // longer under counters_cpu_budget)
  uint64_t counter_rounds = 0;
  double counters_round_cpu_ns = 0, counters_round_interval_s = 0;
};

class Engine {
 public:
  explicit Engine(const EngineConfig& cfg);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  bool start(std::string* err);
  void stop();
  // One tick with an injected monotonic time (manual mode / tests).
  void tick_now(uint64_t now_ns);

  SnapshotStore::Pin snapshot() { return store_.acquire(); }
  std::string snapshot_text();
  int http_port() const { return http_ ? http_->port() : -1; }
  const std::vector<DeviceInfo>& devices() const { return devices_; }
  MockBackend* mock() { return mock_; }
  EngineStats stats();
  void reset_tick_max() {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.max_tick_ns = 0;
    stats_.max_tick_cpu_ns = 0;
  }
  const HttpStats* http_stats() const { return http_ ? &http_->stats() : nullptr; }
  // Runtime pre-wake switch of the HTTP workers (PrewakeMode); false without an HTTP server.
  bool set_prewake_mode(int mode) {
    if (!http_ || mode < kPrewakeOff || mode > kPrewakeSpin) return false;
    http_->set_prewake_mode(mode);
    return true;
  }
  int prewake_mode() const { return http_ ? http_->prewake_mode() : cfg_.http.prewake_mode; }
  std::string source_status();

  // Control-plane inputs (any thread; applied at the next tick).
  // complete: every metadata source answered (a partial list never GCs per-pod totals).
  void set_pods(std::vector<PodMeta> pods, bool complete = true);
  void set_device_owners(std::vector<std::pair<std::string, DeviceOwner>> owners);
  void set_pid_cgroup(int pid, const std::string& cgroup_path);
  void clear_pid_cgroups();
  // Test hook: bytes as if read from device `dev`'s KFD SMI event fd (applied next tick).
  void inject_kfd_events(int dev, const std::string& bytes);

  static const char* stage_name(int i);
  static constexpr int kStages = 8;
  static constexpr uint64_t kStageCpuEvery = 4;  // ticks per sampled per-stage CPU split
  // The devices stage split (gpuexp_device_read_seconds_total{part}): PMC read kick,
  // control-plane apply, gpu_metrics (SMU fetch or cached decode), VRAM-used file, RAS/AER
  // files, GTT file.  Per-GPU parts are summed over GPUs (wall time on whichever thread).
  static const char* dev_part_name(int i);
  static constexpr int kDevParts = 6;

 private:
  struct DevState {
    DeviceSample cur, prev;
    bool have_prev = false;
    // single-pod owner inference, kept while the GPU's processes (by KFD identity) and the
    // control plane stay the same (0: recompute)
    uint64_t owner_sig = 0;
    DeviceOwner owner_inferred;
    double xgmi_rd_rate[kMaxXgmiLinks] = {};
    double xgmi_wr_rate[kMaxXgmiLinks] = {};
    bool rates_valid = false;
    // Last residency-derived values: the PMFW accumulates them at its own rate (slower
    // than a 100 Hz tick), so a tick without a new accumulation re-exports these instead
    // of dropping the series.
    double vram_last = kNaN, gtt_last = kNaN;  // the last VRAM / GTT used read (process_min_interval_s)
    double thr_last[5] = {kNaN, kNaN, kNaN, kNaN, kNaN};
    double xcc_last[kMaxXcc] = {kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN, kNaN};
    double mfma_last = kNaN;  // this tick's amd_gpu_mfma_busy_percent (NaN: no counter window)
    double flops_last[2] = {kNaN, kNaN};  // this tick's bf16 / fp8 MFMA FLOP/s (NaN: not device-wide)
    DeviceOwner owner;
    DeviceOwner owner_built;  // ns/pod/container the refs were built for
    bool owner_built_set = false;
    // cached series handles of every per-GPU family (RefScope::kGpu), addressed by dref();
    // rebuilt on an owner change (new pod labels) or GC
    std::vector<SeriesRef> refs;
    std::vector<SeriesRef> fw;  // amd_gpu_firmware_info, one per component
    uint64_t kfd_events[kKfdEventIds] = {};  // KFD SMI events seen on this GPU, by id
    uint64_t errors = 0;
    uint64_t ras_ns = 0, gtt_ns = 0;  // this tick's RAS / GTT read time (sample_devices)
    double fetch_cost_ns = 0;        // EWMA thread CPU of a fresh gpu_metrics read (0 = none yet)
    double fetch_cpu_s = 0;          // thread CPU of every fresh gpu_metrics read so far
    uint64_t fetch_cap_ns = 0;       // cap currently set on the backend's reader
    uint64_t metrics_fresh_ns = 0;   // tick time of the last fresh gpu_metrics read (0 = none yet)
  };
  // Cached series handles of a (GPU, PID) (and of a PID's legacy series) or a pod, valid while
  // their label values are the ones recorded here: the per-tick path then sets values without
  // building label vectors.  Indexed by family: pref()/podref().
  struct ProcRefs {
    std::string comm, ns, pod, container;
    SeriesRef ref[kFamProcEnd - kFamProcVram];
    uint64_t gen = 0;
  };
  struct PodRefs {
    SeriesRef ref[kFamPodEnd - kFamPodVram + 1];  // (+1: the fp8 series of amd_pod_gpu_mfma_flops)
    uint64_t gen = 0;
  };
  static SeriesRef& pref(ProcRefs& r, Fam f) { return r.ref[f - kFamProcVram]; }
  static SeriesRef& podref(PodRefs& r, Fam f, int k = 0) {
    return r.ref[f == kFamPodFlops && k ? kFamPodEnd - kFamPodVram : f - kFamPodVram];
  }
  // A GPU's gfx activity split over its processes by their share of the occupied CUs.  KFD
  // compute contexts report no per-process engine time (fdinfo drm-engine-* stays empty,
  // profiles/r01/kfd_read_costs.txt); a sole process gets all of it, and with no waves resident
  // at the CU sample the split is even (engine_procs.cc).
  struct CuSplit {
    explicit CuSplit(const std::vector<ProcSample>& procs);
    double frac(const ProcSample& p) const;  // the process's fraction of the GPU (NaN: unknown)
    size_t n = 0;
    bool any = false;  // some process has a CU occupancy
    double sum = 0;    // CUs occupied by all processes
  };
  // A pod's aggregates over one tick (engine_pods.cc)
  struct PodAgg {
    double vram = 0;
    std::set<int> pids;
    int gpus = 0;
    double xrd = 0, xwr = 0, power = 0, gfx = 0, gfx_share = 0;
    double energy_j = 0;          // this tick
    double xrd_b = 0, xwr_b = 0;  // xGMI bytes this tick (owned GPUs whole, shared GPUs by share)
    double mfma = 0, hbm = 0, flops[2] = {0, 0};
    int gfx_n = 0, mfma_n = 0, hbm_n = 0, flops_n = 0;
    double alloc_s = 0, busy_s = 0;  // GPU-seconds this tick
    bool share_known = false;
  };
  struct ProcAttr {
    std::string ns, pod, container, uid;
    // cached across ticks while KFD reads the same process (ProcSample::kfd_id) and no pod
    // list / cgroup override was applied since (ctl_epoch_)
    uint64_t kfd_id = 0, ctl_epoch = 0, seen = 0;
  };
  std::unordered_map<int, ProcAttr> attr_cache_;  // sampler thread
  uint64_t ctl_epoch_ = 1;

  void define_families();
  void register_families(const std::vector<FamilySpec>& specs);
  int counters_interval_ms() const;
  void run_sampler();
  void tick_locked(uint64_t now_ns);
  // engine_device.cc
  uint64_t sample_devices(uint64_t now, bool split_cpu, bool memory_due, uint64_t* part);  // returns failed reads
  void update_fetch_policy(uint64_t now);
  void collect_device(int i, uint64_t gen, double dt_s);
  void collect_counters(int i, uint64_t gen, double dt_s);
  void collect_sentinel(int i, uint64_t gen);
  // engine_procs.cc
  void emit_processes(uint64_t gen, const std::vector<std::vector<ProcSample>>& per_dev);
  // engine_pods.cc
  void infer_owners(const std::vector<std::vector<ProcSample>>& per_dev);
  void emit_pods(uint64_t gen, const std::vector<std::vector<ProcSample>>& per_dev);
  void emit_pod_totals(uint64_t gen);
  // engine_rccl.cc
  void emit_rccl(uint64_t gen);
  void emit_rccl_self(uint64_t gen);
  // engine_kfd_events.cc
  void count_kfd_events();
  void emit_device_kfd_events(int dev, uint64_t gen);
  void emit_kfd_events(uint64_t gen);
  // engine_self.cc
  void emit_self(uint64_t gen);
  void emit_http_self(uint64_t gen, bool publish_hist);
  std::string device_key(size_t i) const;  // "<bdf>/<partition>": stable across restarts
  void load_state();
  bool save_state();
  void trace_event(const char* name, uint64_t start_ns, uint64_t dur_ns);
  // Sets `v` on slot `k` of per-GPU family `f` (labels: the device's, then `extra`).
  void dput(DevState& st, int dev, Fam f, int k, std::initializer_list<const char*> extra, double v, uint64_t gen);
  SeriesRef& dref(DevState& st, Fam f, int k = 0) { return st.refs[size_t(fam_off_[f] + k)]; }
  SeriesRef& gref(Fam f, int k = 0) { return grefs_[size_t(fam_off_[f] + k)]; }
  // Sets `v` on slot `k` of global family `f`; labels() only when the handle is stale.
  template <class F>
  void gput(Fam f, int k, double v, uint64_t gen, F&& labels) {
    cput(gref(f, k), fam_ids_[f], v, gen, std::forward<F>(labels));
  }
  // Sets `v` through the cached handle `r`; builds the label values (labels()) and
  // re-interns only when the handle is stale.
  template <class F>
  void cput(SeriesRef& r, int fid, double v, uint64_t gen, F&& labels) {
    if (!emit_) return;
    if (table_.set(r, v, gen)) return;
    r = table_.upsert(fid, labels());
    table_.set(r, v, gen);
  }

  EngineConfig cfg_;
  std::unique_ptr<Backend> backend_;
  MockBackend* mock_ = nullptr;
  bool compiled_ = true;  // cfg_.exposition == "compiled" (set at start)
  std::vector<DeviceInfo> devices_;
  std::vector<DevState> dstate_;
  std::vector<std::vector<std::string>> owner_keys_;  // per device: device_owner_keys()
  std::unique_ptr<KfdProcReader> kfd_;
  std::unique_ptr<PidResolver> resolver_;
  std::unique_ptr<SentinelSource> sentinel_;
  std::unique_ptr<CounterSource> counters_;
  std::unique_ptr<RcclSource> rccl_;
  std::unique_ptr<KfdEventSource> kfd_events_;
  std::string kfd_events_status_ = "disabled";
  std::vector<std::pair<int, std::string>> pending_kfd_bytes_;  // test injection (ctl_mu_)
  // per-process KFD events attributed to pods: (namespace, pod, event id) -> count
  std::map<std::tuple<std::string, std::string, int>, uint64_t> pod_kfd_events_;
  uint64_t kfd_events_unattributed_ = 0;  // per-process events whose PID resolved to no pod
  bool pending_complete_ = false;  // ctl_mu_: the pending pod list came from a complete refresh
  bool pods_complete_ = false;     // sampler: the applied pod list is complete (per-pod GC allowed)
  uint64_t state_saved_ns_ = 0;
  // read by source_status() from any thread while save_state() may rewrite it on the
  // sampler thread: only through these, under status_mu_
  std::string state_status_ = "disabled";
  mutable std::mutex status_mu_;
  void set_state_status(std::string s) {
    std::lock_guard<std::mutex> lk(status_mu_);
    state_status_ = std::move(s);
  }
  std::string state_status() const {
    std::lock_guard<std::mutex> lk(status_mu_);
    return state_status_;
  }
  std::unique_ptr<ForkJoinPool> pool_;
  // full profile, real backends: RAS/AER readers + last totals (re-read every ras_interval_s)
  std::vector<RasReader> ras_;
  std::vector<RasTotals> ras_cache_;
  std::vector<uint64_t> ras_next_ns_;
  std::vector<CachedFile> gtt_used_f_;  // full profile, real backends: mem_info_gtt_used per device
  std::vector<double> gtt_total_;
  std::vector<uint64_t> metrics_fresh_, metrics_coalesced_;  // per device
  uint64_t gzip_eager_ = 0;  // sampler thread only; copied into stats_ per tick
  uint64_t counters_late_ = 0;
  uint64_t start_mono_ns_ = 0, startup_ns_ = 0;  // start() entry; start() -> first tick
  // thread clocks already charged to gpuexp_sampler_cpu_seconds_total (sampler thread only)
  uint64_t counters_cpu_seen_ = 0, pool_cpu_seen_ = 0, sampler_cpu_seen_ = 0;  // ticks whose counter read missed counters_sync_us (sampler thread)
  std::string counters_kick_mode_ = "start";
  uint64_t sentinel_last_ns_ = 0;  // tick time of the last sentinel run (sentinel_min_interval_s)
  uint64_t sentinel_runs_ = 0;  // ticks that ran the sentinel
  uint64_t last_render_mono_ = 0, renders_skipped_ = 0;  // render_when_due
  // This tick writes the series table (render_when_due: only a tick that renders does; every
  // computation of the series stage -- rates, per-pod integration, event totals, histograms --
  // runs on every tick, only the table writes are skipped).  The write sites: dput / cput /
  // gput and the few direct table_ calls (engine_device / engine_pods / engine_kfd_events /
  // engine_self).
  bool emit_ = true;
  uint64_t tick_index_ = 0;  // ticks so far (render_every_ticks)
  int fetch_groups_ = 0;     // GPUs fetching gpu_metrics on their own (a partitioned socket counts once)
  // PMC round leveling: the auto fetch policy's ticks per fetch (0: every tick), and each recent
  // tick's fresh SMU fetches by tick_index_ (the fetch pattern repeats every fetch_ticks_ ticks)
  int fetch_ticks_ = 0;
  static constexpr int kFreshHist = 32;
  uint8_t fresh_hist_[kFreshHist] = {};
  uint8_t load_hist_[kFreshHist] = {};  // ... and its load: fetches, + 2 for a stretched PMC round
  bool counters_deferred_ = false;  // the due round was put off by one tick (leveling)
  bool leveled_ = false;        // this tick deferred the sentinel or a KFD listing (tick leveling)
  uint64_t procs_read_ns_ = 0;  // tick time of the last per-process read (process_min_interval_s)
  uint64_t counters_kick_ns_ = 0;  // tick time the last PMC read round was for (counters_min_interval_s)
  bool counters_round_next_ = false;  // "end" kick: the next tick has a round to sync
  // counters_cpu_budget: CPU of the round in flight so far, EWMA per round, current interval
  uint64_t counters_round_acc_ns_ = 0, counter_rounds_ = 0, counters_round_plugin_seen_ = 0;
  double counters_round_cpu_ns_ = 0, counters_round_iv_ns_ = 0;
  void counters_round_done(bool late);
  double counters_round_interval_s() const;  // cfg_.counters_kick with "auto" resolved
  std::string sentinel_status_ = "disabled", counters_status_ = "disabled";

  SeriesTable table_;
  SnapshotStore store_;
  std::unique_ptr<HttpServer> http_;
  std::string render_buf_;

  std::mutex tick_mu_;
  std::thread sampler_;
  std::atomic<bool> running_{false};
  int stop_fd_ = -1;
  uint64_t gen_ = 0;
  uint64_t last_tick_now_ = 0;
  int self_pid_ = 0;

  // control plane (guarded by ctl_mu_)
  std::mutex ctl_mu_;
  bool ctl_dirty_ = false;
  std::vector<PodMeta> pending_pods_;
  std::vector<std::pair<std::string, DeviceOwner>> pending_owners_;
  std::vector<std::pair<int, std::string>> pending_overrides_;
  bool clear_overrides_ = false;
  // applied (sampler thread only)
  std::unordered_map<std::string, PodMeta> pods_by_uid_;
  std::unordered_map<std::string, std::string> container_names_;  // cid -> name
  std::unordered_map<std::string, DeviceOwner> owners_;           // lower(device id) -> owner
  std::set<std::string> unresolved_;                               // pod UIDs without metadata (last tick)
  std::vector<std::vector<ProcSample>> per_dev_;  // tick scratch: processes per device
  std::vector<int> live_scratch_;                 // tick scratch: PIDs seen this tick
  struct RcclRefs {  // an RCCL (PID, op)'s series handles and the label values they were made for
    std::string ns, pod;
    int rank = -2, nranks = -2;
    SeriesRef calls, bytes, comm;
    uint64_t gen = 0;
  };
  std::map<std::pair<int, std::string>, RcclRefs> rccl_refs_;
  std::unordered_map<uint64_t, ProcRefs> proc_refs_;               // (device << 32 | pid) -> handles
  std::unordered_map<uint64_t, ProcRefs> legacy_refs_;             // pid -> legacy handles (pod, vram, gfx=perc)
  std::map<std::pair<std::string, std::string>, PodRefs> pod_refs_;  // (ns, pod) -> handles
  std::map<std::pair<std::string, std::string>, double> pod_energy_j_;  // (ns, pod) -> joules so far
  // (ns, pod) -> xGMI bytes (read, write) so far
  std::map<std::pair<std::string, std::string>, std::pair<double, double>> pod_xgmi_;
  // (ns, pod) -> (GPU-seconds allocated, GPU-seconds busy) so far (state file: pod_gpu_seconds)
  std::map<std::pair<std::string, std::string>, std::pair<double, double>> pod_gpu_s_;
  // (ns, pod) -> last time an applied pod list had it (GC of per-pod totals under partial lists)
  std::map<std::pair<std::string, std::string>, uint64_t> pod_last_known_ns_;
  // The self-observability histograms (per-stage tick time, scrape latency) accumulate every
  // tick here; the per-stage one is published into the table at most once a second (every tick
  // at <= 1 Hz), the scrape-latency one (which changes only with scrapes) every tick at <= 10 Hz:
  // a histogram's cumulative buckets nearly all change with each observation, so re-rendering
  // and re-splicing their ~120 bucket lines was most of a tick's exposition work -- at 100 Hz
  // (round 5) and at 10 Hz too (round 6: 95 of the 125 lines a 1-GPU tick changed; mock bench
  // render 152 -> 123 us, sampler 378 -> 336 us per tick on the build VM).
  std::vector<uint64_t> stage_hist_[8];
  double stage_hist_sum_[8] = {};
  uint64_t stage_hist_n_[8] = {};
  uint64_t self_hist_pub_ns_ = 0;
  uint64_t expo_relayouts_ = 0;  // sampler thread
  std::map<std::pair<std::string, std::string>, PodAgg> pod_agg_;  // tick scratch (engine_pods.cc)

  // stats (guarded by stats_mu_)
  std::mutex stats_mu_;
  EngineStats stats_;

  // trace
  FILE* trace_ = nullptr;
  size_t trace_events_ = 0;
  uint64_t trace_t0_ = 0;

  // family ids (table-driven, engine_families.h): SeriesTable id of each Fam (-1: not
  // registered), and the first handle slot of a per-GPU (DevState::refs) or global (grefs_) family
  int fam_ids_[kFamCount];
  int fam_off_[kFamCount];
  int gpu_slots_ = 0;
  std::vector<SeriesRef> grefs_;
  std::string driver_version_, kernel_release_;
  uint64_t last_stage_ns_[kStages] = {};
  double dev_part_total_s_[kDevParts] = {};  // sampler thread
};

}  // namespace gpuexp
