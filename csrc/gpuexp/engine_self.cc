// Exporter self-observability (gpuexp_*): ticks, per-stage tick time, sampler CPU, the
// devices-stage split, gpu_metrics freshness and fetch policy, HTTP / pre-wake / gzip counts,
// the compiled exposition's events, optional-source health.  Own prefix, so the reference's
// families stay as clean as its custom registry keeps them (/root/reference/main.go:40-42).
#include <algorithm>
#include <ctime>

#include "gpuexp/engine.h"

namespace gpuexp {

namespace {
constexpr auto G = MetricType::kGauge;
constexpr auto C = MetricType::kCounter;
constexpr auto H = MetricType::kHistogram;
constexpr auto N = LabelBase::kNone;
constexpr auto kGpu = RefScope::kGpu;
constexpr auto kGlobal = RefScope::kGlobal;

const std::vector<double>& stage_bounds() {
  // 9 bounds: the per-stage histograms are re-rendered and re-compressed every tick (at 14
  // bounds they were a third of a 1-GPU exposition), so keep them coarse.
  static const std::vector<double> b = {5e-6, 25e-6, 100e-6, 250e-6, 500e-6, 1e-3, 2.5e-3, 10e-3, 100e-3};
  return b;
}

std::vector<std::string> none() { return {}; }
}  // namespace

const std::vector<FamilySpec>& self_family_specs() {
  static const std::vector<FamilySpec> t = {
      {kFamSelfBuild, "gpuexp_build_info", "Exporter build and backend", G, N, {"version", "backend"}, kGlobal, 1},
      {kFamSelfTicks, "gpuexp_ticks_total", "Sampler ticks completed", C, N, {}, kGlobal, 1},
      {kFamSelfPodsComplete, "gpuexp_pod_list_complete",
       "1 if the applied pod list came from a refresh in which every metadata source "
       "answered (per-pod totals of pods missing from it are dropped at once); 0: a source "
       "failed, and totals of missing pods are kept for pod_totals_ttl (1 h)",
       G, N, {}, kGlobal, 1},
      {kFamSelfKfdScans, "gpuexp_kfd_proc_scans_total",
       "KFD process scans by kind: list (the /sys/class/kfd/kfd/proc directory was listed: "
       "its mtime moved, a tracked process left, or kfd_rescan_interval passed) or tracked "
       "(only the known processes' files were read)",
       C, N, {"kind"}, kGlobal, 2},
      {kFamSelfKfdTracked, "gpuexp_kfd_procs_tracked",
       "Processes in the KFD proc directory the exporter tracks (any GPU of the node)", G, N, {}, kGlobal, 1},
      {kFamSelfStartup, "gpuexp_startup_seconds",
       "Engine start to its first sample: backend init (amdsmi + raw-path validation), one "
       "HSA queue per GPU with PMC programs and sentinel, plugin probes",
       G, N, {}, kGlobal, 1},
      {kFamSelfLast, "gpuexp_last_sample_timestamp_seconds",
       "Unix time of the tick that produced this exposition (alert on time() - this: a stuck "
       "sampler keeps serving its last snapshot)",
       G, N, {}, kGlobal, 1},
      {kFamSelfStage, "gpuexp_sample_stage_duration_seconds", "Sampler stage duration", H, N, {"stage"}, kGlobal,
       Engine::kStages},
      // counters, not histograms: 6 parts x 11 bucket lines would be re-rendered and re-gzipped
      // every tick for a split whose means (rate / rate(gpuexp_ticks_total)) are what matters
      {kFamSelfDevPart, "gpuexp_device_read_seconds_total",
       "The devices stage split: time in each part (counters_kick: PMC read submitted; "
       "control: control-plane apply; gpu_metrics: SMU fetch or cached decode; vram; ras; "
       "gtt; these three timed on one tick in four and scaled), summed over GPUs",
       C, N, {"part"}, kGlobal, Engine::kDevParts},
      {kFamSelfFetchCpu, "gpuexp_gpu_metrics_fetch_cpu_seconds_total",
       "Thread CPU of fresh gpu_metrics reads (each one an SMU round trip the kernel "
       "busy-waits on)",
       C, N, {"gpu"}, kGpu, 1},
      {kFamSelfFetchCap, "gpuexp_gpu_metrics_min_interval_seconds",
       "Current cap on fresh gpu_metrics reads per GPU (metrics_min_interval; auto: the "
       "measured fetch CPU x GPUs / metrics_cpu_budget)",
       G, N, {"gpu"}, kGpu, 1},
      {kFamSelfMetricsAge, "gpuexp_gpu_metrics_age_seconds",
       "Age of the GPU's gpu_metrics table at this tick: seconds since it was last fetched "
       "fresh from the SMU (0 on a fresh tick).  The families it feeds (power, temperatures, "
       "clocks, activity, throttle residency, xGMI/PCIe bytes) are this old; under the auto "
       "fetch policy it cycles up to about the min interval",
       G, N, {"gpu"}, kGpu, 1},
      {kFamSelfScrape, "gpuexp_scrape_duration_seconds",
       "Server-side /metrics latency (request parsed -> last byte written)", H, N, {}, kGlobal, 1},
      {kFamSelfScrapes, "gpuexp_scrapes_total", "Scrapes of the metrics path", C, N, {}, kGlobal, 1},
      {kFamSelfHttpBytes, "gpuexp_http_response_bytes_total", "HTTP response bytes written", C, N, {}, kGlobal, 1},
      {kFamSelfPrewake, "gpuexp_http_prewake_wakeups_total",
       "Timer wake-ups of the HTTP worker ahead of expected scrapes (scrape-phase pre-wake)", C, N, {}, kGlobal, 1},
      {kFamSelfPrewakeHits, "gpuexp_http_prewake_hits_total",
       "Scrapes of the metrics path that arrived while their HTTP worker was pre-woken "
       "(its pre-wake timer fired within the lead + one slice before the request)",
       C, N, {}, kGlobal, 1},
      {kFamSelfPrewakeHitsNarrow, "gpuexp_http_prewake_hits_narrow_total",
       "Pre-woken scrapes under round 3's narrower window (timer fired within the "
       "minimum lead + one slice before the request)",
       C, N, {}, kGlobal, 1},
      {kFamSelfPrewakeSpins, "gpuexp_http_prewake_spins_total",
       "Spin pre-wake windows the HTTP worker polled in, by how they ended: a /metrics "
       "request arrived (hit) or the window ran out (timeout)",
       C, N, {"outcome"}, kGlobal, 2},
      {kFamSelfPrewakeSpinS, "gpuexp_http_prewake_spin_seconds_total",
       "Wall time the HTTP worker spent polling in spin pre-wake windows (the CPU the "
       "spin mode costs)",
       C, N, {}, kGlobal, 1},
      {kFamSelfRxMoves, "gpuexp_http_rx_cpu_moves_total",
       "Times an HTTP worker moved to the CPU a steady scraper's requests arrive on "
       "(http follow_rx_cpu; 0 when off)",
       C, N, {}, kGlobal, 1},
      {kFamSelfGzip, "gpuexp_gzip_compressions_total",
       "gzip compressions of the exposition: by the sampler (a gzip scrape was expected before "
       "the next tick) or per request (off schedule)",
       C, N, {"where"}, kGlobal, 2},
      {kFamSelfRenderBytes, "gpuexp_render_bytes", "Size of the last rendered exposition", G, N, {}, kGlobal, 1},
      {kFamSelfExpo, "gpuexp_exposition_events_total",
       "Compiled exposition: families laid out again (a series appeared or went, a value outgrew "
       "its field), segments parsed on their own while their layout settled, Huffman code "
       "builds (0 per tick in steady state), and ticks that rendered nothing because no "
       "steady scraper was due (render_when_due)",
       C, N, {"event"}, kGlobal, 4},
      {kFamSelfSeries, "gpuexp_series", "Series in the last rendered exposition", G, N, {}, kGlobal, 1},
      {kFamSelfDevErrors, "gpuexp_device_errors_total", "Failed telemetry reads per GPU", C, N, {"gpu"}, kGpu, 1},
      {kFamSelfOverruns, "gpuexp_tick_overruns_total", "Ticks skipped because a tick ran past its deadline", C, N, {},
       kGlobal, 1},
      {kFamSelfCpu, "gpuexp_sampler_cpu_seconds_total",
       "CPU time of the sampling work: the sampler thread, its per-GPU read threads and the PMC "
       "counter thread (not the HTTP server)",
       C, N, {}, kGlobal, 1},
      {kFamSelfSourceUp, "gpuexp_source_up", "1 if an optional source is active", G, N, {"source"}, kGlobal, 5},
      {kFamSelfMetricsReads, "gpuexp_gpu_metrics_reads_total",
       "gpu_metrics reads by kind: fresh (SMU table fetch) or coalesced (cached table, "
       "PMFW had not refreshed yet)",
       C, N, {"gpu", "kind"}, kGpu, 2},
      {kFamSelfMetricsPeriod, "gpuexp_gpu_metrics_refresh_period_seconds",
       "PMFW gpu_metrics refresh period learnt from firmware timestamps (0 = learning)", G, N, {"gpu"}, kGpu, 1},
      {kFamSelfUnresolved, "gpuexp_pods_unresolved",
       "Pod UIDs found in GPU processes' cgroups that the control plane has not named "
       "yet (their series carry pod=\"\" and no legacy series until it does)",
       G, N, {}, kGlobal, 1},
      {kFamSelfCtrLate, "gpuexp_counters_late_ticks_total",
       "Ticks that exported the previous counter window because this tick's PMC read had not "
       "completed within counters_sync_us (continuous counters)",
       C, N, {}, kGlobal, 1},
      {kFamSelfCtrInterval, "gpuexp_counters_round_interval_seconds",
       "Current minimum interval between PMC read rounds (continuous counters): "
       "counters_min_interval, or longer when the measured round CPU / counters_cpu_budget is "
       "(many logical GPUs, e.g. a CPX node); between rounds a tick exports the last window",
       G, N, {}, kGlobal, 1},
      {kFamSelfCtrEvents, "gpuexp_counters_events_total",
       "PMC read health per GPU: read_stall (a read still queued at the round's end), "
       "reset (a window dropped: counters went backwards), rearm (counting restarted after "
       "another profiler reset or stopped it), rescue / rescue_release (reads moved to a "
       "queue of their own behind a starved sentinel run, and back)",
       C, N, {"gpu", "event"}, kGpu, 5},
      {kFamSelfCtrRescue, "gpuexp_counters_rescue_active",
       "1 while a GPU's PMC reads run on a rescue queue (+173 MiB pinned while it lasts)", G, N, {"gpu"}, kGpu, 1},
      {kFamSelfCtrScope, "gpuexp_counters_device_scope",
       "1 if wave/LDS/HBM PMC counters see every process on the GPU, 0 if they are "
       "VMID-filtered to the exporter (not exported then)",
       G, N, {"gpu"}, kGpu, 1},
  };
  return t;
}

void Engine::emit_self(uint64_t gen) {
  gput(kFamSelfBuild, 0, 1, gen, [&] { return std::vector<std::string>{cfg_.version, backend_->name()}; });
  EngineStats s;
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    s = stats_;
  }
  gput(kFamSelfTicks, 0, double(s.ticks), gen, none);
  if (startup_ns_) gput(kFamSelfStartup, 0, double(startup_ns_) * 1e-9, gen, none);
  {
    timespec rt;
    clock_gettime(CLOCK_REALTIME, &rt);
    gput(kFamSelfLast, 0, double(rt.tv_sec) + double(rt.tv_nsec) * 1e-9, gen, none);
  }
  gput(kFamSelfOverruns, 0, double(s.overruns), gen, none);
  gput(kFamSelfUnresolved, 0, double(unresolved_.size()), gen, none);
  gput(kFamSelfPodsComplete, 0, pods_complete_ ? 1 : 0, gen, none);
  if (kfd_) {
    gput(kFamSelfKfdScans, 0, double(kfd_->lists()), gen, [] { return std::vector<std::string>{"list"}; });
    gput(kFamSelfKfdScans, 1, double(kfd_->scans() - kfd_->lists()), gen,
         [] { return std::vector<std::string>{"tracked"}; });
    gput(kFamSelfKfdTracked, 0, double(kfd_->tracked()), gen, none);
  }
  gput(kFamSelfRenderBytes, 0, double(s.render_bytes), gen, none);
  gput(kFamSelfSeries, 0, double(s.series), gen, none);
  gput(kFamSelfCpu, 0, double(s.sampler_cpu_ns) * 1e-9, gen, none);
  for (int k = 0; k < kDevParts; ++k)
    gput(kFamSelfDevPart, k, dev_part_total_s_[k], gen, [&] { return std::vector<std::string>{dev_part_name(k)}; });
  // histograms: accumulated every tick, published at most once a second (every tick at <= 1 Hz
  // or manual ticks; see engine.h)
  const uint64_t hnow = last_tick_now_;
  const bool publish_hist = emit_ && (cfg_.interval_s <= 0 || cfg_.interval_s >= 1.0 || !self_hist_pub_ns_ ||
                                      hnow < self_hist_pub_ns_ || hnow - self_hist_pub_ns_ >= 1000000000ull);
  if (publish_hist) self_hist_pub_ns_ = hnow;
  // the scrape-latency histogram changes only with scrapes: every tick at <= 10 Hz, so a
  // scraper reads its own previous scrapes counted (above 10 Hz with the others, once a second)
  const bool publish_http_hist = publish_hist || (emit_ && cfg_.interval_s >= 0.1);
  const std::vector<double>& sb = stage_bounds();
  for (int k = 0; k < kStages; ++k) {
    SeriesRef& r = gref(kFamSelfStage, k);
    if (!r.valid() && emit_) r = table_.upsert(fam_ids_[kFamSelfStage], {stage_name(k)});
    std::vector<uint64_t>& h = stage_hist_[k];
    if (h.size() != sb.size() + 1) h.assign(sb.size() + 1, 0);
    if (s.ticks) {
      const double v = double(last_stage_ns_[k]) * 1e-9;
      h[size_t(std::lower_bound(sb.begin(), sb.end(), v) - sb.begin())] += 1;
      stage_hist_sum_[k] += v;
      stage_hist_n_[k] += 1;
    }
    if (emit_ && (!publish_hist || !table_.set_histogram(r, sb, h, stage_hist_sum_[k], stage_hist_n_[k], gen)))
      table_.touch(r, gen);
  }
  if (http_) emit_http_self(gen, publish_http_hist);
  if (!mock_)
    for (size_t i = 0; i < devices_.size(); ++i) {
      DevState& st = dstate_[i];
      const std::string g = std::to_string(devices_[i].index);
      auto gl = [&] { return std::vector<std::string>{g}; };
      cput(dref(st, kFamSelfMetricsReads, 0), fam_ids_[kFamSelfMetricsReads], double(metrics_fresh_[i]), gen,
           [&] { return std::vector<std::string>{g, "fresh"}; });
      cput(dref(st, kFamSelfMetricsReads, 1), fam_ids_[kFamSelfMetricsReads], double(metrics_coalesced_[i]), gen,
           [&] { return std::vector<std::string>{g, "coalesced"}; });
      cput(dref(st, kFamSelfMetricsPeriod), fam_ids_[kFamSelfMetricsPeriod], backend_->metrics_period_s(devices_[i]),
           gen, gl);
      cput(dref(st, kFamSelfFetchCpu), fam_ids_[kFamSelfFetchCpu], st.fetch_cpu_s, gen, gl);
      const double cap = cfg_.metrics_min_interval_s < 0 ? double(st.fetch_cap_ns) * 1e-9
                                                          : std::max(0.0, cfg_.metrics_min_interval_s);
      cput(dref(st, kFamSelfFetchCap), fam_ids_[kFamSelfFetchCap], cap, gen, gl);
      const double age = st.metrics_fresh_ns && last_tick_now_ >= st.metrics_fresh_ns
                             ? double(last_tick_now_ - st.metrics_fresh_ns) * 1e-9
                             : kNaN;
      cput(dref(st, kFamSelfMetricsAge), fam_ids_[kFamSelfMetricsAge], age, gen, gl);
    }
  gput(kFamSelfSourceUp, 0, 1, gen, [&] { return std::vector<std::string>{"backend:" + std::string(backend_->name())}; });
  gput(kFamSelfSourceUp, 1, (sentinel_ || (cfg_.enable_sentinel && mock_)) ? 1 : 0, gen,
       [] { return std::vector<std::string>{"sentinel"}; });
  gput(kFamSelfSourceUp, 2, (counters_ || (cfg_.enable_counters && mock_)) ? 1 : 0, gen,
       [] { return std::vector<std::string>{"counters"}; });
  gput(kFamSelfSourceUp, 3, rccl_ ? 1 : 0, gen, [] { return std::vector<std::string>{"rccl"}; });
  if (counters_ && cfg_.counters_mode == "continuous") {
    gput(kFamSelfCtrLate, 0, double(counters_late_), gen, none);
    if (cfg_.interval_s > 0) gput(kFamSelfCtrInterval, 0, counters_round_interval_s(), gen, none);
  }
  if (cfg_.enable_kfd_events && cfg_.series_profile == "full")
    gput(kFamSelfSourceUp, 4, kfd_events_ ? 1 : 0, gen, [] { return std::vector<std::string>{"kfd_events"}; });
  if (cfg_.series_profile == "full")
    gput(kFamDriver, 0, 1, gen, [&] { return std::vector<std::string>{driver_version_, kernel_release_}; });
  if (compiled_) {
    gput(kFamSelfExpo, 0, double(expo_relayouts_), gen, [] { return std::vector<std::string>{"relayout"}; });
    gput(kFamSelfExpo, 1, double(table_.provisional_parses()), gen,
         [] { return std::vector<std::string>{"provisional_parse"}; });
    gput(kFamSelfExpo, 2, double(table_.code_builds()), gen, [] { return std::vector<std::string>{"code_build"}; });
    gput(kFamSelfExpo, 3, double(renders_skipped_), gen, [] { return std::vector<std::string>{"render_skipped"}; });
  }
  emit_rccl_self(gen);
}

// The HTTP server's counters: scrape latency histogram, scrapes, bytes, pre-wake, gzip.
void Engine::emit_http_self(uint64_t gen, bool publish_hist) {
  const HttpStats& hs = http_->stats();
  auto ld = [](const std::atomic<uint64_t>& a) { return double(a.load(std::memory_order_relaxed)); };
  SeriesRef& sr = gref(kFamSelfScrape);
  if (emit_ && (publish_hist || !table_.touch(sr, gen))) {
    std::vector<uint64_t> counts(HttpStats::kBuckets + 1);
    for (int b = 0; b <= HttpStats::kBuckets; ++b) counts[size_t(b)] = hs.lat_buckets[b].load(std::memory_order_relaxed);
    const uint64_t cnt = hs.lat_count.load(std::memory_order_relaxed);
    const double sum = double(hs.lat_sum_ns.load(std::memory_order_relaxed)) * 1e-9;
    if (!table_.set_histogram(sr, scrape_latency_bounds(), counts, sum, cnt, gen)) {
      sr = table_.upsert(fam_ids_[kFamSelfScrape], {});
      table_.set_histogram(sr, scrape_latency_bounds(), counts, sum, cnt, gen);
    }
  }
  gput(kFamSelfScrapes, 0, ld(hs.metrics_requests), gen, none);
  gput(kFamSelfHttpBytes, 0, ld(hs.bytes_sent), gen, none);
  // every mode: the mode is switched at run time (set_prewake_mode)
  gput(kFamSelfPrewake, 0, ld(hs.prewake_timer_wakeups), gen, none);
  gput(kFamSelfPrewakeHits, 0, ld(hs.prewake_hits), gen, none);
  gput(kFamSelfPrewakeHitsNarrow, 0, ld(hs.prewake_hits_narrow), gen, none);
  gput(kFamSelfPrewakeSpins, 0, ld(hs.prewake_spin_hits), gen, [] { return std::vector<std::string>{"hit"}; });
  gput(kFamSelfPrewakeSpins, 1, ld(hs.prewake_spin_timeouts), gen, [] { return std::vector<std::string>{"timeout"}; });
  gput(kFamSelfPrewakeSpinS, 0, ld(hs.prewake_spin_ns) * 1e-9, gen, none);
  gput(kFamSelfRxMoves, 0, ld(hs.rx_cpu_moves), gen, none);
  if (cfg_.http.enable_gzip) {
    gput(kFamSelfGzip, 0, double(gzip_eager_), gen, [] { return std::vector<std::string>{"sampler"}; });
    gput(kFamSelfGzip, 1, ld(hs.gzip_on_demand), gen, [] { return std::vector<std::string>{"request"}; });
  }
}

}  // namespace gpuexp
