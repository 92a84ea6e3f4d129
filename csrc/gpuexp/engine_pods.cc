// Per-pod families: device ownership (device-plugin map, else single-pod inference), the
// per-pod aggregates of a tick (VRAM, processes, GPUs, xGMI, power, activity, MFMA, HBM) and
// the per-pod totals that outlive GPU processes (energy, xGMI bytes, GPU-seconds; kept in the
// state file across exporter restarts).
//
// Reference counterpart: the pod name is the only per-pod output, as the `pod` label of the two
// legacy gauges (/root/reference/main.go:140-150); pods are listed cluster-wide every cycle
// (main.go:75-89).
#include <climits>
#include <cmath>

#include "gpuexp/engine.h"
#include "gpuexp/engine_util.h"

namespace gpuexp {

using engine_util::acc_delta;

namespace {
constexpr auto G = MetricType::kGauge;
constexpr auto C = MetricType::kCounter;
constexpr auto PO = LabelBase::kPod;
constexpr auto K = RefScope::kKeyed;
}  // namespace

const std::vector<FamilySpec>& pod_family_specs() {
  static const std::vector<FamilySpec> t = {
      {kFamPodVram, "amd_pod_gpu_vram_bytes", "VRAM held by all GPU processes of a pod", G, PO, {}, K, 0},
      {kFamPodProcs, "amd_pod_gpu_processes", "GPU processes of a pod", G, PO, {}, K, 0},
      {kFamPodGpus, "amd_pod_gpus", "GPUs attributed to a pod", G, PO, {}, K, 0},
      {kFamPodXrd, "amd_pod_xgmi_read_bytes_per_second", "xGMI receive rate of the pod's GPUs", G, PO, {}, K, 0},
      {kFamPodXwr, "amd_pod_xgmi_write_bytes_per_second", "xGMI transmit rate of the pod's GPUs", G, PO, {}, K, 0},
      {kFamPodXrdTotal, "amd_pod_xgmi_read_bytes_total",
       "xGMI bytes received by the pod's GPUs (per-tick link accumulator deltas; on a shared GPU "
       "the pod's CU-occupancy share)",
       C, PO, {}, K, 0},
      {kFamPodXwrTotal, "amd_pod_xgmi_write_bytes_total",
       "xGMI bytes sent by the pod's GPUs (per-tick link accumulator deltas; on a shared GPU the "
       "pod's CU-occupancy share)",
       C, PO, {}, K, 0},
      {kFamPodMfma, "amd_pod_gpu_mfma_busy_percent",
       "Mean MFMA busy of the pod's GPUs (amd_gpu_mfma_busy_percent of each GPU it owns)", G, PO, {}, K, 0},
      {kFamPodFlops, "amd_pod_gpu_mfma_flops_per_second",
       "MFMA FLOP/s of the pod's GPUs by operand type (sum of amd_gpu_mfma_flops_per_second over "
       "the GPUs it owns)",
       G, PO, {"dtype"}, K, 0},
      {kFamPodHbm, "amd_pod_gpu_hbm_bandwidth_bytes_per_second",
       "HBM bandwidth of the pod's GPUs (sum of amd_gpu_hbm_bandwidth_bytes_per_second over the GPUs it owns)", G,
       PO, {}, K, 0},
      {kFamPodPower, "amd_pod_gpu_power_watts", "Socket power of the pod's GPUs", G, PO, {}, K, 0},
      {kFamPodAllocS, "amd_pod_gpu_allocated_seconds_total",
       "GPU-seconds the pod has held GPUs (device-plugin allocation; one GPU for one second = 1)", C, PO, {}, K, 0},
      {kFamPodBusyS, "amd_pod_gpu_busy_seconds_total",
       "GPU-seconds the pod's GPUs were busy (per-XCD gfx_busy accumulators; a shared GPU's busy time "
       "split by the pod's CU-occupancy share)",
       C, PO, {}, K, 0},
      {kFamPodEnergy, "amd_pod_gpu_energy_joules_total",
       "GPU energy used by the pod: its GPUs' hardware energy counters, and on a shared GPU the "
       "pod's CU-occupancy share of it (chargeback)",
       C, PO, {}, K, 0},
      {kFamPodGfx, "amd_pod_gpu_gfx_activity_percent", "Mean gfx activity of the pod's GPUs", G, PO, {}, K, 0},
      {kFamPodGfxShare, "amd_pod_gfx_activity_share_percent",
       "GPU gfx activity of the pod's processes summed over GPUs, in percent of one GPU "
       "(per-process CU-occupancy split; covers shared GPUs)",
       G, PO, {}, K, 0},
  };
  return t;
}

// Stage 2 of a tick: each GPU's owner -- the device plugin's map first (PodResources, keyed by
// the device's ids), else the single pod all its processes belong to (cached while the GPU's
// processes, by KFD identity, and the control plane stay the same).
void Engine::infer_owners(const std::vector<std::vector<ProcSample>>& per_dev) {
  for (size_t i = 0; i < devices_.size(); ++i) {
    DevState& st = dstate_[i];
    DeviceOwner own;
    auto it = owners_.end();
    for (const std::string& key : owner_keys_[i]) {
      it = owners_.find(key);
      if (it != owners_.end()) break;
    }
    if (it != owners_.end()) {
      own = it->second;
    } else if (cfg_.pod_attribution && cfg_.infer_device_owner) {
      // the same processes (KFD identities, order-free) under the same control plane infer the
      // same owner: reuse it instead of resolving and building sets of label strings every tick
      uint64_t sig = 0x9E3779B97F4A7C15ull ^ ctl_epoch_;
      bool cacheable = true;
      for (auto& p : per_dev[i]) {
        cacheable = cacheable && p.kfd_id != 0;
        sig += (p.kfd_id ^ (uint64_t(uint32_t(p.pid)) << 32)) * 0xBF58476D1CE4E5B9ull;
      }
      sig = cacheable ? (sig | 1) : 0;
      if (sig && sig == st.owner_sig) {
        st.owner = st.owner_inferred;
        continue;
      }
      std::set<std::tuple<std::string, std::string, std::string>> seen;
      for (auto& p : per_dev[i]) {
        const CgroupInfo* ci = resolver_->resolve(p.pid, p.kfd_id);
        if (!ci) sig = 0;  // unreadable /proc/<pid>: ask again next tick
        if (!ci || !ci->kube) continue;
        auto pit = pods_by_uid_.find(ci->pod_uid);
        if (pit == pods_by_uid_.end()) {
          seen.emplace("", "", "");  // an unnamed pod: ownership stays unknown
          continue;
        }
        auto cn = container_names_.find(ci->container_id);
        seen.emplace(pit->second.ns, pit->second.name, cn != container_names_.end() ? cn->second : "");
      }
      std::set<std::pair<std::string, std::string>> podset;
      for (auto& t : seen) podset.emplace(std::get<0>(t), std::get<1>(t));
      if (podset.size() == 1 && !podset.begin()->second.empty()) {
        own.ns = podset.begin()->first;
        own.pod = podset.begin()->second;
        if (seen.size() == 1) own.container = std::get<2>(*seen.begin());
      }
      st.owner_sig = sig;
      st.owner_inferred = own;
    }
    st.owner = own;
  }
}

void Engine::emit_pods(uint64_t gen, const std::vector<std::vector<ProcSample>>& per_dev) {
  std::map<std::pair<std::string, std::string>, PodAgg>& pods = pod_agg_;
  pods.clear();
  for (size_t di = 0; di < per_dev.size(); ++di) {
    DevState& st = dstate_[di];
    const CuSplit cus(per_dev[di]);
    const double act = st.cur.ok ? st.cur.gfx_activity : kNaN;
    // energy this GPU used since the last tick, from its hardware accumulator (exact)
    double energy_j = kNaN;
    if (st.cur.ok && st.have_prev && st.cur.energy_valid && st.prev.energy_valid) {
      double dacc;
      if (acc_delta(st.cur.energy_acc, st.prev.energy_acc, &dacc)) energy_j = dacc * st.cur.energy_unit_j;
    }
    // this tick's length and the GPU's busy fraction over it (mean of the per-XCD busy from
    // the gfx_busy accumulators; the PMFW's gfx activity where those are missing)
    double tick_s = kNaN, busy_frac = kNaN;
    if (st.cur.ok && st.have_prev && st.cur.host_ns > st.prev.host_ns) {
      tick_s = double(st.cur.host_ns - st.prev.host_ns) * 1e-9;
      if (tick_s > 60.0) tick_s = kNaN;  // a stalled sampler: do not credit the gap
      double sum = 0;
      int n = 0;
      for (int x = 0; x < kMaxXcc; ++x)
        if (!std::isnan(st.xcc_last[x])) {
          sum += st.xcc_last[x];
          ++n;
        }
      busy_frac = n ? sum / n / 100.0 : st.cur.gfx_activity / 100.0;
    }
    // xGMI bytes this GPU moved since the last tick, summed over links (hardware accumulators)
    double xgmi_rd_b = kNaN, xgmi_wr_b = kNaN;
    if (st.cur.ok && st.have_prev && st.cur.xgmi_valid && st.prev.xgmi_valid) {
      double r = 0, w = 0;
      bool ok = true;
      for (int l = 0; l < kMaxXgmiLinks && ok; ++l) {
        double dr, dw;
        ok = acc_delta(st.cur.xgmi_read_kb[l], st.prev.xgmi_read_kb[l], &dr) &&
             acc_delta(st.cur.xgmi_write_kb[l], st.prev.xgmi_write_kb[l], &dw);
        r += ok ? dr : 0;
        w += ok ? dw : 0;
      }
      if (ok) {  // a reset link skips the tick (as the rates do)
        xgmi_rd_b = r * 1024.0;
        xgmi_wr_b = w * 1024.0;
      }
    }
    const bool shared = st.owner.pod.empty();
    for (auto& p : per_dev[di]) {
      const ProcAttr& a = attr_cache_[p.pid];
      if (a.pod.empty()) continue;
      auto& pa = pods[{a.ns, a.pod}];
      pa.vram += p.vram_bytes;
      pa.pids.insert(p.pid);
      const double f = cus.frac(p);
      const double share = std::isnan(act) ? act : act * f;
      if (shared && !std::isnan(energy_j) && !std::isnan(f)) pa.energy_j += energy_j * f;
      if (shared && !std::isnan(xgmi_rd_b) && !std::isnan(f)) {
        pa.xrd_b += xgmi_rd_b * f;
        pa.xwr_b += xgmi_wr_b * f;
      }
      // a shared GPU's time is split like its busy time, so busy <= allocated for every pod
      // (the rules' busy / allocated ratio stays a ratio)
      if (shared && !std::isnan(tick_s) && !std::isnan(f)) {
        pa.alloc_s += tick_s * f;
        if (!std::isnan(busy_frac)) pa.busy_s += busy_frac * tick_s * f;
      }
      if (!std::isnan(share)) {
        pa.gfx_share += share;
        pa.share_known = true;
      }
    }
    if (st.owner.pod.empty()) continue;
    auto& pa = pods[{st.owner.ns, st.owner.pod}];
    pa.gpus += 1;
    if (!st.cur.ok) continue;
    if (st.rates_valid)
      for (int l = 0; l < kMaxXgmiLinks; ++l) {
        pa.xrd += st.xgmi_rd_rate[l];
        pa.xwr += st.xgmi_wr_rate[l];
      }
    if (!std::isnan(st.cur.power_w)) pa.power += st.cur.power_w;
    if (!std::isnan(energy_j)) pa.energy_j += energy_j;  // an owned GPU's energy is all the pod's
    if (!std::isnan(xgmi_rd_b)) {                        // ...and so is its xGMI traffic
      pa.xrd_b += xgmi_rd_b;
      pa.xwr_b += xgmi_wr_b;
    }
    if (!std::isnan(tick_s)) {  // ...and its time, busy or not
      pa.alloc_s += tick_s;
      if (!std::isnan(busy_frac)) pa.busy_s += busy_frac * tick_s;
    }
    if (!std::isnan(st.cur.gfx_activity)) {
      pa.gfx += st.cur.gfx_activity;
      pa.gfx_n += 1;
    }
    if (!std::isnan(st.mfma_last)) {
      pa.mfma += st.mfma_last;
      pa.mfma_n += 1;
    }
    if (!std::isnan(st.flops_last[0]) && !std::isnan(st.flops_last[1])) {  // an owned GPU's work is the pod's
      pa.flops[0] += st.flops_last[0];
      pa.flops[1] += st.flops_last[1];
      pa.flops_n += 1;
    }
    if (!std::isnan(st.cur.umc_activity) && st.cur.vram_max_bw_gbs > 0) {
      pa.hbm += st.cur.umc_activity / 100.0 * st.cur.vram_max_bw_gbs * 1e9;  // as amd_gpu_hbm_bandwidth
      pa.hbm_n += 1;
    }
  }
  for (auto& kv : pods) {
    PodRefs& r = pod_refs_[kv.first];
    r.gen = gen;
    auto L = [&] { return std::vector<std::string>{kv.first.first, kv.first.second}; };
    auto put = [&](Fam f, double v) { cput(podref(r, f), fam_ids_[f], v, gen, L); };
    const PodAgg& pa = kv.second;
    put(kFamPodVram, pa.vram);
    put(kFamPodProcs, double(pa.pids.size()));
    put(kFamPodGpus, double(pa.gpus));
    if (pa.share_known) put(kFamPodGfxShare, pa.gfx_share);
    if (pa.gpus > 0) {
      put(kFamPodXrd, pa.xrd);
      put(kFamPodXwr, pa.xwr);
      put(kFamPodPower, pa.power);
      if (pa.gfx_n) put(kFamPodGfx, pa.gfx / pa.gfx_n);
      if (pa.mfma_n) put(kFamPodMfma, pa.mfma / pa.mfma_n);
      if (pa.hbm_n) put(kFamPodHbm, pa.hbm);
      if (pa.flops_n) {
        static const char* kTypes[2] = {"bf16", "fp8"};
        for (int k = 0; k < 2; ++k)
          cput(podref(r, kFamPodFlops, k), fam_ids_[kFamPodFlops], pa.flops[k], gen,
               [&] { return std::vector<std::string>{kv.first.first, kv.first.second, kTypes[k]}; });
      }
    }
  }
  for (auto it = pod_refs_.begin(); it != pod_refs_.end();)
    it = it->second.gen != gen ? pod_refs_.erase(it) : std::next(it);
  emit_pod_totals(gen);
}

// Energy, xGMI bytes and GPU-seconds per pod: counters that live as long as the control plane
// knows the pod, so a pod between GPU processes keeps its totals (and an exporter restart too,
// through the state file).
void Engine::emit_pod_totals(uint64_t gen) {
  for (auto& kv : pod_agg_) {
    if (kv.second.energy_j > 0) pod_energy_j_[kv.first] += kv.second.energy_j;
    if (kv.second.xrd_b > 0 || kv.second.xwr_b > 0) {
      auto& x = pod_xgmi_[kv.first];
      x.first += kv.second.xrd_b;
      x.second += kv.second.xwr_b;
    }
    if (kv.second.alloc_s > 0 || kv.second.busy_s > 0) {
      auto& g = pod_gpu_s_[kv.first];
      g.first += kv.second.alloc_s;
      g.second += kv.second.busy_s;
    }
  }
  std::set<std::pair<std::string, std::string>> known;
  for (auto& kv : pods_by_uid_) known.emplace(kv.second.ns, kv.second.name);
  // A pod's totals go when a complete pod list no longer has it -- or, while refreshes stay
  // partial (a metadata source keeps failing), once no applied list has had it for
  // pod_totals_ttl_s (so the maps and the state file cannot grow with every pod ever run).
  const uint64_t now_ns = mono_ns();
  auto gone = [&](const std::pair<std::string, std::string>& k) {
    if (known.count(k)) return false;
    if (pods_complete_) return true;
    auto it = pod_last_known_ns_.find(k);
    if (it == pod_last_known_ns_.end()) {  // restored from the state file, never listed yet
      pod_last_known_ns_[k] = now_ns;
      return false;
    }
    return now_ns - it->second > uint64_t(cfg_.pod_totals_ttl_s * 1e9);
  };
  for (auto it = pod_energy_j_.begin(); it != pod_energy_j_.end();) {
    if (gone(it->first)) {
      it = pod_energy_j_.erase(it);
      continue;
    }
    if (emit_) table_.put(fam_ids_[kFamPodEnergy], {it->first.first, it->first.second}, it->second, gen);
    ++it;
  }
  for (auto it = pod_xgmi_.begin(); it != pod_xgmi_.end();) {
    if (gone(it->first)) {
      it = pod_xgmi_.erase(it);
      continue;
    }
    if (emit_) table_.put(fam_ids_[kFamPodXrdTotal], {it->first.first, it->first.second}, it->second.first, gen);
    if (emit_) table_.put(fam_ids_[kFamPodXwrTotal], {it->first.first, it->first.second}, it->second.second, gen);
    ++it;
  }
  for (auto it = pod_gpu_s_.begin(); it != pod_gpu_s_.end();) {
    if (gone(it->first)) {
      it = pod_gpu_s_.erase(it);
      continue;
    }
    if (emit_) table_.put(fam_ids_[kFamPodAllocS], {it->first.first, it->first.second}, it->second.first, gen);
    if (emit_) table_.put(fam_ids_[kFamPodBusyS], {it->first.first, it->first.second}, it->second.second, gen);
    ++it;
  }
  // a pod's stamp lives while any of its totals does (KFD event counts included: they expire
  // in emit_kfd_events against the same stamp)
  auto has_kfd = [&](const std::pair<std::string, std::string>& k) {
    auto kt = pod_kfd_events_.lower_bound(std::make_tuple(k.first, k.second, INT_MIN));
    return kt != pod_kfd_events_.end() && std::get<0>(kt->first) == k.first && std::get<1>(kt->first) == k.second;
  };
  for (auto it = pod_last_known_ns_.begin(); it != pod_last_known_ns_.end();)
    it = !known.count(it->first) && !pod_energy_j_.count(it->first) && !pod_xgmi_.count(it->first) &&
                 !pod_gpu_s_.count(it->first) && !has_kfd(it->first)
             ? pod_last_known_ns_.erase(it)
             : std::next(it);
}

}  // namespace gpuexp
