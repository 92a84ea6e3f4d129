// Per-process families: PID -> pod attribution (cgroup-v2 path -> pod UID -> control-plane
// metadata, cached while KFD vouches for the process), the per-(GPU, PID) series, the GPU's
// process count / CU occupancy, and the reference's two legacy families.
//
// Reference counterpart: kubectl exec `ps` per container (/root/reference/main.go:91-113) and
// the index-vs-PID join (main.go:140-150): here host PIDs end to end.
#include <cmath>

#include "gpuexp/engine.h"

namespace gpuexp {

namespace {
constexpr auto G = MetricType::kGauge;
constexpr auto C = MetricType::kCounter;
constexpr auto P = LabelBase::kProcess;
constexpr auto K = RefScope::kKeyed;
}  // namespace

const std::vector<FamilySpec>& process_family_specs() {
  static const std::vector<FamilySpec> t = {
      {kFamProcVram, "amd_gpu_process_vram_bytes", "VRAM held by a process on a GPU (KFD)", G, P, {}, K, 0},
      {kFamProcCu, "amd_gpu_process_cu_occupancy",
       "Resident waves of a process on a GPU in CU-equivalents (KFD stats_<id>/cu_occupancy)", G, P, {}, K, 0},
      {kFamProcSdma, "amd_gpu_process_sdma_seconds_total",
       "KFD's per-process SDMA activity (sdma_<gpu_id>, read as microseconds); only with "
       "kfd_sdma_activity: on MI355X the file is not SDMA time (one jump at the first copy, "
       "then flat under 55 GB/s of copies)",
       C, P, {}, K, 0},
      {kFamProcEvicted, "amd_gpu_process_evicted_seconds_total",
       "Time the process's GPU queues were evicted (memory pressure / preemption; KFD stats)", C, P, {}, K, 0},
      {kFamProcGfx, "amd_gpu_process_gfx_activity_percent",
       "GPU gfx activity attributed to a process: the GPU's activity split by the processes' "
       "occupied CUs (estimate on shared GPUs; exact for a sole process)",
       G, P, {}, K, 0},
      // Byte-compatible with the reference (/root/reference/main.go:22-35): names, HELP, label
      // names and order {pid, pod}.  `pid` is the host PID (the reference's intended meaning;
      // it accidentally exported a slice index, main.go:144).
      {kFamLegacyMem, "pod_gpu_memory_usage", "GPU memory used by Kubernetes Pod", G, LabelBase::kNone,
       {"pid", "pod"}, K, 0, true},
      {kFamLegacyPerc, "docker_gpu_memory_perc_usage", "GPU memory in percentage used by pod", G, LabelBase::kNone,
       {"pid", "pod"}, K, 0, true},
  };
  return t;
}

Engine::CuSplit::CuSplit(const std::vector<ProcSample>& procs) : n(procs.size()) {
  for (auto& q : procs)
    if (!std::isnan(q.cu_occupancy)) {
      sum += q.cu_occupancy;
      any = true;
    }
}

double Engine::CuSplit::frac(const ProcSample& p) const {
  if (n == 0) return kNaN;
  if (n == 1) return 1.0;
  if (any && sum > 0) return std::isnan(p.cu_occupancy) ? kNaN : p.cu_occupancy / sum;
  return 1.0 / double(n);
}

void Engine::emit_processes(uint64_t gen, const std::vector<std::vector<ProcSample>>& per_dev) {
  // pid -> attribution, resolved once per tick (and kept while KFD vouches for the process)
  unresolved_.clear();
  std::vector<int>& live = live_scratch_;
  live.clear();
  for (auto& lst : per_dev)
    for (auto& p : lst) {
      ProcAttr& a = attr_cache_[p.pid];
      if (a.seen == gen) continue;
      a.seen = gen;
      live.push_back(p.pid);
      if (p.kfd_id && a.kfd_id == p.kfd_id && a.ctl_epoch == ctl_epoch_) {
        if (!a.uid.empty() && a.pod.empty()) unresolved_.insert(a.uid);
        continue;
      }
      a.ns.clear();
      a.pod.clear();
      a.container.clear();
      a.uid.clear();
      a.kfd_id = p.kfd_id;
      a.ctl_epoch = ctl_epoch_;
      if (cfg_.pod_attribution) {
        const CgroupInfo* ci = resolver_->resolve(p.pid, p.kfd_id);
        if (!ci) a.kfd_id = 0;  // not looked up (unreadable /proc/<pid>): ask the resolver again
        if (ci && ci->kube) {
          a.uid = ci->pod_uid;
          auto it = pods_by_uid_.find(ci->pod_uid);
          if (it != pods_by_uid_.end()) {
            a.ns = it->second.ns;
            a.pod = it->second.name;
          } else {
            // Name unknown until the control plane reports it: pod="" meanwhile (a UID
            // in `pod` would change the series identity once the name arrives).
            unresolved_.insert(ci->pod_uid);
          }
          auto cn = container_names_.find(ci->container_id);
          if (cn != container_names_.end()) a.container = cn->second;
        }
      }
    }
  for (auto it = attr_cache_.begin(); it != attr_cache_.end();)
    it = it->second.seen != gen ? attr_cache_.erase(it) : std::next(it);
  resolver_->gc(live);

  struct PidAgg {
    double used = 0, total = 0;
  };
  std::map<int, PidAgg> legacy;
  const bool legacy_only = cfg_.series_profile == "legacy";
  for (size_t di = 0; di < per_dev.size(); ++di) {
    const DeviceInfo& d = devices_[di];
    DevState& st = dstate_[di];
    const double act = st.cur.ok ? st.cur.gfx_activity : kNaN;
    const CuSplit cus(per_dev[di]);
    for (auto& p : per_dev[di]) {
      const ProcAttr& a = attr_cache_[p.pid];
      if (!legacy_only) {
        // handles cached per (GPU, PID) for as long as the label values stay the same
        ProcRefs& pr = proc_refs_[(uint64_t(uint32_t(di)) << 32) | uint32_t(p.pid)];
        if (pr.comm != p.name || pr.ns != a.ns || pr.pod != a.pod || pr.container != a.container) {
          pr = ProcRefs();
          pr.comm = p.name;
          pr.ns = a.ns;
          pr.pod = a.pod;
          pr.container = a.container;
        }
        pr.gen = gen;
        auto L = [&] {
          return std::vector<std::string>{std::to_string(d.index), std::to_string(p.pid), p.name, a.ns, a.pod,
                                          a.container};
        };
        const double share = std::isnan(act) ? act : act * cus.frac(p);
        cput(pref(pr, kFamProcVram), fam_ids_[kFamProcVram], p.vram_bytes, gen, L);
        if (!std::isnan(p.cu_occupancy)) cput(pref(pr, kFamProcCu), fam_ids_[kFamProcCu], p.cu_occupancy, gen, L);
        if (!std::isnan(p.sdma_us)) cput(pref(pr, kFamProcSdma), fam_ids_[kFamProcSdma], p.sdma_us * 1e-6, gen, L);
        if (!std::isnan(p.evicted_ms))
          cput(pref(pr, kFamProcEvicted), fam_ids_[kFamProcEvicted], p.evicted_ms * 1e-3, gen, L);
        if (!std::isnan(share)) cput(pref(pr, kFamProcGfx), fam_ids_[kFamProcGfx], share, gen, L);
      }
      if (!a.pod.empty()) {
        auto& la = legacy[p.pid];
        la.used += p.vram_bytes;
        la.total += double(d.vram_total);
      }
    }
    if (st.cur.ok && !legacy_only) {
      dput(st, int(di), kFamNprocs, 0, {}, double(per_dev[di].size()), gen);
      // No processes -> 0 CUs occupied (a known value, not an unknown one).
      if (cus.any || per_dev[di].empty()) dput(st, int(di), kFamCuOcc, 0, {}, cus.sum, gen);
    }
  }
  if (fam_ids_[kFamLegacyMem] >= 0) {
    // Legacy families: one series per attributed host PID, summed over GPUs (the
    // reference overwrote per device, last-device-wins, main.go:147-150).
    for (auto& kv : legacy) {
      const ProcAttr& a = attr_cache_[kv.first];
      ProcRefs& pr = legacy_refs_[uint64_t(uint32_t(kv.first))];
      if (pr.pod != a.pod) {
        pr = ProcRefs();
        pr.pod = a.pod;
      }
      pr.gen = gen;
      auto L = [&] { return std::vector<std::string>{std::to_string(kv.first), a.pod}; };
      cput(pref(pr, kFamLegacyMem), fam_ids_[kFamLegacyMem], kv.second.used, gen, L);
      cput(pref(pr, kFamLegacyPerc), fam_ids_[kFamLegacyPerc],
           kv.second.total > 0 ? kv.second.used / kv.second.total * 100.0 : 0.0, gen, L);
    }
  }
  // forget the handles of processes gone this tick (their series are GC'd by the table)
  for (auto* m : {&proc_refs_, &legacy_refs_})
    for (auto it = m->begin(); it != m->end();) it = it->second.gen != gen ? m->erase(it) : std::next(it);
}

}  // namespace gpuexp
