// KFD SMI event families: per-GPU event counts (VM faults, thermal throttling, resets, queue
// evictions / restores) from the KFD SMI event fds, and per-pod counts of the events that name
// a process (PID -> cgroup -> pod through the resolver's cache, so a process killed by its own
// VM fault is still attributed if it was seen before).
//
// Reference counterpart: none -- the reference's only error path is log.Fatalf on an NVML
// failure (/root/reference/main.go:119-137).
#include <set>

#include "gpuexp/engine.h"

namespace gpuexp {

const std::vector<FamilySpec>& kfd_event_family_specs() {
  static const std::vector<FamilySpec> t = {
      {kFamKfdEv, "amd_gpu_kfd_events_total",
       "KFD SMI events on this GPU: vm_fault (a process's GPU page fault), thermal_throttle, "
       "gpu_pre_reset / gpu_post_reset, queue_eviction / queue_restore (full profile)",
       MetricType::kCounter, LabelBase::kDevice, {"event"}, RefScope::kGpu, int(std::size(kKfdSubscribed))},
      {kFamPodKfdEv, "amd_pod_gpu_kfd_events_total",
       "Per-process KFD SMI events (vm_fault, queue_eviction, queue_restore) of a pod's processes, "
       "over all GPUs",
       MetricType::kCounter, LabelBase::kNone, {"namespace", "pod", "event"}, RefScope::kKeyed, 0},
  };
  return t;
}

// Drains the KFD event fds (and injected bytes) into per-GPU and per-pod counts.
void Engine::count_kfd_events() {
  std::vector<KfdEvent> evs;
  kfd_events_->drain(&evs);
  {
    std::lock_guard<std::mutex> lk(ctl_mu_);
    for (auto& b : pending_kfd_bytes_) kfd_events_->feed(b.first, b.second.data(), b.second.size(), &evs);
    pending_kfd_bytes_.clear();
  }
  for (const KfdEvent& e : evs) {
    if (e.dev < 0 || size_t(e.dev) >= dstate_.size() || e.event <= 0 || e.event >= kKfdEventIds) continue;
    dstate_[size_t(e.dev)].kfd_events[e.event] += 1;
    if (e.pid <= 0) continue;
    const CgroupInfo* ci = cfg_.pod_attribution ? resolver_->resolve(e.pid) : nullptr;
    auto pit = ci && ci->kube ? pods_by_uid_.find(ci->pod_uid) : pods_by_uid_.end();
    if (pit == pods_by_uid_.end()) {
      ++kfd_events_unattributed_;
      continue;
    }
    pod_kfd_events_[std::make_tuple(pit->second.ns, pit->second.name, e.event)] += 1;
  }
}

// A GPU's event counts (with its device labels; collect_device, every tick, also when the
// telemetry read failed: a reset shows here first).
void Engine::emit_device_kfd_events(int dev, uint64_t gen) {
  DevState& st = dstate_[size_t(dev)];
  for (size_t k = 0; k < std::size(kKfdSubscribed); ++k)
    dput(st, dev, kFamKfdEv, int(k), {kfd_event_name(kKfdSubscribed[k])}, double(st.kfd_events[kKfdSubscribed[k]]),
         gen);
}

void Engine::emit_kfd_events(uint64_t gen) {
  // a pod's counts live as long as the control plane knows the pod
  std::set<std::pair<std::string, std::string>> live;
  for (auto& kv : pods_by_uid_) live.emplace(kv.second.ns, kv.second.name);
  for (auto it = pod_kfd_events_.begin(); it != pod_kfd_events_.end();) {
    const auto& k = it->first;
    // restored from the state file while the pod list is not here yet: keep (and export);
    // gone from a complete list, or from every partial one for the TTL: drop
    const std::pair<std::string, std::string> pk{std::get<0>(k), std::get<1>(k)};
    auto lk = pod_last_known_ns_.find(pk);
    if (lk == pod_last_known_ns_.end() && !live.count(pk))  // never listed yet: the TTL starts now
      lk = pod_last_known_ns_.emplace(pk, mono_ns()).first;
    const bool expired =
        lk != pod_last_known_ns_.end() && mono_ns() - lk->second > uint64_t(cfg_.pod_totals_ttl_s * 1e9);
    if (!live.count(pk) && (pods_complete_ || expired)) {
      it = pod_kfd_events_.erase(it);
      continue;
    }
    if (emit_)
      table_.put(fam_ids_[kFamPodKfdEv], {std::get<0>(k), std::get<1>(k), kfd_event_name(std::get<2>(k))},
                 double(it->second), gen);
    ++it;
  }
}

}  // namespace gpuexp
