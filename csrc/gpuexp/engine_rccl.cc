// RCCL families: per-(process, op) collective calls and payload bytes, and each process's
// largest communicator, from the rocprofiler-sdk tracer tool's shared-memory files
// (rccl_tracer.cc -> rccl_shm.h), attributed to pods like the GPU processes.
//
// Reference counterpart: none -- the reference issues and observes no collectives (SURVEY
// §2.5); the exporter observes RCCL-over-xGMI traffic per pod.
#include "gpuexp/engine.h"

namespace gpuexp {

namespace {
constexpr auto G = MetricType::kGauge;
constexpr auto C = MetricType::kCounter;
constexpr auto N = LabelBase::kNone;
}  // namespace

const std::vector<FamilySpec>& rccl_family_specs() {
  static const std::vector<FamilySpec> t = {
      {kFamRcclCalls, "amd_rccl_collective_calls_total", "RCCL collective/p2p calls by op (rocprofiler-sdk tracer)", C,
       N, {"namespace", "pod", "pid", "op"}, RefScope::kKeyed, 0},
      {kFamRcclBytes, "amd_rccl_collective_bytes_total", "RCCL payload bytes by op (rocprofiler-sdk tracer)", C, N,
       {"namespace", "pod", "pid", "op"}, RefScope::kKeyed, 0},
      {kFamRcclComm, "amd_rccl_communicator_info",
       "Rank and size of the largest RCCL communicator of a process (value is always 1)", G, N,
       {"namespace", "pod", "pid", "rank", "nranks"}, RefScope::kKeyed, 0},
      {kFamSelfRcclFiles, "gpuexp_rccl_files",
       "RCCL tracer directory entries by state: active (writer identified, exported), "
       "unverified (no live process maps it as claimed), exited (writer gone, file left "
       "behind), ignored (not a tracer file, not a regular file, or over the 1024-file cap)",
       G, N, {"state"}, RefScope::kGlobal, 4},
      {kFamSelfRcclScans, "gpuexp_rccl_dir_scans_total",
       "Listings of the RCCL tracer directory (only when it changed, at most once per "
       "rccl_scan_interval_s)",
       C, N, {}, RefScope::kGlobal, 1},
  };
  return t;
}

void Engine::emit_rccl(uint64_t gen) {
  if (!rccl_) return;
  std::vector<RcclTotals> tot;
  rccl_->poll(&tot);
  for (auto& t : tot) {
    ProcAttr a;
    auto it = attr_cache_.find(t.pid);
    if (it != attr_cache_.end()) {
      a = it->second;
    } else if (cfg_.pod_attribution) {
      const CgroupInfo* ci = resolver_->resolve(t.pid);
      if (ci && ci->kube) {
        auto pit = pods_by_uid_.find(ci->pod_uid);
        if (pit != pods_by_uid_.end()) {
          a.ns = pit->second.ns;
          a.pod = pit->second.name;
        } else {
          unresolved_.insert(ci->pod_uid);
        }
      }
    }
    // handles cached per (PID, op) while the labels stay the same (no label vector per tick)
    RcclRefs& r = rccl_refs_[{t.pid, t.op}];
    if (r.ns != a.ns || r.pod != a.pod || r.rank != t.rank || r.nranks != t.nranks) {
      r = RcclRefs();
      r.ns = a.ns;
      r.pod = a.pod;
      r.rank = t.rank;
      r.nranks = t.nranks;
    }
    r.gen = gen;
    auto L = [&] { return std::vector<std::string>{a.ns, a.pod, std::to_string(t.pid), t.op}; };
    cput(r.calls, fam_ids_[kFamRcclCalls], double(t.calls), gen, L);
    cput(r.bytes, fam_ids_[kFamRcclBytes], double(t.bytes), gen, L);
    if (t.nranks > 0 && t.rank >= 0)
      cput(r.comm, fam_ids_[kFamRcclComm], 1, gen, [&] {
        return std::vector<std::string>{a.ns, a.pod, std::to_string(t.pid), std::to_string(t.rank),
                                        std::to_string(t.nranks)};
      });
  }
  for (auto it = rccl_refs_.begin(); it != rccl_refs_.end();)
    it = it->second.gen != gen ? rccl_refs_.erase(it) : std::next(it);
}

// The tracer directory's own health (emitted with the self-metrics).
void Engine::emit_rccl_self(uint64_t gen) {
  if (!rccl_) return;
  int a = 0, u = 0, x = 0;
  rccl_->file_states(&a, &u, &x);
  static const char* const kStates[4] = {"active", "unverified", "exited", "ignored"};
  const double v[4] = {double(a), double(u), double(x), double(rccl_->ignored())};
  for (int k = 0; k < 4; ++k)
    gput(kFamSelfRcclFiles, k, v[k], gen, [&] { return std::vector<std::string>{kStates[k]}; });
  gput(kFamSelfRcclScans, 0, double(rccl_->scans()), gen, [] { return std::vector<std::string>{}; });
}

}  // namespace gpuexp
