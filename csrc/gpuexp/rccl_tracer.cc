// libgpuexp_rccl_tracer.so — rocprofiler-sdk tool that makes RCCL collectives visible per
// pod (SURVEY.md §2.5 / §5 "Distributed communication backend").
//
// Inject into a workload with ROCP_TOOL_LIBRARIES=/path/libgpuexp_rccl_tracer.so (and
// GPUEXP_RCCL_DIR pointing at a hostPath the exporter also mounts).  On every RCCL API
// ENTER callback for a data-moving call it adds {calls += 1, bytes += payload} to the
// per-op counters of a shared-memory file (csrc/gpuexp/rccl_shm.h).  The exporter maps
// the file's (pid-namespace inode, in-namespace pid) to a host PID, then to the pod, and
// exports amd_rccl_collective_{calls,bytes}_total{namespace,pod,pid,op} — DP all-reduce,
// TP/SP all-gather + reduce-scatter, EP/Ulysses all-to-all, PP/CP send/recv.
//
// Payload bytes per call, per rank (what this rank contributes to the wire pattern):
//   allreduce/reduce/broadcast: count * size       allgather: sendcount * size * nranks
//   reducescatter: recvcount * size * nranks        alltoall: count * size * nranks
//   alltoallv: sum(sendcounts) * size               send/recv: count * size
//   gather: sendcount * size                        scatter: recvcount * size
// (pinned at nranks 1/2/8 for every op by tests/test_rccl_tracer_bytes.py)
// nranks (and the process's rank) come from the communicator's creation call
// (ncclCommInitRank / ncclCommInitRankConfig EXIT: nranks, myrank, *newcomm), cached per
// communicator; communicators made otherwise (ncclCommSplit, ncclCommInitAll) are asked
// with ncclCommCount / ncclCommUserRank, resolved in the already-loaded librccl (torch
// loads it RTLD_LOCAL, so a plain dlsym(RTLD_DEFAULT) does not see it).
#include <dlfcn.h>
#include <link.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>

#include "gpuexp/rccl_shm.h"

namespace {

using gpuexp::RcclShmFile;

RcclShmFile* g_shm = nullptr;
std::string g_path;
rocprofiler_context_id_t g_ctx{};
std::mutex g_comm_mu;
std::unordered_map<const void*, int> g_nranks;
thread_local bool t_in_query = false;

size_t dtype_size(int t) {
  switch (t) {
    case 0: case 1: case 10: case 11: return 1;  // int8 uint8 fp8e4m3 fp8e5m2
    case 6: case 9: return 2;                    // float16 bfloat16
    case 2: case 3: case 7: return 4;            // int32 uint32 float32
    case 4: case 5: case 8: return 8;            // int64 uint64 float64
    default: return 1;
  }
}

// Handle of the librccl the process already loaded (never loads one itself).
void* rccl_lib() {
  static void* h = [] {
    std::string name;
    dl_iterate_phdr(
        [](dl_phdr_info* info, size_t, void* out) -> int {
          if (info->dlpi_name && std::strstr(info->dlpi_name, "librccl")) {
            *static_cast<std::string*>(out) = info->dlpi_name;
            return 1;
          }
          return 0;
        },
        &name);
    void* lib = name.empty() ? nullptr : ::dlopen(name.c_str(), RTLD_NOW | RTLD_NOLOAD);
    return lib ? lib : RTLD_DEFAULT;
  }();
  return h;
}

// Caller holds g_comm_mu.  The file reports the process's largest communicator (its world
// / data-parallel group; TP/PP/EP sub-communicators are smaller), so the rank is stable.
void note_comm_locked(const void* comm, int n, int rank) {
  g_nranks[comm] = n;
  // a larger communicator wins; an equal-sized one only fills in an unknown rank (never
  // replaces a known rank with -1 from a communicator that could not be queried)
  if (g_shm && (n > g_shm->nranks || (n == g_shm->nranks && g_shm->rank < 0 && rank >= 0))) {
    g_shm->nranks = n;
    g_shm->rank = rank;
  }
}

int comm_nranks(const void* comm) {
  if (!comm) return 1;
  {
    std::lock_guard<std::mutex> lk(g_comm_mu);
    auto it = g_nranks.find(comm);
    if (it != g_nranks.end()) return it->second;
  }
  using query_fn = int (*)(const void*, int*);
  static query_fn count = reinterpret_cast<query_fn>(::dlsym(rccl_lib(), "ncclCommCount"));
  static query_fn user_rank = reinterpret_cast<query_fn>(::dlsym(rccl_lib(), "ncclCommUserRank"));
  int n = 1, rank = -1;
  if (!t_in_query) {
    t_in_query = true;  // the queries are themselves traced: do not recurse
    if (count && (count(comm, &n) != 0 || n < 1)) n = 1;
    if (user_rank && user_rank(comm, &rank) != 0) rank = -1;
    t_in_query = false;
  }
  std::lock_guard<std::mutex> lk(g_comm_mu);
  note_comm_locked(comm, n, rank);
  return n;
}

void account(int op, uint64_t bytes) {
  if (!g_shm || op < 0) return;
  g_shm->ops[op].calls.fetch_add(1, std::memory_order_relaxed);
  g_shm->ops[op].bytes.fetch_add(bytes, std::memory_order_relaxed);
}

// RCCL implements some collectives with its own public API (all-to-all = a group of
// ncclSend/ncclRecv): only the outermost data-moving call on a thread is accounted.
thread_local int t_depth = 0;

bool moves_data(int op) {
  switch (op) {
    case ROCPROFILER_RCCL_API_ID_ncclAllReduce: case ROCPROFILER_RCCL_API_ID_ncclAllGather:
    case ROCPROFILER_RCCL_API_ID_ncclReduceScatter: case ROCPROFILER_RCCL_API_ID_ncclAllToAll:
    case ROCPROFILER_RCCL_API_ID_ncclAllToAllv: case ROCPROFILER_RCCL_API_ID_ncclBroadcast:
    case ROCPROFILER_RCCL_API_ID_ncclReduce: case ROCPROFILER_RCCL_API_ID_ncclSend:
    case ROCPROFILER_RCCL_API_ID_ncclRecv: case ROCPROFILER_RCCL_API_ID_ncclGather:
    case ROCPROFILER_RCCL_API_ID_ncclScatter:
      return true;
    default:
      return false;
  }
}

void on_rccl(rocprofiler_callback_tracing_record_t rec, rocprofiler_user_data_t*, void*) {
  if (t_in_query) return;
  if (rec.phase == ROCPROFILER_CALLBACK_PHASE_EXIT &&
      (rec.operation == ROCPROFILER_RCCL_API_ID_ncclCommInitRank ||
       rec.operation == ROCPROFILER_RCCL_API_ID_ncclCommInitRankConfig)) {
    // the new communicator exists now: remember its size and this process's rank
    const auto& a = static_cast<const rocprofiler_callback_tracing_rccl_api_data_t*>(rec.payload)->args;
    const bool cfg = rec.operation == ROCPROFILER_RCCL_API_ID_ncclCommInitRankConfig;
    ncclComm_t* out = cfg ? a.ncclCommInitRankConfig.comm : a.ncclCommInitRank.newcomm;
    const int n = cfg ? a.ncclCommInitRankConfig.nranks : a.ncclCommInitRank.nranks;
    const int rank = cfg ? a.ncclCommInitRankConfig.myrank : a.ncclCommInitRank.myrank;
    if (out && *out && n > 0) {
      std::lock_guard<std::mutex> lk(g_comm_mu);
      note_comm_locked(*out, n, rank);
    }
    return;
  }
  if (!moves_data(int(rec.operation))) return;
  if (rec.phase == ROCPROFILER_CALLBACK_PHASE_EXIT) {
    if (t_depth > 0) --t_depth;
    return;
  }
  if (rec.phase != ROCPROFILER_CALLBACK_PHASE_ENTER) return;
  if (t_depth++ > 0) return;  // nested inside another collective
  const auto* d = static_cast<const rocprofiler_callback_tracing_rccl_api_data_t*>(rec.payload);
  const auto& a = d->args;
  using namespace gpuexp;
  switch (rec.operation) {
    case ROCPROFILER_RCCL_API_ID_ncclAllReduce:
      account(kOpAllReduce, a.ncclAllReduce.count * dtype_size(a.ncclAllReduce.datatype));
      break;
    case ROCPROFILER_RCCL_API_ID_ncclAllGather:
      account(kOpAllGather, a.ncclAllGather.sendcount * dtype_size(a.ncclAllGather.datatype) *
                                uint64_t(comm_nranks(a.ncclAllGather.comm)));
      break;
    case ROCPROFILER_RCCL_API_ID_ncclReduceScatter:
      account(kOpReduceScatter, a.ncclReduceScatter.recvcount * dtype_size(a.ncclReduceScatter.datatype) *
                                    uint64_t(comm_nranks(a.ncclReduceScatter.comm)));
      break;
    case ROCPROFILER_RCCL_API_ID_ncclAllToAll:
      account(kOpAllToAll, a.ncclAllToAll.count * dtype_size(a.ncclAllToAll.datatype) *
                               uint64_t(comm_nranks(a.ncclAllToAll.comm)));
      break;
    case ROCPROFILER_RCCL_API_ID_ncclAllToAllv: {
      int n = comm_nranks(a.ncclAllToAllv.comm);
      uint64_t tot = 0;
      for (int i = 0; i < n && a.ncclAllToAllv.sendcounts; ++i) tot += a.ncclAllToAllv.sendcounts[i];
      account(kOpAllToAllv, tot * dtype_size(a.ncclAllToAllv.datatype));
      break;
    }
    case ROCPROFILER_RCCL_API_ID_ncclBroadcast:
      account(kOpBroadcast, a.ncclBroadcast.count * dtype_size(a.ncclBroadcast.datatype));
      break;
    case ROCPROFILER_RCCL_API_ID_ncclReduce:
      account(kOpReduce, a.ncclReduce.count * dtype_size(a.ncclReduce.datatype));
      break;
    case ROCPROFILER_RCCL_API_ID_ncclSend:
      account(kOpSend, a.ncclSend.count * dtype_size(a.ncclSend.datatype));
      break;
    case ROCPROFILER_RCCL_API_ID_ncclRecv:
      account(kOpRecv, a.ncclRecv.count * dtype_size(a.ncclRecv.datatype));
      break;
    case ROCPROFILER_RCCL_API_ID_ncclGather:
      account(kOpGather, a.ncclGather.sendcount * dtype_size(a.ncclGather.datatype));
      break;
    case ROCPROFILER_RCCL_API_ID_ncclScatter:
      account(kOpScatter, a.ncclScatter.recvcount * dtype_size(a.ncclScatter.datatype));
      break;
    default:
      break;
  }
}

bool open_shm() {
  const char* dir = std::getenv("GPUEXP_RCCL_DIR");
  std::string d = dir && *dir ? dir : "/dev/shm";
  struct stat st;
  uint64_t ino = ::stat("/proc/self/ns/pid", &st) == 0 ? uint64_t(st.st_ino) : 0;
  int pid = int(::getpid());
  g_path = d + "/gpuexp-rccl-" + std::to_string(ino) + "-" + std::to_string(pid);
  int fd = ::open(g_path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) return false;
  if (::ftruncate(fd, sizeof(RcclShmFile)) != 0) {
    ::close(fd);
    return false;
  }
  void* p = ::mmap(nullptr, sizeof(RcclShmFile), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) return false;
  g_shm = static_cast<RcclShmFile*>(p);
  g_shm->version = 1;
  g_shm->ns_pid = pid;
  g_shm->pidns_ino = ino;
  g_shm->rank = -1;
  g_shm->nranks = 0;
  __atomic_store_n(&g_shm->magic, gpuexp::kRcclShmMagic, __ATOMIC_RELEASE);  // publish last
  return true;
}

int tool_init(rocprofiler_client_finalize_t, void*) {
  if (!open_shm()) return -1;
  if (rocprofiler_create_context(&g_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
  if (rocprofiler_configure_callback_tracing_service(g_ctx, ROCPROFILER_CALLBACK_TRACING_RCCL_API, nullptr, 0,
                                                     on_rccl, nullptr) != ROCPROFILER_STATUS_SUCCESS)
    return -1;
  return rocprofiler_start_context(g_ctx) == ROCPROFILER_STATUS_SUCCESS ? 0 : -1;
}

void tool_fini(void*) {
  if (g_shm) {
    ::munmap(g_shm, sizeof(RcclShmFile));
    g_shm = nullptr;
    if (!std::getenv("GPUEXP_RCCL_KEEP")) ::unlink(g_path.c_str());
  }
}

}  // namespace

// The rocprofiler-sdk this tool was compiled against (10000 * major + 100 * minor + patch).
// The RCCL domain id and the RCCL API argument layout it uses are that version's, so it
// loads only under a runtime of the same major version at or above it; an older (or the
// next major) runtime gets no configuration and the workload runs untraced instead of
// tracing whatever domain that id means there.  GPUEXP_RCCL_TRACER_ANY_SDK=1 overrides.
constexpr uint32_t kBuiltSdk = ROCPROFILER_VERSION_MAJOR * 10000 + ROCPROFILER_VERSION_MINOR * 100 + ROCPROFILER_VERSION_PATCH;

extern "C" __attribute__((visibility("default"))) uint32_t gpuexp_rccl_tracer_built_sdk_version() { return kBuiltSdk; }

extern "C" __attribute__((visibility("default"))) rocprofiler_tool_configure_result_t* rocprofiler_configure(
    uint32_t version, const char*, uint32_t, rocprofiler_client_id_t* id) {
  const char* any = std::getenv("GPUEXP_RCCL_TRACER_ANY_SDK");
  const bool ok = version / 10000 == kBuiltSdk / 10000 && version >= kBuiltSdk / 100 * 100;
  if (!ok && !(any && any[0] == '1')) {
    std::fprintf(stderr, "[gpuexp-rccl-tracer] rocprofiler-sdk %u.%u.%u is not the 1.%u+ this tracer was built for; "
                 "not loading (RCCL collectives of this process are not traced)\n",
                 version / 10000, version / 100 % 100, version % 100, kBuiltSdk / 100 % 100);
    return nullptr;
  }
  id->name = "gpuexp-rccl-tracer";
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                 &tool_fini, nullptr};
  return &cfg;
}
