// Shared-memory layout written by the RCCL tracer tool library (libgpuexp_rccl_tracer.so,
// injected into workload pods via ROCP_TOOL_LIBRARIES) and read by the exporter.
//
// One file per traced process: <dir>/gpuexp-rccl-<pidns_ino>-<ns_pid>.  Cumulative
// per-op counters (atomically incremented by the tracer), so the exporter never loses
// records the way a drained ring could.  The writer records its PID-namespace inode and
// its in-namespace PID; the exporter (hostPID) maps that to a host PID through
// /proc/<pid>/ns/pid + NSpid — the same container-vs-host PID problem the reference
// never solved (/root/reference/main.go:101 vs :135).
#pragma once

#include <atomic>
#include <cstdint>

namespace gpuexp {

constexpr uint64_t kRcclShmMagic = 0x3158455550474d52ull;  // "RMGPUEX1"
constexpr int kRcclMaxOps = 16;

enum RcclOp : int {
  kOpAllReduce = 0,
  kOpAllGather,
  kOpReduceScatter,
  kOpAllToAll,
  kOpAllToAllv,
  kOpBroadcast,
  kOpReduce,
  kOpSend,
  kOpRecv,
  kOpGather,
  kOpScatter,
  kOpNumOps
};

inline const char* rccl_op_name(int op) {
  static const char* n[] = {"allreduce", "allgather", "reducescatter", "alltoall", "alltoallv", "broadcast",
                            "reduce",    "send",      "recv",          "gather",   "scatter"};
  return op >= 0 && op < kOpNumOps ? n[op] : "other";
}

struct RcclShmOp {
  std::atomic<uint64_t> calls;
  std::atomic<uint64_t> bytes;
};

struct RcclShmFile {
  uint64_t magic;
  uint32_t version;
  int32_t ns_pid;       // getpid() inside the writer's PID namespace
  uint64_t pidns_ino;   // inode of /proc/self/ns/pid of the writer
  int32_t rank;         // last seen communicator rank (-1 unknown)
  int32_t nranks;
  uint64_t pad[4];
  RcclShmOp ops[kRcclMaxOps];
};

}  // namespace gpuexp
