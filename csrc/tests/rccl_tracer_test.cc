// Drives the RCCL tracer's rocprofiler callback (csrc/gpuexp/rccl_tracer.cc) with synthetic
// API records — no GPU, no RCCL — and prints what landed in its shared-memory counters as
// JSON, so tests/test_rccl_tracer_bytes.py can pin every op's byte formula at any nranks.
//
// Built by that test with the rocprofiler-sdk headers only: the tool-registration symbols
// this TU references (rocprofiler_create_context, ...) are never called here and are left
// unresolved at link time (-Wl,--unresolved-symbols=ignore-in-object-files).
//
// usage: rccl_tracer_test <dir> <nranks> <myrank> <count>
#include "gpuexp/rccl_tracer.cc"  // same TU: on_rccl / open_shm are file-local

#include <cstdio>
#include <cstdlib>

namespace {

rocprofiler_callback_tracing_rccl_api_data_t g_data;

void fire(int op, rocprofiler_callback_phase_t phase) {
  rocprofiler_callback_tracing_record_t rec{};
  rec.kind = ROCPROFILER_CALLBACK_TRACING_RCCL_API;
  rec.operation = uint32_t(op);
  rec.phase = phase;
  rec.payload = &g_data;
  on_rccl(rec, nullptr, nullptr);
}

void call(int op) {  // one complete (ENTER, EXIT) API call with the current g_data
  fire(op, ROCPROFILER_CALLBACK_PHASE_ENTER);
  fire(op, ROCPROFILER_CALLBACK_PHASE_EXIT);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 5) {
    std::fprintf(stderr, "usage: %s <dir> <nranks> <myrank> <count>\n", argv[0]);
    return 2;
  }
  ::setenv("GPUEXP_RCCL_DIR", argv[1], 1);
  ::setenv("GPUEXP_RCCL_KEEP", "1", 1);
  const int nranks = std::atoi(argv[2]), myrank = std::atoi(argv[3]);
  const size_t count = std::strtoull(argv[4], nullptr, 10);
  if (!open_shm()) return 3;

  // The world communicator, created by ncclCommInitRank (its EXIT carries *newcomm).
  ncclComm_t world = reinterpret_cast<ncclComm_t>(uintptr_t(0x1000));
  g_data = {};
  g_data.size = sizeof(g_data);
  g_data.args.ncclCommInitRank.newcomm = &world;
  g_data.args.ncclCommInitRank.nranks = nranks;
  g_data.args.ncclCommInitRank.myrank = myrank;
  fire(ROCPROFILER_RCCL_API_ID_ncclCommInitRank, ROCPROFILER_CALLBACK_PHASE_ENTER);
  fire(ROCPROFILER_RCCL_API_ID_ncclCommInitRank, ROCPROFILER_CALLBACK_PHASE_EXIT);

  const ncclDataType_t bf16 = ncclBfloat16;
  auto& a = g_data.args;
  g_data = {};
  g_data.size = sizeof(g_data);
  a.ncclAllReduce = {nullptr, nullptr, count, bf16, ncclSum, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclAllReduce);
  a.ncclAllGather = {nullptr, nullptr, count, bf16, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclAllGather);
  a.ncclReduceScatter = {nullptr, nullptr, count, bf16, ncclSum, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclReduceScatter);
  // all-to-all: RCCL implements it with its own public ncclSend/ncclRecv inside a group;
  // the nested calls must not be counted again
  a.ncclAllToAll = {nullptr, nullptr, count, bf16, world, nullptr};
  fire(ROCPROFILER_RCCL_API_ID_ncclAllToAll, ROCPROFILER_CALLBACK_PHASE_ENTER);
  {
    rocprofiler_callback_tracing_rccl_api_data_t outer = g_data;
    for (int p = 0; p < nranks; ++p) {
      a.ncclSend = {nullptr, count, bf16, p, world, nullptr};
      call(ROCPROFILER_RCCL_API_ID_ncclSend);
      a.ncclRecv = {nullptr, count, bf16, p, world, nullptr};
      call(ROCPROFILER_RCCL_API_ID_ncclRecv);
    }
    g_data = outer;
  }
  fire(ROCPROFILER_RCCL_API_ID_ncclAllToAll, ROCPROFILER_CALLBACK_PHASE_EXIT);
  size_t counts[64];
  size_t displs[64];
  for (int p = 0; p < nranks && p < 64; ++p) {
    counts[p] = count + size_t(p);  // uneven split: sum = nranks*count + nranks(nranks-1)/2
    displs[p] = 0;
  }
  a.ncclAllToAllv = {nullptr, counts, displs, nullptr, counts, displs, bf16, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclAllToAllv);
  a.ncclBroadcast = {nullptr, nullptr, count, bf16, 0, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclBroadcast);
  a.ncclReduce = {nullptr, nullptr, count, bf16, ncclSum, 0, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclReduce);
  // PP: one send to the next stage, one recv from the previous; CP: 2 neighbours per hop
  a.ncclSend = {nullptr, count, bf16, (myrank + 1) % nranks, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclSend);
  a.ncclRecv = {nullptr, count, bf16, (myrank + nranks - 1) % nranks, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclRecv);
  a.ncclGather = {nullptr, nullptr, count, bf16, 0, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclGather);
  a.ncclScatter = {nullptr, nullptr, count, bf16, 0, world, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclScatter);
  // a communicator the tracer never saw created (e.g. from ncclCommSplit) and no librccl
  // in the process to ask: its size is unknown and counted as 1
  ncclComm_t unknown = reinterpret_cast<ncclComm_t>(uintptr_t(0x2000));
  a.ncclAllGather = {nullptr, nullptr, count, ncclFloat32, unknown, nullptr};
  call(ROCPROFILER_RCCL_API_ID_ncclAllGather);

  std::printf("{\"rank\": %d, \"nranks\": %d, \"ops\": {", g_shm->rank, g_shm->nranks);
  for (int op = 0; op < gpuexp::kOpNumOps; ++op)
    std::printf("%s\"%s\": [%llu, %llu]", op ? ", " : "", gpuexp::rccl_op_name(op),
                (unsigned long long)g_shm->ops[op].calls.load(), (unsigned long long)g_shm->ops[op].bytes.load());
  std::printf("}, \"path\": \"%s\"}\n", g_path.c_str());
  tool_fini(nullptr);
  return 0;
}
