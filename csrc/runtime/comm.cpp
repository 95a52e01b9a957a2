// RCCL communicator over xGMI (one process per GPU).
//
// Replaces the reference's implicit ProcessGroupNCCL/Gloo data plane (utils.py:5-14,
// SURVEY.md §2.2 N2): the Python layer bootstraps the rendezvous through the c10d
// TCPStore (rank 0 publishes the ncclUniqueId bytes), then every rank calls
// ncclCommInitRank here.  Collectives are enqueued on caller-provided HIP streams
// so they can be overlapped with compute and captured in hipGraphs.  Links
// against the RCCL that ships inside the torch wheel (one RCCL per process).
#include <atomic>
#include <cstring>

#include "runtime/runtime.h"

namespace ddp_amd {

static std::atomic<bool> g_exiting{false};
void mark_exiting() { g_exiting.store(true); }
bool process_exiting() { return g_exiting.load(); }

static ncclDataType_t to_nccl(int dtype) {
  switch (dtype) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclInt32;
    case 3: return ncclInt64;
    case 4: return ncclUint8;
  }
  throw std::runtime_error("unsupported dtype code " + std::to_string(dtype));
}

static ncclRedOp_t to_op(int op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclAvg;
    case 2: return ncclMax;
  }
  throw std::runtime_error("unsupported reduce op code " + std::to_string(op));
}

std::string Comm::new_unique_id() {
  ncclUniqueId id;
  DDP_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

Comm::Comm(const std::string& uid, int rank, int world, int device) : rank_(rank), world_(world) {
  if (uid.size() != sizeof(ncclUniqueId))
    throw std::runtime_error("bad ncclUniqueId size " + std::to_string(uid.size()));
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  DDP_HIP_CHECK(hipSetDevice(device));
  DDP_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
}

Comm::~Comm() {
  if (comm_ && !process_exiting()) {
    for (auto& kv : premul_) ncclRedOpDestroy(kv.second, comm_);
    ncclCommDestroy(comm_);
  }
}

void Comm::all_reduce_premul(float* buf, size_t count, float scale, hipStream_t s) {
  ncclRedOp_t op{};
  bool have = false;
  for (auto& kv : premul_)
    if (kv.first == scale) {
      op = kv.second;
      have = true;
    }
  if (!have) {
    // the scalar is captured by value (host-immediate), so the op stays valid inside
    // captured graphs; it lives as long as the communicator
    DDP_NCCL_CHECK(ncclRedOpCreatePreMulSum(&op, &scale, ncclFloat32, ncclScalarHostImmediate, comm_));
    premul_.emplace_back(scale, op);
  }
  DDP_NCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat32, op, comm_, s));
}

void Comm::all_reduce(void* buf, size_t count, int dtype, int op, hipStream_t s) {
  DDP_NCCL_CHECK(ncclAllReduce(buf, buf, count, to_nccl(dtype), to_op(op), comm_, s));
}

void Comm::broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) {
  DDP_NCCL_CHECK(ncclBroadcast(buf, buf, count, to_nccl(dtype), root, comm_, s));
}

void Comm::all_gather(const void* send, void* recv, size_t count, int dtype, hipStream_t s) {
  DDP_NCCL_CHECK(ncclAllGather(send, recv, count, to_nccl(dtype), comm_, s));
}

void Comm::reduce_scatter(const void* send, void* recv, size_t count, int dtype, int op,
                          hipStream_t s) {
  DDP_NCCL_CHECK(ncclReduceScatter(send, recv, count, to_nccl(dtype), to_op(op), comm_, s));
}

}  // namespace ddp_amd
