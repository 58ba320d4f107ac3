// Native RCCL communicators for the collectives of the training step (DDP gradient buckets,
// sync-BN statistics / gradient sums).
//
// torch.distributed's ProcessGroupNCCL wraps every collective in a Work object whose end event
// its watchdog thread polls. On this stack a Work created while a stream is being captured into
// a hipGraph is still handed to the watchdog, and the watchdog's query of that captured event
// aborts the process ("operation not permitted on an event last recorded in a capturing
// stream", scripts/probe/capture_collectives_probe.py) as soon as a capture lasts longer than
// one poll interval — i.e. for any real training step. These entry points call RCCL directly
// on the caller's (current PyTorch) HIP stream: no Work objects, no events, no watchdog, so a
// step holding them captures and replays like any kernel sequence. The communicator is
// bootstrapped from the torch.distributed group (rank 0's unique id travels over it once, see
// parallel/rccl.py); hang detection for these collectives is the iteration watchdog of
// utils/health.py.
//
// Reference: the reference issues its collectives through torch DDP / torch SyncBatchNorm
// (utils/trainer.py:206-214, layers/activation_norm.py:403-410); it has no native
// communicator and runs no captured step.
#include "common.h"

#include <rccl/rccl.h>

#include <mutex>
#include <vector>

namespace iamd {
namespace {

std::mutex g_comm_mu;
std::vector<ncclComm_t> g_comms;

#define IAMD_NCCL_CHECK(expr)                                                        \
  do {                                                                               \
    ncclResult_t _r = (expr);                                                        \
    TORCH_CHECK(_r == ncclSuccess, "imaginaire_amd: RCCL error: ", ncclGetErrorString(_r), \
                " at ", __FILE__, ":", __LINE__);                                    \
  } while (0)

ncclComm_t comm_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_comm_mu);
  IAMD_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] != nullptr,
             "rccl: bad communicator handle ", h);
  return g_comms[h];
}

ncclDataType_t dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kDouble: return ncclFloat64;
    default: IAMD_CHECK(false, "rccl: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

}  // namespace

// 128-byte unique id (uint8 CPU tensor) created by rank 0 and shared over torch.distributed.
at::Tensor rccl_unique_id() {
  ncclUniqueId id;
  IAMD_NCCL_CHECK(ncclGetUniqueId(&id));
  auto t = at::empty({NCCL_UNIQUE_ID_BYTES}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), id.internal, NCCL_UNIQUE_ID_BYTES);
  return t;
}

// Joins the communicator named by ``uid`` on the current device; returns its handle.
int64_t rccl_comm_init(const at::Tensor& uid, int64_t rank, int64_t world) {
  IAMD_CHECK(uid.device().is_cpu() && uid.scalar_type() == at::kByte &&
                 uid.numel() == NCCL_UNIQUE_ID_BYTES,
             "rccl_comm_init: uid must be the 128-byte CPU tensor of rccl_unique_id()");
  IAMD_CHECK(world >= 1 && rank >= 0 && rank < world, "rccl_comm_init: bad rank / world");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.contiguous().data_ptr(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm;
  IAMD_NCCL_CHECK(ncclCommInitRank(&comm, (int)world, id, (int)rank));
  std::lock_guard<std::mutex> lk(g_comm_mu);
  g_comms.push_back(comm);
  return (int64_t)g_comms.size() - 1;
}

void rccl_comm_destroy(int64_t h) {
  ncclComm_t c = comm_of(h);
  IAMD_NCCL_CHECK(ncclCommDestroy(c));
  std::lock_guard<std::mutex> lk(g_comm_mu);
  g_comms[h] = nullptr;
}

// In-place all-reduce of a dense HIP tensor on the current stream. op: 0 sum, 1 average, 2 max.
void rccl_all_reduce(const at::Tensor& t, int64_t h, int64_t op) {
  IAMD_CHECK(t.is_cuda() && t.is_non_overlapping_and_dense(),
             "rccl_all_reduce: dense HIP tensor expected");
  const ncclRedOp_t rop = op == 1 ? ncclAvg : op == 2 ? ncclMax : ncclSum;
  IAMD_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), rop,
                                comm_of(h), stream()));
}

// out [world * n] <- every rank's ``in`` [n], rank-major, on the current stream.
void rccl_all_gather(const at::Tensor& out, const at::Tensor& in, int64_t h) {
  IAMD_CHECK(out.is_cuda() && in.is_cuda() && out.is_contiguous() && in.is_contiguous() &&
                 out.scalar_type() == in.scalar_type(),
             "rccl_all_gather: contiguous HIP tensors of one dtype expected");
  int world = 0;
  IAMD_NCCL_CHECK(ncclCommCount(comm_of(h), &world));
  IAMD_CHECK(out.numel() == (int64_t)world * in.numel(), "rccl_all_gather: out size");
  IAMD_NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), dtype_of(in),
                                comm_of(h), stream()));
}

}  // namespace iamd
