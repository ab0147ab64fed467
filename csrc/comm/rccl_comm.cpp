// xflow-amd: native RCCL transport (see rccl_comm.h).
#include "rccl_comm.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace xflow {

namespace {

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

}  // namespace

std::vector<uint8_t> RcclComm::unique_id() {
  ncclUniqueId id;
  check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::vector<uint8_t> out(sizeof(id.internal));
  std::memcpy(out.data(), id.internal, sizeof(id.internal));
  return out;
}

RcclComm::RcclComm(const std::vector<uint8_t>& id, int world, int rank, int device)
    : world_(world), rank_(rank) {
  ncclUniqueId uid;
  if (id.size() != sizeof(uid.internal)) throw std::invalid_argument("RCCL unique id size");
  std::memcpy(uid.internal, id.data(), sizeof(uid.internal));
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  ncclComm_t c = nullptr;
  check(ncclCommInitRank(&c, world, uid, rank), "ncclCommInitRank");
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (comm_) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::abort() {
  if (comm_) {
    ncclCommAbort(static_cast<ncclComm_t>(comm_));
    comm_ = nullptr;
  }
}

void RcclComm::alltoallv(const void* send, const std::vector<int64_t>& send_counts, void* recv,
                         const std::vector<int64_t>& recv_counts, int elem_bytes,
                         uintptr_t stream) {
  alltoallv_group({A2AOp{send, send_counts, recv, recv_counts, elem_bytes}}, stream);
}

void RcclComm::alltoallv_group(const std::vector<A2AOp>& ops, uintptr_t stream) {
  if (!comm_) throw std::runtime_error("RCCL communicator was aborted");
  for (const A2AOp& op : ops) {
    if ((int)op.send_counts.size() != world_ || (int)op.recv_counts.size() != world_)
      throw std::invalid_argument("alltoallv: counts must have world entries");
    for (int p = 0; p < world_; ++p)
      if (op.send_counts[p] < 0 || op.recv_counts[p] < 0)
        throw std::invalid_argument("alltoallv: negative count");
  }
  ncclComm_t c = static_cast<ncclComm_t>(comm_);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  grouped([&] {
    for (const A2AOp& op : ops) {
      const char* s = static_cast<const char*>(op.send);
      char* r = static_cast<char*>(op.recv);
      size_t so = 0, ro = 0;
      for (int p = 0; p < world_; ++p) {
        const size_t sb = (size_t)op.send_counts[p] * op.elem_bytes;
        const size_t rb = (size_t)op.recv_counts[p] * op.elem_bytes;
        if (sb) check(ncclSend(s + so, sb, ncclUint8, p, c, st), "ncclSend");
        if (rb) check(ncclRecv(r + ro, rb, ncclUint8, p, c, st), "ncclRecv");
        so += sb;
        ro += rb;
      }
    }
  });
}

// ncclGroupStart, the calls, ncclGroupEnd -- and when a call inside fails,
// the group is still closed before the error propagates (an open group
// would swallow every later RCCL call of this thread into it)
template <typename F>
void RcclComm::grouped(F&& calls) {
  check(ncclGroupStart(), "ncclGroupStart");
  try {
    calls();
  } catch (...) {
    (void)ncclGroupEnd();
    throw;
  }
  check(ncclGroupEnd(), "ncclGroupEnd");
}

void RcclComm::send_recv(const std::vector<int>& peers, const std::vector<uintptr_t>& sends,
                         const std::vector<int64_t>& send_bytes,
                         const std::vector<uintptr_t>& recvs,
                         const std::vector<int64_t>& recv_bytes, uintptr_t stream) {
  if (!comm_) throw std::runtime_error("RCCL communicator was aborted");
  const size_t n = peers.size();
  if (sends.size() != n || send_bytes.size() != n || recvs.size() != n || recv_bytes.size() != n)
    throw std::invalid_argument("send_recv: list lengths differ");
  // (validated before the group opens: a throw must not leave it open)
  for (size_t i = 0; i < n; ++i)
    if (peers[i] < 0 || peers[i] >= world_ || send_bytes[i] < 0 || recv_bytes[i] < 0)
      throw std::invalid_argument("send_recv: bad peer or size");
  ncclComm_t c = static_cast<ncclComm_t>(comm_);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  grouped([&] {
    for (size_t i = 0; i < n; ++i) {
      if (send_bytes[i] > 0)
        check(ncclSend(reinterpret_cast<const void*>(sends[i]), (size_t)send_bytes[i], ncclUint8,
                       peers[i], c, st), "ncclSend");
      if (recv_bytes[i] > 0)
        check(ncclRecv(reinterpret_cast<void*>(recvs[i]), (size_t)recv_bytes[i], ncclUint8,
                       peers[i], c, st), "ncclRecv");
    }
  });
}

void RcclComm::alltoall(const void* send, void* recv, int64_t count, int elem_bytes,
                        uintptr_t stream) {
  std::vector<int64_t> cnt(world_, count);
  alltoallv(send, cnt, recv, cnt, elem_bytes, stream);
}

}  // namespace xflow
