// xflow-amd: native RCCL transport for the sharded sparse step.
//
// The sharded step's all-to-alls (xflow_amd/parallel/sparse_a2a.py) run
// through this communicator on the ENGINE'S stream: the exchange is ordered
// with the dedup / pull / forward kernels in one HIP queue instead of crossing
// to a process-group stream and back (a cross-queue event costs ~14 us per
// collective on MI355X, 4 collectives per step).  A variable-size all-to-all
// is one ncclGroupStart/End of per-peer ncclSend/ncclRecv, which RCCL maps
// onto the node's xGMI peer links.
//
// The unique id travels over the job's torch.distributed group; the library
// is the RCCL torch has already loaded (resolved by SONAME librccl.so.1).
// The header is HIP-free (opaque communicator, stream as an integer handle)
// so host-only translation units can include it.
#pragma once

#include <cstdint>
#include <vector>

namespace xflow {

class RcclComm {
 public:
  static std::vector<uint8_t> unique_id();
  RcclComm(const std::vector<uint8_t>& id, int world, int rank, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int world() const { return world_; }
  int rank() const { return rank_; }
  // variable splits (elements of elem_bytes), host-side counts, on `stream`
  void alltoallv(const void* send, const std::vector<int64_t>& send_counts, void* recv,
                 const std::vector<int64_t>& recv_counts, int elem_bytes, uintptr_t stream);
  // several variable all-to-alls with the same split counts in ONE group call
  // (one RCCL kernel): e.g. gradients + slice masks, values + next counts
  struct A2AOp {
    const void* send;
    std::vector<int64_t> send_counts;
    void* recv;
    std::vector<int64_t> recv_counts;
    int elem_bytes;
  };
  void alltoallv_group(const std::vector<A2AOp>& ops, uintptr_t stream);
  // grouped point-to-point: for each i, send send_bytes[i] bytes to peers[i]
  // and receive recv_bytes[i] bytes from it (0 = none); one group call
  void send_recv(const std::vector<int>& peers, const std::vector<uintptr_t>& sends,
                 const std::vector<int64_t>& send_bytes, const std::vector<uintptr_t>& recvs,
                 const std::vector<int64_t>& recv_bytes, uintptr_t stream);
  // equal splits: `count` elements to / from every peer
  void alltoall(const void* send, void* recv, int64_t count, int elem_bytes, uintptr_t stream);
  // abandon in-flight work (used when a self-test times out)
  void abort();

 private:
  template <typename F>
  void grouped(F&& calls);
  void* comm_ = nullptr;  // ncclComm_t
  int world_ = 1, rank_ = 0;
};

}  // namespace xflow
