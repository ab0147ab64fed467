// xflow-amd: the lock-step sharded training step, orchestrated natively.
//
// The same step as xflow_amd/parallel/sparse_a2a.py ShardedEngine (its
// docstring has the phase list; the reference's Pull/Push call sites are
// lr_worker.cc:170/175 and the server handler ftrl.h:38-152), with the host
// side of a step -- split-size decoding, the all-to-all op lists, the RCCL
// group calls and the per-source applies -- in C++ on the engine's stream:
// Python makes one call per step.  Used on GPUs with the native RCCL
// communicator (and for the world-1 self-exchange); the torch.distributed
// transport (gloo on CPU) keeps the Python implementation, which these
// semantics mirror step for step (tests/test_native_sharded.py).
//
// Pipelining: train_step(batch, next) prepares `next` (dedup, owner counts,
// counts exchange into the other worker buffer set) in the middle of the
// current step and -- with early keys -- sends its keys inside the current
// step's gradient group call: two group calls per steady-state step.
#pragma once

#include <cstdint>
#include <deque>
#include <functional>
#include <vector>

#include "rccl_comm.h"
#include "xflow/engine.h"

namespace xflow {

class ShardedStep {
 public:
  // comm: null for world 1 (self-exchange aliased: the owner reads the send
  // buffers in place); otherwise the job's verified communicator.
  // staleness k > 0: the bounded-staleness step (xflow_amd/parallel/
  // async_p2p.py AsyncShardedEngine): a step's pushes are exchanged with the
  // keys of step t+k and applied after that step's pull.
  ShardedStep(Engine& e, RcclComm* comm, int world, int rank, bool early_keys,
              int staleness = 0);
  ~ShardedStep();
  ShardedStep(const ShardedStep&) = delete;
  ShardedStep& operator=(const ShardedStep&) = delete;

  // One step on batch `b` (identified by `id`, any value unique among the
  // caller's live batches).  next / next_id: the batch the next call will
  // train (prepared and, with early keys, its keys exchanged here), or null.
  // S: slices per step (identical on every rank).  Returns false, having
  // done nothing, when no rank had data for b.
  // prefetch (optional): called once the step's pull is queued -- device work
  // producing `next` (e.g. the synthetic generator), which its prepare follows
  bool train_step(const BatchView& b, int64_t id, int S, const BatchView* next, int64_t next_id,
                  const std::function<void()>& prefetch = nullptr);
  // Forward-only step (keys looked up, never inserted) writing pctr (may be
  // null when b has no rows); false when no rank had rows.
  bool eval_step(const BatchView& b, float* pctr);
  // staleness k: exchange and apply every pending push in step order (before
  // evaluation / checkpoints; every rank calls it)
  void flush();

  // host-side counters (see ShardedEngine): reads of split sizes whose copy
  // was still in flight at a step start / in the middle of a step, the host
  // seconds those waits took, steps whose next keys rode with the gradients,
  // steps that prepared their own batch, steps no rank had data for, bytes
  // sent + received, exchange buffers that grew (stream-ordered, no host wait)
  int64_t buffer_growths = 0;
  int64_t host_waits = 0, mid_step_waits = 0, early_key_exchanges = 0, inline_prepares = 0,
          empty_steps = 0, bytes_moved = 0, drop_exchanges = 0;
  double host_wait_s = 0.0;
  int64_t last_send = 0, last_recv = 0;
  int64_t p2p_ops = 0;  // staleness k: push exchanges so far
  // several slices on the CSR exchange: steps, and the host waits for the
  // per-owner entry totals (the entries' all-to-all sizes are known only
  // after the forward/backward)
  int64_t csr_exchanges = 0, csr_waits = 0;
  double csr_wait_s = 0.0;

 private:
  struct Buf {  // grow-only device buffer
    void* p = nullptr;
    size_t bytes = 0;
  };
  struct Split {
    int wb = 0;
    std::vector<int64_t> send, recv;
    bool any = false;
  };
  struct PendGroup {  // one slice group's pushes of a pending step
    float* gin;
    float* gout;
    u32* min;
    u32* mout;
    int S;
  };
  struct Pending {  // a staleness-k step whose pushes are not applied yet
    u64* rk = nullptr;
    std::vector<PendGroup> groups;
    std::vector<int64_t> send, recv, offsets;
    int buf = 0;
  };
  struct Ahead {  // a prepared batch whose keys were already received
    bool valid = false;
    int64_t id = 0;
    Split sp;
    int64_t n_send = 0, n_recv = 0;
    u64* keys = nullptr;
  };

  void* get(Buf& b, size_t bytes);
  bool self_only() const { return comm_ == nullptr; }
  void prepare(const BatchView& b, int64_t id, bool exchange);
  RcclComm::A2AOp counts_op(int wb);
  void counts_sent(int wb);
  Split take(const BatchView& b, int64_t id, bool mid_step,
             const std::function<void()>* prefetch = nullptr);
  void a2a_group(std::vector<RcclComm::A2AOp>& ops);
  void apply_groups(const u64* recv_keys, const std::vector<const float*>& grads,
                    const std::vector<const u32*>& masks, const std::vector<int>& group_S,
                    const std::vector<int64_t>& offsets, int buf = 0);
  bool train_step_async(const BatchView& b, int64_t id, int S, const BatchView* next,
                        int64_t next_id, const std::function<void()>& prefetch);
  void push_ops(const Pending& p, std::vector<RcclComm::A2AOp>& ops);
  void apply_pending(const Pending& p);
  static std::vector<int64_t> offsets_of(const std::vector<int64_t>& splits);
  uintptr_t stream() const;

  Engine& e_;
  RcclComm* comm_;
  int world_, rank_;
  bool early_keys_;
  int64_t* counts_both_[2] = {nullptr, nullptr};  // device [2*world]: send | recv counts
  u64* send_keys_[2] = {nullptr, nullptr};        // device [max_nnz]
  int64_t* counts_host_[2] = {nullptr, nullptr};  // pinned [2*world]
  void* counts_ready_[2] = {nullptr, nullptr};    // events behind the D2H copies
  Buf recv_keys_, vals_, pulled_, ahead_keys_[2];
  std::vector<Buf> grads_out_, grads_in_, masks_out_, masks_in_;
  int next_wb_ = 0, ahead_no_ = 0;
  int64_t seq_ = 0, prep_seq_[2] = {0, 0};
  bool prep_valid_ = false;
  int64_t prep_id_ = 0;
  int prep_wb_ = 0;
  Ahead ahead_;
  // staleness k (> 0): per step buffer (k + 1 of them) the received keys,
  // pulled values and per-group gradient / mask buffers, and the queue of
  // steps whose pushes are pending
  int staleness_ = 0;
  int64_t step_no_ = 0;
  std::vector<Buf> rk_, vals_k_;
  std::vector<std::vector<Buf>> gin_k_, gout_k_, min_k_, mout_k_;
  std::deque<Pending> pending_;
  // CSR exchange: per-key entry counts out / in, packed entries out / in,
  // per-owner totals (device [2 * world]: send | recv) and their pinned copy
  Buf csr_cnt_o_, csr_cnt_i_, csr_ent_o_, csr_ent_i_;
  int64_t* csr_tot_ = nullptr;
  int64_t* csr_tot_host_ = nullptr;
  void* csr_tot_ready_ = nullptr;
  // the gradient half of a CSR step (forward/backward, the two exchanges,
  // the per-source applies); ops holds the early next-keys op, if any
  void csr_gradients(const BatchView& b, int S, const Split& sp, const float* pulled,
                     int64_t n_send, int64_t n_recv, const u64* recv_keys,
                     const std::vector<int64_t>& offsets, const BatchView* next, int64_t next_id);
};

}  // namespace xflow
