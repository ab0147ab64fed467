// xflow-amd: native lock-step sharded step (see sharded_step.h).
#include "sharded_step.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>

namespace xflow {

ShardedStep::ShardedStep(Engine& e, RcclComm* comm, int world, int rank, bool early_keys,
                         int staleness)
    : e_(e), comm_(comm), world_(world), rank_(rank), early_keys_(early_keys),
      staleness_(staleness) {
  if (staleness < 0 || staleness > 3) throw std::invalid_argument("ShardedStep: staleness in [0, 3]");
  if (staleness > 0) {
    const int nbuf = staleness + 1;  // step t's buffers live until its apply at step t+k
    rk_.resize(nbuf);
    vals_k_.resize(nbuf);
    gin_k_.assign(nbuf, std::vector<Buf>(1));
    gout_k_.assign(nbuf, std::vector<Buf>(1));
    min_k_.assign(nbuf, std::vector<Buf>(1));
    mout_k_.assign(nbuf, std::vector<Buf>(1));
  }
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("ShardedStep: bad world/rank");
  if (!comm && world != 1)
    throw std::invalid_argument("ShardedStep: world > 1 needs a communicator");
  if (comm && (comm->world() != world || comm->rank() != rank))
    throw std::invalid_argument("ShardedStep: communicator world/rank mismatch");
  Backend& be = e_.backend();
  const int64_t nnz = e_.config().max_nnz > 0 ? e_.config().max_nnz : 1;
  for (int i = 0; i < 2; ++i) {
    counts_both_[i] = static_cast<int64_t*>(be.alloc(sizeof(int64_t) * 2 * world_));
    be.memset(counts_both_[i], 0, sizeof(int64_t) * 2 * world_);
    send_keys_[i] = static_cast<u64*>(be.alloc(sizeof(u64) * (size_t)nnz));
    counts_host_[i] = static_cast<int64_t*>(be.host_alloc(sizeof(int64_t) * 2 * world_));
    counts_ready_[i] = be.event_create();
  }
  grads_out_.resize(1);
  grads_in_.resize(1);
  masks_out_.resize(1);
  masks_in_.resize(1);
  csr_tot_ = static_cast<int64_t*>(be.alloc(sizeof(int64_t) * 2 * world_));
  csr_tot_host_ = static_cast<int64_t*>(be.host_alloc(sizeof(int64_t) * 2 * world_));
  csr_tot_ready_ = be.event_create();
}

ShardedStep::~ShardedStep() {
  Backend& be = e_.backend();
  be.synchronize();
  for (int i = 0; i < 2; ++i) {
    be.free(counts_both_[i]);
    be.free(send_keys_[i]);
    be.host_free(counts_host_[i]);
    be.event_destroy(counts_ready_[i]);
  }
  be.free(csr_tot_);
  be.host_free(csr_tot_host_);
  be.event_destroy(csr_tot_ready_);
  std::vector<Buf*> all = {&recv_keys_, &vals_, &pulled_, &ahead_keys_[0], &ahead_keys_[1],
                           &csr_cnt_o_, &csr_cnt_i_, &csr_ent_o_, &csr_ent_i_};
  for (auto* v : {&grads_out_, &grads_in_, &masks_out_, &masks_in_, &rk_, &vals_k_})
    for (Buf& b : *v) all.push_back(&b);
  for (auto* vv : {&gin_k_, &gout_k_, &min_k_, &mout_k_})
    for (auto& v : *vv)
      for (Buf& b : v) all.push_back(&b);
  for (Buf* b : all)
    if (b->p) be.free_stream(b->p);
  be.synchronize();
}

void* ShardedStep::get(Buf& b, size_t bytes) {
  if (bytes < 256) bytes = 256;
  if (b.bytes < bytes) {
    // Stream-ordered: the old buffer is released behind the queued work that
    // still reads it, the new one is usable by the work queued next -- a
    // buffer that grows mid-step costs no host wait (no device synchronize)
    Backend& be = e_.backend();
    if (b.p) be.free_stream(b.p);
    const size_t n = bytes + bytes / 4 + 4096;
    b.p = be.alloc_stream(n);
    b.bytes = n;
    ++buffer_growths;
  }
  return b.p;
}

uintptr_t ShardedStep::stream() const {
  return reinterpret_cast<uintptr_t>(e_.backend().stream());
}

std::vector<int64_t> ShardedStep::offsets_of(const std::vector<int64_t>& splits) {
  std::vector<int64_t> o(1, 0);
  for (int64_t c : splits) o.push_back(o.back() + c);
  return o;
}

void ShardedStep::a2a_group(std::vector<RcclComm::A2AOp>& ops) {
  if (ops.empty()) return;
  if (drop_exchanges > 0) {  // injected fault: this rank misses a collective
    --drop_exchanges;
    return;
  }
  if (self_only()) {
    for (const auto& op : ops) {
      const size_t bytes = (size_t)op.send_counts[0] * op.elem_bytes;
      if (op.recv != op.send && bytes) e_.backend().copy_d2d(op.recv, op.send, bytes);
    }
    return;
  }
  comm_->alltoallv_group(ops, stream());
}

RcclComm::A2AOp ShardedStep::counts_op(int wb) {
  RcclComm::A2AOp op;
  op.send = counts_both_[wb];
  op.recv = counts_both_[wb] + world_;
  op.send_counts.assign(world_, 1);
  op.recv_counts.assign(world_, 1);
  op.elem_bytes = sizeof(int64_t);
  return op;
}

void ShardedStep::counts_sent(int wb) {
  // the split sizes come back through pinned memory right behind the counts
  // exchange; read by the step that uses this batch
  e_.download_small(counts_host_[wb], counts_both_[wb], sizeof(int64_t) * 2 * world_);
  e_.backend().event_record(counts_ready_[wb]);
}

void ShardedStep::prepare(const BatchView& b, int64_t id, bool exchange) {
  const int wb = next_wb_;
  next_wb_ ^= 1;
  ++seq_;  // (prepares are collective: every rank counts alike)
  e_.w_prepare(b, world_, counts_both_[wb], send_keys_[wb], wb, world_ > 1 ? seq_ : -1);
  prep_seq_[wb] = seq_;
  prep_valid_ = true;
  prep_id_ = id;
  prep_wb_ = wb;
  if (self_only()) {
    counts_sent(wb);  // (receive counts = send counts)
  } else if (exchange) {
    std::vector<RcclComm::A2AOp> ops{counts_op(wb)};
    a2a_group(ops);
    counts_sent(wb);
  }
}

ShardedStep::Split ShardedStep::take(const BatchView& b, int64_t id, bool mid_step,
                                     const std::function<void()>* prefetch) {
  if (!prep_valid_ || prep_id_ != id) {
    ++inline_prepares;
    prepare(b, id, true);
    if (prefetch && *prefetch) {  // device work to overlap the split-size round trip
      (*prefetch)();
      prefetch = nullptr;
    }
  }
  prep_valid_ = false;
  Split sp;
  sp.wb = prep_wb_;
  const int W = world_;
  Backend& be = e_.backend();
  if (!be.event_done(counts_ready_[sp.wb])) {
    ++(mid_step ? mid_step_waits : host_waits);
    const auto t0 = std::chrono::steady_clock::now();
    be.event_spin(counts_ready_[sp.wb]);
    host_wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  std::vector<int64_t> both(2 * W);
  std::memcpy(both.data(), counts_host_[sp.wb], sizeof(int64_t) * 2 * W);
  std::vector<int64_t> send(both.begin(), both.begin() + W);
  std::vector<int64_t> recv = self_only() ? send : std::vector<int64_t>(both.begin() + W, both.end());
  if (W > 1) {
    // (count + 1, sender's prepare number): a peer that skipped an exchange
    // shows up as a different number -- fail now, not later
    const int64_t mask = (1ll << kCountBits) - 1, want = prep_seq_[sp.wb] & kSeqMask;
    for (int64_t c : recv) {
      if ((c >> kCountBits) != want) {
        std::string got;
        for (int64_t x : recv) got += std::to_string(x >> kCountBits) + " ";
        throw std::runtime_error("rank " + std::to_string(rank_) +
                                 ": counts exchange out of step (expected prepare " +
                                 std::to_string(want) + ", peers sent " + got +
                                 "): a rank skipped or repeated a collective");
      }
    }
    for (int64_t& c : send) c = (c & mask) - 1;
    for (int64_t& c : recv) c = (c & mask) - 1;
  }
  sp.any = false;
  for (int64_t c : recv) sp.any |= c >= 0;
  sp.send.resize(W);
  sp.recv.resize(W);
  last_send = last_recv = 0;
  for (int i = 0; i < W; ++i) {
    sp.send[i] = send[i] > 0 ? send[i] : 0;
    sp.recv[i] = recv[i] > 0 ? recv[i] : 0;
    last_send += sp.send[i];
    last_recv += sp.recv[i];
  }
  return sp;
}

void ShardedStep::apply_groups(const u64* recv_keys, const std::vector<const float*>& grads,
                               const std::vector<const u32*>& masks, const std::vector<int>& group_S,
                               const std::vector<int64_t>& offsets, int buf) {
  if (grads.size() == 1) {
    e_.s_apply(recv_keys, grads[0], masks[0], offsets, group_S[0], buf);
    return;
  }
  // several slice groups: the pushes go in (source, slice) order -- source by
  // source, each source's groups in order (ShardedEngine._apply_groups)
  const int W = (int)offsets.size() - 1;
  for (int src = 0; src < W; ++src) {
    if (offsets[src + 1] <= offsets[src]) continue;
    std::vector<int64_t> offs(W + 1);
    for (int i = 0; i <= W; ++i) offs[i] = i <= src ? offsets[src] : offsets[src + 1];
    for (size_t g = 0; g < grads.size(); ++g)
      e_.s_apply(recv_keys, grads[g], masks[g], offs, group_S[g], buf);
  }
}

bool ShardedStep::train_step(const BatchView& b, int64_t id, int S, const BatchView* next,
                             int64_t next_id, const std::function<void()>& prefetch) {
  if (staleness_ > 0) return train_step_async(b, id, S, next, next_id, prefetch);
  bool prefetched = false;
  const int ps = e_.value_width();
  const bool ordered_masks = S > 1 && !e_.config().sum_slices;
  const Ahead ah = ahead_;
  ahead_.valid = false;
  Split sp;
  const bool was_ahead = ah.valid && ah.id == id;
  if (was_ahead) {  // prepared AND its keys received during the previous step
    sp = ah.sp;
    last_send = ah.n_send;
    last_recv = ah.n_recv;
  } else {
    const bool inline_prep = !prep_valid_ || prep_id_ != id;
    sp = take(b, id, false, &prefetch);
    prefetched = inline_prep && prefetch;
  }
  if (!sp.any) {
    ++empty_steps;
    return false;
  }
  const int64_t n_send = last_send, n_recv = last_recv;
  const u64* recv_keys;
  if (was_ahead) {
    recv_keys = ah.keys;
  } else if (self_only()) {  // world 1: the owner reads the send buffer in place
    recv_keys = send_keys_[sp.wb];
  } else {
    u64* rk = static_cast<u64*>(get(recv_keys_, sizeof(u64) * (size_t)n_recv));
    std::vector<RcclComm::A2AOp> ops(1);
    ops[0] = {send_keys_[sp.wb], sp.send, rk, sp.recv, (int)sizeof(u64)};
    a2a_group(ops);
    recv_keys = rk;
  }
  const std::vector<int64_t> offsets = offsets_of(sp.recv);
  const int ngroups = Engine::slice_groups(S);
  float* vals = static_cast<float*>(get(vals_, sizeof(float) * (size_t)(n_recv * ps)));
  // the CSR exchange applies source by source (s_apply_csr): no owner
  // grouping, and compact FM rows of a later source expand with the pulled
  // weights, not the table's (the earlier sources updated it)
  const bool csr = e_.csr_slog2(S) >= 0 && e_.backend().csr_exchange();
  if (csr)
    e_.s_pull(recv_keys, n_recv, vals, true, 0, {}, true);
  else
    e_.s_pull(recv_keys, n_recv, vals, true, 0, offsets, ngroups > 1);
  if (prefetch && !prefetched) prefetch();
  const bool alias = self_only();
  float* pulled = alias ? vals : static_cast<float*>(get(pulled_, sizeof(float) * (size_t)(n_send * ps)));
  std::vector<RcclComm::A2AOp> ops;
  if (!alias) ops.push_back({vals, sp.recv, pulled, sp.send, (int)sizeof(float) * ps});
  if (next) {
    // the next batch's counts travel in the same group call as the values
    prepare(*next, next_id, false);
    if (!alias) ops.push_back(counts_op(prep_wb_));
  }
  a2a_group(ops);
  if (next && !alias) counts_sent(prep_wb_);

  if (csr) {
    // several slices as CSR entries: only the touched (key, slice) pairs move
    csr_gradients(b, S, sp, pulled, n_send, n_recv, recv_keys, offsets, next, next_id);
    e_.w_finish();
    return true;
  }
  // one gradient exchange per step; a step of more than 32 slices sends one
  // (gradients, masks) pair per slice group in it
  const int gw = e_.grad_width();
  for (auto* v : {&grads_out_, &grads_in_, &masks_out_, &masks_in_})
    if ((int)v->size() < ngroups) v->resize(ngroups);
  std::vector<const float*> gin;
  std::vector<const u32*> min_;
  std::vector<int> gS;
  ops.clear();
  for (int k = 0; k < ngroups; ++k) {
    const int Sg = Engine::group_slices(S, k);
    const int Wd = Sg * gw;
    const bool om = ordered_masks && Sg > 1;
    float* go = static_cast<float*>(get(grads_out_[k], sizeof(float) * (size_t)(n_send * Wd)));
    u32* mo = om ? static_cast<u32*>(get(masks_out_[k], sizeof(u32) * (size_t)n_send)) : nullptr;
    e_.w_forward_backward(b, pulled, n_send, go, mo, S, sp.wb, k);
    gS.push_back(Sg);
    if (alias) {
      gin.push_back(go);
      min_.push_back(mo);
      continue;
    }
    float* gi = static_cast<float*>(get(grads_in_[k], sizeof(float) * (size_t)(n_recv * Wd)));
    u32* mi = om ? static_cast<u32*>(get(masks_in_[k], sizeof(u32) * (size_t)n_recv)) : nullptr;
    gin.push_back(gi);
    min_.push_back(mi);
    ops.push_back({go, sp.send, gi, sp.recv, (int)sizeof(float) * Wd});
    if (om) ops.push_back({mo, sp.send, mi, sp.recv, (int)sizeof(u32)});  // same group call
  }
  if (!alias) {
    if (next && early_keys_) {
      // the next batch's keys ride in this group call: its split sizes came
      // with the values exchange above, so the host reads them now -- while
      // the device still runs this step's forward/backward
      Split s2 = take(*next, next_id, true);
      const int64_t n2s = last_send, n2r = last_recv;
      ahead_no_ ^= 1;
      u64* rk2 = static_cast<u64*>(get(ahead_keys_[ahead_no_], sizeof(u64) * (size_t)n2r));
      ops.push_back({send_keys_[s2.wb], s2.send, rk2, s2.recv, (int)sizeof(u64)});
      ahead_.valid = true;
      ahead_.id = next_id;
      ahead_.sp = s2;
      ahead_.n_send = n2s;
      ahead_.n_recv = n2r;
      ahead_.keys = rk2;
      ++early_key_exchanges;
      last_send = n_send;
      last_recv = n_recv;
    }
    a2a_group(ops);
  }
  apply_groups(recv_keys, gin, min_, gS, offsets);
  e_.w_finish();
  bytes_moved += (n_send + n_recv) * (8 + 4 * ps + 4 * (int64_t)S * gw);
  return true;
}

// Gradients of a step of several slices as CSR entries (Engine::
// w_forward_backward_csr): the reference's per-slice pushes carry only the
// keys the slice touched (lr_worker.cc:162-175), so instead of a dense
// [n_send][S x width] block per slice group only the (key, slice) pairs that
// exist move.  The entries' all-to-all sizes depend on the forward/backward,
// so the exchange takes two group calls: (entry counts per key + entry
// totals per owner [+ the next batch's keys]) then, once the host has read
// the totals, the entries; owners apply source by source from the entries.
void ShardedStep::csr_gradients(const BatchView& b, int S, const Split& sp, const float* pulled,
                                int64_t n_send, int64_t n_recv, const u64* recv_keys,
                                const std::vector<int64_t>& offsets, const BatchView* next,
                                int64_t next_id) {
  const int W = world_;
  const bool alias = self_only();
  ++csr_exchanges;
  if (alias) {  // world 1: the owner reads the worker's entries in place
    e_.w_forward_backward_csr(b, pulled, n_send, S, sp.wb, false, nullptr, nullptr, nullptr, 1,
                              false, nullptr);
    e_.s_apply_csr(recv_keys, nullptr, nullptr, offsets, S);
    // (the logical exchange: keys, values, entry counts -- the entries'
    // count stays on the device here)
    bytes_moved += (n_send + n_recv) * (8 + 4 * e_.value_width() + 4);
    return;
  }
  const int eb = e_.csr_entry_bytes();
  // entries <= (key, slice) pairs <= occurrences
  const int64_t emax = std::min<int64_t>(b.nnz, n_send * (int64_t)S);
  u32* cnt_o = static_cast<u32*>(get(csr_cnt_o_, sizeof(u32) * (size_t)n_send));
  void* ent_o = get(csr_ent_o_, (size_t)eb * (size_t)(emax > 0 ? emax : 1));
  e_.w_forward_backward_csr(b, pulled, n_send, S, sp.wb, true, cnt_o, ent_o, counts_both_[sp.wb],
                            W, W > 1, csr_tot_);
  u32* cnt_i = static_cast<u32*>(get(csr_cnt_i_, sizeof(u32) * (size_t)n_recv));
  std::vector<RcclComm::A2AOp> ops;
  ops.push_back({cnt_o, sp.send, cnt_i, sp.recv, (int)sizeof(u32)});
  RcclComm::A2AOp tot;
  tot.send = csr_tot_;
  tot.recv = csr_tot_ + W;
  tot.send_counts.assign(W, 1);
  tot.recv_counts.assign(W, 1);
  tot.elem_bytes = sizeof(int64_t);
  ops.push_back(tot);
  if (next && early_keys_) {
    // the next batch's keys ride in this group call (their split sizes came
    // with the values exchange)
    Split s2 = take(*next, next_id, true);
    const int64_t n2s = last_send, n2r = last_recv;
    ahead_no_ ^= 1;
    u64* rk2 = static_cast<u64*>(get(ahead_keys_[ahead_no_], sizeof(u64) * (size_t)n2r));
    ops.push_back({send_keys_[s2.wb], s2.send, rk2, s2.recv, (int)sizeof(u64)});
    ahead_.valid = true;
    ahead_.id = next_id;
    ahead_.sp = s2;
    ahead_.n_send = n2s;
    ahead_.n_recv = n2r;
    ahead_.keys = rk2;
    ++early_key_exchanges;
    last_send = n_send;
    last_recv = n_recv;
  }
  a2a_group(ops);
  Backend& be = e_.backend();
  e_.download_small(csr_tot_host_, csr_tot_, sizeof(int64_t) * 2 * W);
  be.event_record(csr_tot_ready_);
  if (!be.event_done(csr_tot_ready_)) {
    ++csr_waits;
    const auto t0 = std::chrono::steady_clock::now();
    be.event_spin(csr_tot_ready_);
    csr_wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  std::vector<int64_t> es(W), er(W);
  int64_t ein = 0, eout = 0;
  for (int r = 0; r < W; ++r) {
    es[r] = csr_tot_host_[r];
    er[r] = csr_tot_host_[W + r];
    if (es[r] < 0 || er[r] < 0) throw std::runtime_error("CSR exchange: negative entry totals");
    eout += es[r];
    ein += er[r];
  }
  if (eout > emax) throw std::runtime_error("CSR exchange: more entries than (key, slice) pairs");
  void* ent_i = get(csr_ent_i_, (size_t)eb * (size_t)(ein > 0 ? ein : 1));
  ops.clear();
  ops.push_back({ent_o, es, ent_i, er, eb});
  a2a_group(ops);
  e_.s_apply_csr(recv_keys, cnt_i, ent_i, offsets, S);
  bytes_moved += (n_send + n_recv) * (8 + 4 * e_.value_width() + 4) + (eout + ein) * eb +
                 16 * (int64_t)W;
}

void ShardedStep::push_ops(const Pending& p, std::vector<RcclComm::A2AOp>& ops) {
  // gradients (+ slice masks) to their owners: the reverse of the step's key
  // exchange, one pair per slice group
  const int gw = e_.grad_width();
  for (const PendGroup& g : p.groups) {
    ops.push_back({g.gout, p.send, g.gin, p.recv, (int)sizeof(float) * g.S * gw});
    if (g.min) ops.push_back({g.mout, p.send, g.min, p.recv, (int)sizeof(u32)});
  }
}

void ShardedStep::apply_pending(const Pending& p) {
  std::vector<const float*> g;
  std::vector<const u32*> m;
  std::vector<int> gs;
  for (const PendGroup& x : p.groups) {
    g.push_back(x.gin);
    m.push_back(x.min);
    gs.push_back(x.S);
  }
  apply_groups(p.rk, g, m, gs, p.offsets, p.buf);
}

// The staleness-k step (AsyncShardedEngine.train_step): step t-k's pushes
// ride in the group call of step t's keys and land after step t's pull.
bool ShardedStep::train_step_async(const BatchView& b, int64_t id, int S, const BatchView* next,
                                   int64_t next_id, const std::function<void()>& prefetch) {
  const int ps = e_.value_width(), gw = e_.grad_width();
  const bool ordered_masks = S > 1 && !e_.config().sum_slices;
  const bool inline_prep = !prep_valid_ || prep_id_ != id;
  Split sp = take(b, id, false, &prefetch);
  const bool prefetched = inline_prep && prefetch;
  if (!sp.any) {
    ++empty_steps;
    return false;
  }
  const int buf = (int)(step_no_ % (staleness_ + 1));
  const int64_t n_send = last_send, n_recv = last_recv;
  const bool alias = self_only();
  // this step's received keys stay alive until its pushes are applied
  u64* rk = static_cast<u64*>(get(rk_[buf], sizeof(u64) * (size_t)n_recv));
  std::vector<RcclComm::A2AOp> ops;
  ops.push_back({send_keys_[sp.wb], sp.send, rk, sp.recv, (int)sizeof(u64)});
  const bool due = (int)pending_.size() == staleness_;
  if (due && !alias) push_ops(pending_.front(), ops);  // step t-k's pushes ride with step t's keys
  a2a_group(ops);
  if (due) ++p2p_ops;
  const std::vector<int64_t> offsets = offsets_of(sp.recv);
  float* vals = static_cast<float*>(get(vals_k_[buf], sizeof(float) * (size_t)(n_recv * ps)));
  // (applied after the next k pulls: keep the pulled weights)
  e_.s_pull(rk, n_recv, vals, true, buf, offsets, true);
  if (prefetch && !prefetched) prefetch();
  float* pulled = alias ? vals : static_cast<float*>(get(pulled_, sizeof(float) * (size_t)(n_send * ps)));
  ops.clear();
  if (!alias) ops.push_back({vals, sp.recv, pulled, sp.send, (int)sizeof(float) * ps});
  if (next) {
    prepare(*next, next_id, false);
    if (!alias) ops.push_back(counts_op(prep_wb_));
  }
  a2a_group(ops);
  if (next && !alias) counts_sent(prep_wb_);
  // staleness k: step t-k's pushes land after this step's pull
  if (due) {
    apply_pending(pending_.front());
    pending_.pop_front();
  }
  const int ngroups = Engine::slice_groups(S);
  for (auto* vv : {&gin_k_, &gout_k_, &min_k_, &mout_k_})
    if ((int)(*vv)[buf].size() < ngroups) (*vv)[buf].resize(ngroups);
  Pending p;
  for (int k = 0; k < ngroups; ++k) {
    const int Sg = Engine::group_slices(S, k);
    const int Wd = Sg * gw;
    const bool om = ordered_masks && Sg > 1;
    float* go = static_cast<float*>(get(gout_k_[buf][k], sizeof(float) * (size_t)(n_send * Wd)));
    u32* mo = om ? static_cast<u32*>(get(mout_k_[buf][k], sizeof(u32) * (size_t)n_send)) : nullptr;
    e_.w_forward_backward(b, pulled, n_send, go, mo, S, sp.wb, k);
    float* gi = go;
    u32* mi = mo;
    if (!alias) {  // (world 1: the owner reads the pushes in place)
      gi = static_cast<float*>(get(gin_k_[buf][k], sizeof(float) * (size_t)(n_recv * Wd)));
      mi = om ? static_cast<u32*>(get(min_k_[buf][k], sizeof(u32) * (size_t)n_recv)) : nullptr;
    }
    p.groups.push_back({gi, go, mi, mo, Sg});
  }
  p.rk = rk;
  p.send = sp.send;
  p.recv = sp.recv;
  p.offsets = offsets;
  p.buf = buf;
  pending_.push_back(std::move(p));
  ++step_no_;
  e_.w_finish();
  bytes_moved += (n_send + n_recv) * (8 + 4 * ps + 4 * (int64_t)S * gw);
  return true;
}

void ShardedStep::flush() {
  while (!pending_.empty()) {
    if (!self_only()) {
      std::vector<RcclComm::A2AOp> ops;
      push_ops(pending_.front(), ops);
      a2a_group(ops);
    }
    ++p2p_ops;
    apply_pending(pending_.front());
    pending_.pop_front();
  }
}

bool ShardedStep::eval_step(const BatchView& b, float* pctr) {
  flush();
  // (keys exchanged ahead for a training batch no step will take now: every
  // rank drops them at the same point)
  ahead_.valid = false;
  prep_valid_ = false;
  Split sp = take(b, 0, false);
  if (!sp.any) return false;
  const int ps = e_.value_width();
  const u64* recv_keys;
  if (self_only()) {
    recv_keys = send_keys_[sp.wb];
  } else {
    u64* rk = static_cast<u64*>(get(recv_keys_, sizeof(u64) * (size_t)last_recv));
    std::vector<RcclComm::A2AOp> ops(1);
    ops[0] = {send_keys_[sp.wb], sp.send, rk, sp.recv, (int)sizeof(u64)};
    a2a_group(ops);
    recv_keys = rk;
  }
  float* vals = static_cast<float*>(get(vals_, sizeof(float) * (size_t)(last_recv * ps)));
  e_.s_pull(recv_keys, last_recv, vals, false, 0);
  float* pulled = static_cast<float*>(get(pulled_, sizeof(float) * (size_t)(last_send * ps)));
  std::vector<RcclComm::A2AOp> ops(1);
  ops[0] = {vals, sp.recv, pulled, sp.send, (int)sizeof(float) * ps};
  a2a_group(ops);
  e_.w_forward(b, pulled, last_send, b.rows ? pctr : nullptr, sp.wb);
  return true;
}

}  // namespace xflow
