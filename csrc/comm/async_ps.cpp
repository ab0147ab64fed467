// xflow-amd: asynchronous parameter server (see async_ps.h).
#include "async_ps.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <string>

namespace xflow {

namespace {

using Clock = std::chrono::steady_clock;

double since(Clock::time_point t0) {
  return std::chrono::duration<double>(Clock::now() - t0).count();
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// One sequence word plus its payload on its own cache line.  A writer stores
// the payload, then seq with release; a reader loads seq with acquire, then
// the payload.  Every cell has exactly one writing process.
struct alignas(64) Cell {
  std::atomic<int64_t> seq;
  int64_t a, b, c;
  char pad[32];
};
static_assert(sizeof(Cell) == 64, "control cell must be one cache line");
static_assert(std::atomic<int64_t>::is_always_lock_free, "cross-process atomics need lock-free int64");

constexpr int64_t kMagic = 0x78666c6f77617073ll;  // "xflowaps"
constexpr int kMaxWorld = 64;

}  // namespace

// Control segment: header, then per (source, owner, slot) request and push
// cells (written by the source), per (owner, source) response and applied
// cells (written by the owner), per rank progress cells (written by the rank).
struct AsyncPS::Ctl {
  struct Hdr {
    std::atomic<int64_t> magic;
    int64_t world, ring;
    std::atomic<int64_t> abort;  // 1 + the first failing rank (0: none)
    char pad[32];
  };
  Hdr* hdr = nullptr;
  Cell *req = nullptr, *push = nullptr, *resp = nullptr, *appl = nullptr, *prog = nullptr;
  int W = 1, R = 1;
  static size_t bytes(int W, int R) {
    return sizeof(Hdr) + sizeof(Cell) * ((size_t)2 * W * W * R + (size_t)2 * W * W + W);
  }
  void bind(void* p, int w, int r) {
    W = w;
    R = r;
    char* q = static_cast<char*>(p);
    hdr = reinterpret_cast<Hdr*>(q);
    Cell* c = reinterpret_cast<Cell*>(q + sizeof(Hdr));
    req = c;
    push = req + (size_t)W * W * R;
    resp = push + (size_t)W * W * R;
    appl = resp + (size_t)W * W;
    prog = appl + (size_t)W * W;
  }
  Cell& req_c(int s, int o, int slot) { return req[((size_t)s * W + o) * R + slot]; }
  Cell& push_c(int s, int o, int slot) { return push[((size_t)s * W + o) * R + slot]; }
  Cell& resp_c(int o, int s) { return resp[(size_t)o * W + s]; }
  Cell& appl_c(int o, int s) { return appl[(size_t)o * W + s]; }
  Cell& prog_c(int r) { return prog[r]; }
};

AsyncPS::AsyncPS(Engine& worker, Engine& server, const Config& c)
    : wk_(worker), sv_(server), c_(c), W_(c.world), R_(c.staleness + 1) {
  if (W_ < 1 || W_ > kMaxWorld || c_.rank < 0 || c_.rank >= W_)
    throw std::invalid_argument("AsyncPS: bad world / rank");
  if (c_.staleness < 0 || c_.staleness > 7) throw std::invalid_argument("AsyncPS: staleness in [0, 7]");
  if ((int64_t)W_ * R_ > Engine::kSrvBufs)
    throw std::invalid_argument("AsyncPS: world x (staleness + 1) must be <= " +
                                std::to_string(Engine::kSrvBufs) + " (server buffers)");
  if (c_.name.empty()) throw std::invalid_argument("AsyncPS: needs a job-unique name");
  if (&worker == &server) throw std::invalid_argument("AsyncPS: worker and server need two engines");
  if (worker.is_gpu() != server.is_gpu()) throw std::invalid_argument("AsyncPS: engines on different backends");
  if (c_.pair_frac <= 0.0 || c_.pair_frac > 1.0) throw std::invalid_argument("AsyncPS: pair_frac in (0, 1]");
  const int S = c_.slices;
  if (S < 1 || S > wk_.config().max_slices || S > sv_.config().max_slices)
    throw std::invalid_argument("AsyncPS: slices outside both engines' max_slices");
  csr_ = wk_.csr_slog2(S) >= 0 && wk_.backend().csr_exchange();
  if (!csr_ && Engine::slice_groups(S) > 1)
    throw std::invalid_argument("AsyncPS: more than 32 slices need the CSR gradients (GPU backend)");
  masks_ = !csr_ && S > 1 && !wk_.config().sum_slices;
  const ModelSpec& m = wk_.config().model;
  fm_keep_ = m.kind == kFM && m.fm_math == kFmReference;
  vw_ = wk_.value_width();
  gw_ = wk_.grad_width();
  eb_ = wk_.csr_entry_bytes();
  if (vw_ != sv_.value_width() || gw_ != sv_.grad_width() || csr_ != (sv_.csr_slog2(S) >= 0))
    throw std::invalid_argument("AsyncPS: worker and server engines disagree on the step layout");
  const int64_t nnz = std::max<int64_t>(1, wk_.config().max_nnz);
  ncap_ = nnz;
  kcap_ = std::max<int64_t>(1, (int64_t)std::ceil((double)nnz * c_.pair_frac));
  ecap_ = kcap_;
  keys_b_ = align256(8 * (size_t)kcap_);
  cnt_b_ = align256(4 * (size_t)kcap_);
  pay_b_ = csr_ ? align256((size_t)eb_ * ecap_) : align256(4 * (size_t)S * gw_ * kcap_);
  slot_b_ = keys_b_ + cnt_b_ + pay_b_;
  inbox_b_ = slot_b_ * (size_t)W_ * R_;
  resp_b_ = align256(4 * (size_t)vw_ * ncap_);
  const size_t win = inbox_b_ + resp_b_ * R_;
  if (c_.rank == 0) {
    ctl_seg_ = std::make_unique<ShmSegment>(c_.name + "_ctl", Ctl::bytes(W_, R_), true);
    ctl_ = new Ctl();
    ctl_->bind(ctl_seg_->data(), W_, R_);
    Ctl& k = *ctl_;
    k.hdr->world = W_;
    k.hdr->ring = R_;
    k.hdr->abort.store(0);
    for (size_t i = 0; i < (size_t)W_ * W_ * R_; ++i) {
      k.req[i].seq.store(-1);
      k.push[i].seq.store(-1);
    }
    for (size_t i = 0; i < (size_t)W_ * W_; ++i) {
      k.resp[i].seq.store(-1);
      k.appl[i].seq.store(-1);
    }
    for (int r = 0; r < W_; ++r) k.prog[r].seq.store(0);
    k.hdr->magic.store(kMagic, std::memory_order_release);
  }
  win_ = c_.device >= 0 ? make_ipc_window(win, W_, c_.rank, c_.device)
                        : make_shm_window(win, W_, c_.rank, c_.name);
  Backend& be = wk_.backend();
  counts_d_ = static_cast<int64_t*>(be.alloc(sizeof(int64_t) * W_));
  tot_d_ = static_cast<int64_t*>(be.alloc(sizeof(int64_t) * W_));
  counts_h_ = static_cast<int64_t*>(be.host_alloc(sizeof(int64_t) * W_));
  tot_h_ = static_cast<int64_t*>(be.host_alloc(sizeof(int64_t) * W_));
  keys_d_ = static_cast<u64*>(be.alloc(sizeof(u64) * (size_t)nnz));
  cnt_d_ = static_cast<u32*>(be.alloc(sizeof(u32) * (size_t)nnz));
  pay_d_ = be.alloc(csr_ ? (size_t)eb_ * nnz : 4 * (size_t)S * gw_ * nnz);
  wev_ = be.event_create();
  srv_stream_ = sv_.backend().stream();
  served_.assign(W_, -1);
  applied_.assign(W_, -1);
  kind_.assign((size_t)W_ * R_, 0);
  nkeys_.assign((size_t)W_ * R_, 0);
}

AsyncPS::~AsyncPS() {
  stop_.store(true);
  if (thr_.joinable()) thr_.join();
  Backend& be = wk_.backend();
  be.synchronize();
  be.free(counts_d_);
  be.free(tot_d_);
  be.free(keys_d_);
  be.free(cnt_d_);
  be.free(pay_d_);
  be.host_free(counts_h_);
  be.host_free(tot_h_);
  be.event_destroy(wev_);
  delete ctl_;
}

void AsyncPS::connect(const std::vector<std::vector<uint8_t>>& handles) {
  if (connected_) return;
  if (!ctl_) {
    ctl_seg_ = std::make_unique<ShmSegment>(c_.name + "_ctl", Ctl::bytes(W_, R_), false);
    ctl_ = new Ctl();
    ctl_->bind(ctl_seg_->data(), W_, R_);
    if (ctl_->hdr->magic.load(std::memory_order_acquire) != kMagic || ctl_->hdr->world != W_ ||
        ctl_->hdr->ring != R_)
      throw std::runtime_error("AsyncPS: control segment of another job (world / staleness differ)");
  }
  win_->open(handles);
  connected_ = true;
}

void AsyncPS::start() {
  if (!connected_) throw std::logic_error("AsyncPS: connect() before start()");
  if (running_.load()) return;
  check_abort();
  // (the caller may have used the server engine on its own stream meanwhile)
  sv_.backend().set_stream(srv_stream_);
  stop_.store(false);
  running_.store(true);
  thr_ = std::thread([this] { server_loop(); });
}

void AsyncPS::stop() {
  stop_.store(true);
  if (thr_.joinable()) thr_.join();
  running_.store(false);
  check_abort();
}

std::vector<int64_t> AsyncPS::log() const {
  std::lock_guard<std::mutex> g(log_mu_);
  return log_;
}

void AsyncPS::fail(const std::string& msg) {
  {
    std::lock_guard<std::mutex> g(log_mu_);  // (the server thread fails too)
    if (err_.empty()) err_ = msg;
  }
  if (ctl_) {
    int64_t z = 0;
    ctl_->hdr->abort.compare_exchange_strong(z, 1 + c_.rank);
  }
}

void AsyncPS::check_abort() const {
  std::string e;
  {
    std::lock_guard<std::mutex> g(log_mu_);
    e = err_;
  }
  if (!e.empty()) throw std::runtime_error("AsyncPS (rank " + std::to_string(c_.rank) + "): " + e);
  const int64_t a = ctl_ ? ctl_->hdr->abort.load(std::memory_order_relaxed) : 0;
  if (a) throw std::runtime_error("AsyncPS: rank " + std::to_string(a - 1) + " failed");
}

template <typename Pred>
void AsyncPS::wait_until(Pred p, const char* what, double* acc) {
  if (p()) return;
  const auto t0 = Clock::now();
  for (int64_t spin = 0; !p(); ++spin) {
    if (spin < 256) {
      std::this_thread::yield();
      continue;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(spin < 4096 ? 5 : 50));
    if ((spin & 255) == 0) {
      check_abort();
      if (since(t0) > c_.timeout_s) {
        fail(std::string("timed out waiting for ") + what);
        check_abort();
      }
    }
  }
  if (acc) *acc += since(t0);
}

void AsyncPS::wait_event(void* ev) {
  const auto t0 = Clock::now();
  Backend& be = wk_.backend();
  be.event_record(ev);
  be.event_spin(ev);
  sync_s += since(t0);
}

u64* AsyncPS::in_keys(void* win, int s, int slot) const {
  return reinterpret_cast<u64*>(static_cast<char*>(win) + slot_b_ * ((size_t)s * R_ + slot));
}
u32* AsyncPS::in_cnt(void* win, int s, int slot) const {
  return reinterpret_cast<u32*>(reinterpret_cast<char*>(in_keys(win, s, slot)) + keys_b_);
}
void* AsyncPS::in_pay(void* win, int s, int slot) const {
  return reinterpret_cast<char*>(in_keys(win, s, slot)) + keys_b_ + cnt_b_;
}
float* AsyncPS::resp(void* win, int slot) const {
  return reinterpret_cast<float*>(static_cast<char*>(win) + inbox_b_ + resp_b_ * slot);
}

bool AsyncPS::train_step(const BatchView& b) { return step(b, nullptr, true); }

bool AsyncPS::eval_step(const BatchView& b, float* pctr) { return step(b, pctr, false); }

// One worker step (lr_worker.cc:145-177 per slice: keys -> Pull -> forward /
// backward -> Push), with every transfer a direct write into the peer's
// window and every hand-over a sequence word.
bool AsyncPS::step(const BatchView& b, float* pctr, bool train) {
  if (!running_.load()) throw std::logic_error("AsyncPS: start() before stepping");
  check_abort();
  if (b.rows == 0) return false;
  if (train && c_.slow_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(c_.slow_ms));
  const int me = c_.rank, S = c_.slices;
  const int64_t t = seq_;
  const int slot = (int)(t % R_);
  Ctl& k = *ctl_;
  Backend& be = wk_.backend();
  if (train && __atomic_load_n(&k.prog_c(me).a, __ATOMIC_RELAXED))
    __atomic_store_n(&k.prog_c(me).a, 0, __ATOMIC_RELEASE);  // (training again after finish)
  // 1. bounded staleness / slot reuse: every owner applied (or retired) step t - R
  wait_until(
      [&] {
        for (int o = 0; o < W_; ++o)
          if (k.appl_c(o, me).seq.load(std::memory_order_acquire) < t - R_) return false;
        return true;
      },
      "the owners to apply this worker's earlier pushes", &wait_slot_s);
  if (train) {
    int64_t lo = INT64_MAX;
    for (int o = 0; o < W_; ++o) lo = std::min(lo, k.appl_c(o, me).seq.load(std::memory_order_acquire));
    max_staleness = std::max<int64_t>(max_staleness, t - 1 - lo);
    int64_t slow = INT64_MAX;
    for (int r = 0; r < W_; ++r)
      if (!__atomic_load_n(&k.prog_c(r).a, __ATOMIC_ACQUIRE)) slow = std::min(slow, k.prog_c(r).seq.load(std::memory_order_relaxed));
    if (slow != INT64_MAX) max_lead = std::max<int64_t>(max_lead, steps - slow);
  }
  // 2. dedup + owner grouping (send order = owner order)
  wk_.w_prepare(b, W_, counts_d_, keys_d_, 0, -1);
  be.download_small(counts_h_, counts_d_, sizeof(int64_t) * W_);
  wait_event(wev_);
  std::vector<int64_t> n(W_), off(W_ + 1, 0);
  for (int o = 0; o < W_; ++o) {
    n[o] = std::max<int64_t>(0, counts_h_[o]);
    if (n[o] > kcap_)
      fail("step " + std::to_string(t) + ": " + std::to_string(n[o]) + " keys for owner " +
           std::to_string(o) + " exceed the inbox (" + std::to_string(kcap_) + "; raise pair_frac)");
    off[o + 1] = off[o] + n[o];
  }
  check_abort();
  const int64_t n_send = off[W_];
  // 3. keys into the owners' inboxes, then the requests
  for (int o = 0; o < W_; ++o)
    if (n[o]) be.copy_d2d(in_keys(win_->peer(o), me, slot), keys_d_ + off[o], sizeof(u64) * n[o]);
  wait_event(wev_);
  for (int o = 0; o < W_; ++o) {
    Cell& c = k.req_c(me, o, slot);
    c.a = n[o];
    c.b = off[o];
    c.c = train ? 0 : 1;
    c.seq.store(t, std::memory_order_release);
  }
  // 4. the owners' pull kernels write the values into this rank's response slot
  wait_until(
      [&] {
        for (int o = 0; o < W_; ++o)
          if (k.resp_c(o, me).seq.load(std::memory_order_acquire) < t) return false;
        return true;
      },
      "pull responses", &wait_pull_s);
  const float* pulled = resp(win_->local(), slot);
  if (!train) {
    wk_.w_forward(b, pulled, n_send, pctr, 0);
    wk_.w_finish();
    ++seq_;
    ++evals;
    return true;
  }
  // 5. forward / backward, gradients into the owners' inboxes, then the pushes
  std::vector<int64_t> e(W_, 0);
  int64_t moved = 0;
  if (csr_) {
    wk_.w_forward_backward_csr(b, pulled, n_send, S, 0, true, cnt_d_, pay_d_, counts_d_, W_, false,
                               tot_d_);
    be.download_small(tot_h_, tot_d_, sizeof(int64_t) * W_);
    wait_event(wev_);
    int64_t eo = 0;
    for (int o = 0; o < W_; ++o) {
      e[o] = tot_h_[o];
      if (e[o] < 0 || e[o] > ecap_)
        fail("step " + std::to_string(t) + ": " + std::to_string(e[o]) +
             " gradient entries for owner " + std::to_string(o) + " exceed the inbox");
    }
    check_abort();
    for (int o = 0; o < W_; ++o) {
      if (n[o]) be.copy_d2d(in_cnt(win_->peer(o), me, slot), cnt_d_ + off[o], sizeof(u32) * n[o]);
      if (e[o])
        be.copy_d2d(in_pay(win_->peer(o), me, slot), static_cast<char*>(pay_d_) + (size_t)eb_ * eo,
                    (size_t)eb_ * e[o]);
      eo += e[o];
      moved += 4 * n[o] + (int64_t)eb_ * e[o];
    }
  } else {
    const int row = S * gw_;
    wk_.w_forward_backward(b, pulled, n_send, static_cast<float*>(pay_d_), masks_ ? cnt_d_ : nullptr,
                           S, 0, 0);
    for (int o = 0; o < W_; ++o) {
      e[o] = n[o];
      if (!n[o]) continue;
      be.copy_d2d(in_pay(win_->peer(o), me, slot), static_cast<float*>(pay_d_) + off[o] * row,
                  sizeof(float) * row * n[o]);
      if (masks_) be.copy_d2d(in_cnt(win_->peer(o), me, slot), cnt_d_ + off[o], sizeof(u32) * n[o]);
      moved += (4 * (int64_t)row + (masks_ ? 4 : 0)) * n[o];
    }
  }
  wait_event(wev_);
  for (int o = 0; o < W_; ++o) {
    Cell& c = k.push_c(me, o, slot);
    c.a = e[o];
    c.seq.store(t, std::memory_order_release);
  }
  wk_.w_finish();
  bytes_moved += moved + n_send * (8 + 4 * (int64_t)vw_);
  ++seq_;
  ++steps;
  k.prog_c(me).seq.store(steps, std::memory_order_release);
  return true;
}

void AsyncPS::finish() {
  if (!running_.load()) return;
  const int me = c_.rank;
  Ctl& k = *ctl_;
  const int64_t last = seq_ - 1;
  wait_until(
      [&] {
        for (int o = 0; o < W_; ++o)
          if (k.appl_c(o, me).seq.load(std::memory_order_acquire) < last) return false;
        return true;
      },
      "the owners to apply this worker's last pushes", &wait_slot_s);
  __atomic_store_n(&k.prog_c(me).a, 1, __ATOMIC_RELEASE);
}

// The server thread: a ps-lite KVServer for this rank's shard.  Requests of
// every source are taken in arrival order (each source's in step order), a
// push only after its own pull; completions are published in stream order.
void AsyncPS::server_loop() {
  try {
    Backend& be = sv_.backend();
    be.bind_thread();
    const int me = c_.rank, S = c_.slices;
    Ctl& k = *ctl_;
    std::vector<int64_t>& served = served_;
    std::vector<int64_t>& applied = applied_;
    std::vector<int>& kind = kind_;
    std::vector<int64_t>& nkeys = nkeys_;
    struct Pend {
      void* ev;
      bool resp;
      int s;
      int64_t t;
    };
    std::deque<Pend> pend;
    std::vector<void*> evs;
    auto get_ev = [&]() -> void* {
      if (evs.empty()) return be.event_create();
      void* e = evs.back();
      evs.pop_back();
      return e;
    };
    auto note = [&](int64_t a, int64_t b2, int64_t c, int64_t d) {
      std::lock_guard<std::mutex> g(log_mu_);
      log_.insert(log_.end(), {a, b2, c, d});
    };
    void* local = win_->local();
    int rr = 0;
    int64_t idle = 0;
    while (true) {
      bool did = false;
      const auto ti = Clock::now();
      for (int i = 0; i < W_; ++i) {
        const int s = (rr + i) % W_;
        const int64_t pt = served[s] + 1;
        const int ps = (int)(pt % R_);
        Cell& rq = k.req_c(s, me, ps);
        if (rq.seq.load(std::memory_order_acquire) == pt) {
          const int64_t n = rq.a, off = rq.b;
          const int kd = (int)rq.c;
          const size_t ix = (size_t)s * R_ + ps;
          kind[ix] = kd;
          nkeys[ix] = n;
          float* out = resp(win_->peer(s), ps) + off * vw_;
          sv_.s_pull(in_keys(local, s, ps), n, out, kd == 0, (int)ix, {0, n}, kd == 0 && fm_keep_);
          void* ev = get_ev();
          be.event_record(ev);
          pend.push_back({ev, true, s, pt});
          note(kd == 0 ? 0 : 2, s, pt, n);
          served[s] = pt;
          ++served_pulls;
          did = true;
        }
        const int64_t at = applied[s] + 1;
        if (at <= served[s]) {
          const int as = (int)(at % R_);
          const size_t ix = (size_t)s * R_ + as;
          if (kind[ix] != 0) {  // an eval pull: nothing to apply, retire the slot in order
            applied[s] = at;
            pend.push_back({nullptr, false, s, at});
            did = true;
          } else {
            Cell& pc = k.push_c(s, me, as);
            if (pc.seq.load(std::memory_order_acquire) == at) {
              const int64_t n = nkeys[ix], ne = pc.a;
              const std::vector<int64_t> offs{0, n};
              if (csr_)
                sv_.s_apply_csr(in_keys(local, s, as), in_cnt(local, s, as), in_pay(local, s, as),
                                offs, S, (int)ix);
              else
                sv_.s_apply(in_keys(local, s, as), static_cast<const float*>(in_pay(local, s, as)),
                            masks_ ? in_cnt(local, s, as) : nullptr, offs, S, (int)ix);
              sv_.end_step();
              void* ev = get_ev();
              be.event_record(ev);
              pend.push_back({ev, false, s, at});
              note(1, s, at, ne);
              applied[s] = at;
              ++applied_pushes;
              did = true;
            }
          }
        }
      }
      rr = (rr + 1) % W_;
      while (!pend.empty()) {
        const Pend& p = pend.front();
        if (p.ev && !be.event_done(p.ev)) break;
        (p.resp ? k.resp_c(me, p.s) : k.appl_c(me, p.s)).seq.store(p.t, std::memory_order_release);
        if (p.ev) evs.push_back(p.ev);
        pend.pop_front();
      }
      if (did) {
        server_busy_s += since(ti);  // (host time issuing the server's work)
        idle = 0;
        continue;
      }
      if (stop_.load() && pend.empty()) break;
      if (k.hdr->abort.load(std::memory_order_relaxed)) break;
      ++idle;
      if (idle < 128) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(idle < 4096 ? 5 : 50));
    }
    be.synchronize();
    for (void* e : evs) be.event_destroy(e);
    for (const Pend& p : pend)
      if (p.ev) be.event_destroy(p.ev);
  } catch (const std::exception& ex) {
    fail(ex.what());
  }
}

}  // namespace xflow
