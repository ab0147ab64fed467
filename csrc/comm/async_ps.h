// xflow-amd: the asynchronous parameter server (BASELINE config 4).
//
// The reference's workers never wait for each other: each Hogwild slice pulls
// its keys, computes, pushes, and the server applies every push the moment
// it arrives (lr_worker.cc:145-205, ftrl.h:54-80; M workers started
// independently, scripts/local.sh:31-35).  The lock-step ShardedStep makes
// every rank enter every all-to-all; this class removes that coupling:
//
//   * every process runs a SERVER THREAD that owns the rank's table shard
//     (its own Engine and HIP stream).  It serves pull requests and applies
//     pushes of any source in arrival order -- per source in step order --
//     exactly like a ps-lite KVServer handle;
//   * the caller's thread is the WORKER (a second Engine: dedup, forward,
//     backward).  Its keys go straight into the owners' inboxes, the owners'
//     pull kernels write the values straight into its response slot, and its
//     CSR (key, slice) gradient entries go into the owners' inboxes;
//   * all of that memory is a per-rank PeerWindow (HIP IPC, fine-grained
//     HBM over xGMI; /dev/shm on the CPU backend) and all synchronisation is
//     sequence words in a shared control segment: no collective, no RCCL
//     call, no rank ever waits for another rank's worker.
//
// Bounded staleness k: a worker pulls for step t only once every owner has
// applied its own pushes of steps <= t - k - 1 (k = 0: the reference's
// Push + Wait; pushes in flight per worker <= k).  Ring slots R = k + 1 per
// (source, owner) hold the keys / entries of the steps in flight, so the
// same wait also frees the slot.  Nothing bounds how far a fast worker runs
// ahead of a slow one -- the reference's asynchronous data parallelism; the
// measured lead is reported (max_lead).
//
// Every owner logs its operations (pull / push / eval, source, step) in the
// order its stream ran them: replaying the logs reproduces the tables bit for
// bit (tests/test_async_ps.py).
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "peer_window.h"
#include "xflow/engine.h"

namespace xflow {

class AsyncPS {
 public:
  struct Config {
    int world = 1, rank = 0;
    int staleness = 1;       // k (>= 0)
    int slices = 1;          // S per step, identical on every rank
    std::string name;        // job-unique name of the shared segments
    double timeout_s = 600;  // a wait for a peer longer than this fails
    int slow_ms = 0;         // fault knob: this worker sleeps per training step
    // inbox capacity per (source, owner) as a fraction of max_nnz keys and
    // entries (1: any key distribution fits; smaller: less memory, a step
    // whose keys are skewed past it fails)
    double pair_frac = 1.0;
    int device = -1;         // HIP device (IPC window); -1: CPU backend (shm window)
  };
  // worker / server: two engines of the same model on this rank (the server's
  // owns the table shard; its stream is the server thread's)
  AsyncPS(Engine& worker, Engine& server, const Config& c);
  ~AsyncPS();
  AsyncPS(const AsyncPS&) = delete;
  AsyncPS& operator=(const AsyncPS&) = delete;

  // handshake: every rank's handle() to every rank's connect(), then start()
  std::vector<uint8_t> handle() const { return win_->handle(); }
  void connect(const std::vector<std::vector<uint8_t>>& handles);
  void start();

  // worker: one training step (false: b has no rows, nothing done)
  bool train_step(const BatchView& b);
  // worker: forward only, keys looked up without insertion (pctr: rows)
  bool eval_step(const BatchView& b, float* pctr);
  // worker: wait until every push of this worker is applied; mark it done
  void finish();
  // server: exit the thread (every rank finished: the caller's barrier).
  // start() again resumes serving where it stopped (e.g. after an epoch's
  // statistics / checkpoint, which read the server engine from the caller)
  void stop();
  bool serving() const { return running_.load(); }

  // (kind, source, step, count) per owner operation in stream order:
  // kind 0 pull (count keys), 1 push (count entries / keys), 2 eval pull
  std::vector<int64_t> log() const;
  std::string transport() const { return win_->kind(); }
  bool csr() const { return csr_; }

  // worker counters
  int64_t steps = 0, evals = 0, bytes_moved = 0;
  int64_t max_staleness = 0;  // most own pushes unapplied at a pull
  int64_t max_lead = 0;       // most steps ahead of the slowest worker at a pull
  double wait_slot_s = 0, wait_pull_s = 0, sync_s = 0;
  // server counters (read after stop)
  int64_t served_pulls = 0, applied_pushes = 0;
  double server_busy_s = 0;

 private:
  struct Ctl;      // layout of the shared control segment (async_ps.cpp)
  void server_loop();
  bool step(const BatchView& b, float* pctr, bool train);
  void check_abort() const;
  void fail(const std::string& msg);
  void wait_event(void* ev);
  template <typename Pred>
  void wait_until(Pred p, const char* what, double* acc);
  // inbox of (owner o's window, source s, slot): keys, counts / masks, payload
  u64* in_keys(void* win, int s, int slot) const;
  u32* in_cnt(void* win, int s, int slot) const;
  void* in_pay(void* win, int s, int slot) const;
  float* resp(void* win, int slot) const;

  Engine& wk_;
  Engine& sv_;
  Config c_;
  int W_, R_;
  bool csr_ = false, masks_ = false, fm_keep_ = false;
  int vw_ = 1, gw_ = 1, eb_ = 8;
  int64_t kcap_ = 0, ecap_ = 0, ncap_ = 0;
  size_t keys_b_ = 0, cnt_b_ = 0, pay_b_ = 0, slot_b_ = 0, inbox_b_ = 0, resp_b_ = 0;
  std::unique_ptr<ShmSegment> ctl_seg_;
  Ctl* ctl_ = nullptr;
  std::unique_ptr<PeerWindow> win_;
  bool connected_ = false;
  // worker state
  int64_t seq_ = 0;  // next request number (training and eval steps)
  int64_t* counts_d_ = nullptr;
  int64_t* counts_h_ = nullptr;
  int64_t* tot_d_ = nullptr;
  int64_t* tot_h_ = nullptr;
  u64* keys_d_ = nullptr;
  u32* cnt_d_ = nullptr;
  void* pay_d_ = nullptr;
  void* wev_ = nullptr;
  // server state (kept across stop / start): per source the last step
  // whose pull was served / whose push was applied, and per (source, slot)
  // the request kind and key count
  std::vector<int64_t> served_, applied_;
  std::vector<int> kind_;
  std::vector<int64_t> nkeys_;
  void* srv_stream_ = nullptr;  // the server engine's stream at construction (restored by start)
  std::thread thr_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> running_{false};
  std::string err_;
  mutable std::mutex log_mu_;
  std::vector<int64_t> log_;
};

}  // namespace xflow
