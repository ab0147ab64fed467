// xflow-amd: memory every rank of a one-node job can address directly.
//
// The asynchronous parameter server (async_ps.h) keeps each owner's inboxes
// and each worker's pull-response slots in a per-rank "window":
//   IPC  (HIP backend): fine-grained device memory exported with a HIP IPC
//        handle and mapped by every peer process -- a worker's copy into an
//        owner's inbox and an owner's pull kernel writing a worker's response
//        slot are plain device stores / DMA over xGMI, no collective, no host
//        staging.  Fine-grained so that a peer's writes into this GPU's HBM
//        are not hidden behind stale lines of its L2 (remote writes bypass it).
//   SHM  (CPU backend): a /dev/shm file mapped by every process.
// Plus ShmSegment, the small host-shared control block (sequence words) both
// transports synchronise through.  The reference's equivalent is ps-lite's
// ZeroMQ van; one node's ranks need no sockets.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace xflow {

class PeerWindow {
 public:
  virtual ~PeerWindow() = default;
  virtual void* local() const = 0;
  virtual size_t bytes() const = 0;
  // what a peer needs to map this window (IPC handle bytes / shm name)
  virtual std::vector<uint8_t> handle() const = 0;
  // map every peer's window (handles[r] from rank r's handle())
  virtual void open(const std::vector<std::vector<uint8_t>>& handles) = 0;
  // rank r's window in this process's address space (own rank: local())
  virtual void* peer(int r) const = 0;
  virtual const char* kind() const = 0;
};

// HIP IPC window on `device` (csrc/comm/peer_window.cpp, built with hipcc)
std::unique_ptr<PeerWindow> make_ipc_window(size_t bytes, int world, int rank, int device);
// /dev/shm window "<name>_w<rank>" (host memory: the CPU backend's transport)
std::unique_ptr<PeerWindow> make_shm_window(size_t bytes, int world, int rank,
                                            const std::string& name);

// A named POSIX shared-memory segment.  create: make it (replacing a stale
// one of the same name) and zero it; else open an existing one of >= bytes.
// The creator unlinks the name on destruction (mappings stay valid).
class ShmSegment {
 public:
  ShmSegment(const std::string& name, size_t bytes, bool create);
  ~ShmSegment();
  ShmSegment(const ShmSegment&) = delete;
  ShmSegment& operator=(const ShmSegment&) = delete;
  void* data() const { return p_; }
  size_t bytes() const { return bytes_; }
  void unlink();

 private:
  std::string name_;
  void* p_ = nullptr;
  size_t bytes_ = 0;
  bool owner_ = false;
};

}  // namespace xflow
