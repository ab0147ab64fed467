// xflow-amd: peer-addressable windows and shared control segments (see
// peer_window.h).  Host code against the HIP runtime (built with hipcc).
#include "peer_window.h"

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

namespace xflow {

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("peer window: ") + what + ": " + hipGetErrorString(e));
}

std::string shm_path(const std::string& name) {
  // POSIX shm names: one leading '/', no other '/'
  std::string n = name;
  for (char& c : n)
    if (c == '/') c = '_';
  return "/" + n;
}

void* map_shm(const std::string& name, size_t bytes, bool create) {
  const std::string p = shm_path(name);
  int fd;
  if (create) {
    shm_unlink(p.c_str());  // (a stale segment of a crashed run)
    fd = shm_open(p.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  } else {
    fd = shm_open(p.c_str(), O_RDWR, 0600);
  }
  if (fd < 0)
    throw std::runtime_error("shm_open(" + p + "): " + std::strerror(errno));
  if (create && ftruncate(fd, (off_t)bytes) != 0) {
    const int e = errno;
    close(fd);
    throw std::runtime_error("ftruncate(" + p + "): " + std::strerror(e));
  }
  if (!create) {
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < bytes) {
      close(fd);
      throw std::runtime_error("shm segment " + p + " is smaller than expected");
    }
  }
  void* q = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (q == MAP_FAILED) throw std::runtime_error("mmap(" + p + "): " + std::strerror(errno));
  return q;
}

class IpcWindow final : public PeerWindow {
 public:
  IpcWindow(size_t bytes, int world, int rank, int device)
      : bytes_(bytes), world_(world), rank_(rank), device_(device), peers_(world, nullptr) {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    // XFLOW_APS_COARSE=1: plain hipMalloc (A/B; remote writes may then sit
    // behind stale L2 lines of the owner)
    const char* c = std::getenv("XFLOW_APS_COARSE");
    coarse_ = c && *c && *c != '0';
    if (coarse_)
      hip_check(hipMalloc(&p_, bytes_), "hipMalloc");
    else
      hip_check(hipExtMallocWithFlags(&p_, bytes_, hipDeviceMallocFinegrained),
                "hipExtMallocWithFlags(fine-grained)");
    hip_check(hipMemset(p_, 0, bytes_), "hipMemset");
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_check(hipIpcGetMemHandle(&h_, p_), "hipIpcGetMemHandle");
    peers_[rank_] = p_;
  }
  ~IpcWindow() override {
    (void)hipSetDevice(device_);
    for (int r = 0; r < world_; ++r)
      if (r != rank_ && peers_[r]) (void)hipIpcCloseMemHandle(peers_[r]);
    if (p_) (void)hipFree(p_);
  }
  void* local() const override { return p_; }
  size_t bytes() const override { return bytes_; }
  std::vector<uint8_t> handle() const override {
    const uint8_t* b = reinterpret_cast<const uint8_t*>(&h_);
    return std::vector<uint8_t>(b, b + sizeof(h_));
  }
  void open(const std::vector<std::vector<uint8_t>>& hs) override {
    if ((int)hs.size() != world_) throw std::invalid_argument("peer window: one handle per rank");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    for (int r = 0; r < world_; ++r) {
      if (r == rank_ || peers_[r]) continue;
      if (hs[r].size() != sizeof(hipIpcMemHandle_t))
        throw std::invalid_argument("peer window: bad IPC handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, hs[r].data(), sizeof(h));
      void* q = nullptr;
      hip_check(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess),
                ("hipIpcOpenMemHandle(rank " + std::to_string(r) + ")").c_str());
      peers_[r] = q;
    }
  }
  void* peer(int r) const override { return peers_.at(r); }
  const char* kind() const override { return coarse_ ? "ipc-coarse" : "ipc"; }

 private:
  size_t bytes_;
  int world_, rank_, device_;
  void* p_ = nullptr;
  hipIpcMemHandle_t h_{};
  std::vector<void*> peers_;
  bool coarse_ = false;
};

class ShmWindow final : public PeerWindow {
 public:
  ShmWindow(size_t bytes, int world, int rank, const std::string& name)
      : bytes_(bytes), world_(world), rank_(rank), peers_(world, nullptr) {
    name_ = name + "_w" + std::to_string(rank);
    p_ = map_shm(name_, bytes_, true);
    peers_[rank_] = p_;
  }
  ~ShmWindow() override {
    for (int r = 0; r < world_; ++r)
      if (peers_[r]) munmap(peers_[r], bytes_);
    shm_unlink(shm_path(name_).c_str());
  }
  void* local() const override { return p_; }
  size_t bytes() const override { return bytes_; }
  std::vector<uint8_t> handle() const override {
    return std::vector<uint8_t>(name_.begin(), name_.end());
  }
  void open(const std::vector<std::vector<uint8_t>>& hs) override {
    if ((int)hs.size() != world_) throw std::invalid_argument("peer window: one handle per rank");
    for (int r = 0; r < world_; ++r) {
      if (r == rank_ || peers_[r]) continue;
      peers_[r] = map_shm(std::string(hs[r].begin(), hs[r].end()), bytes_, false);
    }
  }
  void* peer(int r) const override { return peers_.at(r); }
  const char* kind() const override { return "shm"; }

 private:
  size_t bytes_;
  int world_, rank_;
  std::string name_;
  void* p_ = nullptr;
  std::vector<void*> peers_;
};

}  // namespace

std::unique_ptr<PeerWindow> make_ipc_window(size_t bytes, int world, int rank, int device) {
  return std::make_unique<IpcWindow>(bytes, world, rank, device);
}

std::unique_ptr<PeerWindow> make_shm_window(size_t bytes, int world, int rank,
                                            const std::string& name) {
  return std::make_unique<ShmWindow>(bytes, world, rank, name);
}

ShmSegment::ShmSegment(const std::string& name, size_t bytes, bool create)
    : name_(name), bytes_(bytes), owner_(create) {
  p_ = map_shm(name, bytes, create);
  if (create) std::memset(p_, 0, bytes);
}

void ShmSegment::unlink() {
  if (owner_) shm_unlink(shm_path(name_).c_str());
  owner_ = false;
}

ShmSegment::~ShmSegment() {
  if (p_) munmap(p_, bytes_);
  unlink();
}

}  // namespace xflow
