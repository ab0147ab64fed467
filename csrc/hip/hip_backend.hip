// xflow-amd: HipBackend — the gfx950 implementation of xflow::Backend.
// Memory comes straight from hipMalloc, except the parameter table's slot
// array: one reserved address range with memory mapped behind it as the table
// grows (table_reserve / table_commit); all work is queued on one HIP stream that the
// caller may replace (e.g. with PyTorch's current stream) so engine kernels and
// RCCL collectives are ordered without extra events.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "hip_util.h"
#include "kernels.h"
#include "xflow/backend.h"

namespace xflow {

namespace {

class HipBackend final : public Backend {
 public:
  explicit HipBackend(int device) : device_(device) {
    XF_HIP_CHECK(hipSetDevice(device_));
    XF_HIP_CHECK(hipStreamCreateWithFlags(&own_stream_, hipStreamNonBlocking));
    stream_ = own_stream_;
    XF_HIP_CHECK(hipMalloc(&counter_, sizeof(unsigned long long)));
  }
  ~HipBackend() override {
    hipSetDevice(device_);
    if (copy_stream_) (void)hipStreamSynchronize(copy_stream_);
    for (int s = 0; s < 2; ++s) {
      if (pinned_[s]) (void)hipHostFree(pinned_[s]);
      if (ev_copied_[s]) (void)hipEventDestroy(ev_copied_[s]);
      if (ev_used_[s]) (void)hipEventDestroy(ev_used_[s]);
    }
    if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
    if (counter_) (void)hipFree(counter_);
    if (scan_tiles_) {  // (stream-ordered allocation; the caller's stream may be gone)
      (void)hipDeviceSynchronize();
      (void)hipFreeAsync(scan_tiles_, own_stream_);
      (void)hipStreamSynchronize(own_stream_);
    }
    if (split_marks_) (void)hipFree(split_marks_);
    if (own_stream_) (void)hipStreamDestroy(own_stream_);
  }

  // ---- double-buffered H2D staging on a copy stream (see Backend) ----
  void stage_begin(int s) override {
    if (!copy_stream_) {
      XF_HIP_CHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
      for (int i = 0; i < 2; ++i) {
        XF_HIP_CHECK(hipEventCreateWithFlags(&ev_copied_[i], hipEventDisableTiming));
        XF_HIP_CHECK(hipEventCreateWithFlags(&ev_used_[i], hipEventDisableTiming));
      }
    }
    if (copied_pending_[s]) {  // the pinned buffer is free once its copies finished
      XF_HIP_CHECK(hipEventSynchronize(ev_copied_[s]));
      copied_pending_[s] = false;
    }
    waited_used_[s] = false;
  }
  void* stage_pinned(int s, size_t bytes) override {
    if (bytes > pinned_cap_[s]) {
      if (pinned_[s]) XF_HIP_CHECK(hipHostFree(pinned_[s]));
      pinned_cap_[s] = bytes + bytes / 4;
      XF_HIP_CHECK(hipHostMalloc(&pinned_[s], pinned_cap_[s], hipHostMallocDefault));
    }
    return pinned_[s];
  }
  void stage_copy(int s, void* dst, size_t off, size_t bytes) override {
    if (!bytes) return;
    if (used_pending_[s] && !waited_used_[s]) {  // the last step reading slot s's buffers
      XF_HIP_CHECK(hipStreamWaitEvent(copy_stream_, ev_used_[s], 0));
      waited_used_[s] = true;
    }
    XF_HIP_CHECK(hipMemcpyAsync(dst, static_cast<char*>(pinned_[s]) + off, bytes,
                                hipMemcpyHostToDevice, copy_stream_));
  }
  void stage_commit(int s) override {
    XF_HIP_CHECK(hipEventRecord(ev_copied_[s], copy_stream_));
    XF_HIP_CHECK(hipStreamWaitEvent(stream_, ev_copied_[s], 0));
    copied_pending_[s] = true;
  }
  void stage_release(int s) override {
    XF_HIP_CHECK(hipEventRecord(ev_used_[s], stream_));
    used_pending_[s] = true;
  }

  bool is_gpu() const override { return true; }
  std::string name() const override { return "hip:gfx950:" + std::to_string(device_); }

  void* alloc(size_t bytes) override {
    void* p = nullptr;
    if (bytes == 0) bytes = 16;
    XF_HIP_CHECK(hipSetDevice(device_));
    XF_HIP_CHECK(hipMalloc(&p, bytes));
    return p;
  }
  void free(void* p) override {
    if (p) (void)hipFree(p);
  }
  void* alloc_stream(size_t bytes) override {
    void* p = nullptr;
    if (bytes == 0) bytes = 16;
    XF_HIP_CHECK(hipSetDevice(device_));
    XF_HIP_CHECK(hipMallocAsync(&p, bytes, stream_));
    return p;
  }
  void free_stream(void* p) override {
    if (p) XF_HIP_CHECK(hipFreeAsync(p, stream_));
  }
  void memset(void* p, int v, size_t bytes) override {
    if (bytes) XF_HIP_CHECK(hipMemsetAsync(p, v, bytes, stream_));
  }
  void fill_u64(u64* p, u64 v, size_t n) override { hip::launch_fill_u64(p, v, n, stream_); }
  void copy_h2d(void* dst, const void* src, size_t bytes) override {
    if (bytes) XF_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream_));
    // host buffer may be reused by the caller right away
    XF_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void copy_d2h(void* dst, const void* src, size_t bytes) override {
    if (bytes) XF_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream_));
    XF_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void copy_d2h_async(void* dst, const void* src, size_t bytes) override {
    if (bytes) XF_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream_));
  }
  void copy_h2d_async(void* dst, const void* src, size_t bytes) override {
    if (bytes) XF_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream_));
  }
  void* staging_alloc(size_t bytes) override {
    void* p = nullptr;
    XF_HIP_CHECK(hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault));
    return p;
  }
  void staging_free(void* p) override {
    if (p) (void)hipHostFree(p);
  }
  void copy_d2d(void* dst, const void* src, size_t bytes) override {
    if (bytes) XF_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream_));
  }
  void download_small(void* dst, const void* src, size_t bytes) override {
    hip::launch_download_small(dst, src, bytes, stream_);
  }
  void upload_small(void* dst, const void* src, size_t bytes) override {
    hip::launch_upload_small(dst, src, bytes, stream_);
  }
  void synchronize() override { XF_HIP_CHECK(hipStreamSynchronize(stream_)); }
  size_t free_memory() const override {
    size_t fr = 0, tot = 0;
    XF_HIP_CHECK(hipSetDevice(device_));
    XF_HIP_CHECK(hipMemGetInfo(&fr, &tot));
    return fr;
  }
  void snapshot(HostSnap* dst, const u32* mon, unsigned long long seq) override {
    hip::launch_snapshot(dst, mon, seq, stream_);
  }
  // (coherent: the monitor polls snapshots the kernels write, no event)
  void* host_alloc(size_t bytes) override {
    void* p = nullptr;
    XF_HIP_CHECK(hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocCoherent));
    std::memset(p, 0, bytes ? bytes : 16);
    return p;
  }
  void host_free(void* p) override {
    if (p) (void)hipHostFree(p);
  }
  void* event_create() override {
    hipEvent_t e = nullptr;
    XF_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }
  void event_destroy(void* e) override {
    if (e) (void)hipEventDestroy(static_cast<hipEvent_t>(e));
  }
  void event_record(void* e) override {
    XF_HIP_CHECK(hipEventRecord(static_cast<hipEvent_t>(e), stream_));
  }
  bool event_done(void* e) override {
    const hipError_t r = hipEventQuery(static_cast<hipEvent_t>(e));
    if (r == hipErrorNotReady) return false;
    XF_HIP_CHECK(r);
    return true;
  }
  void event_wait(void* e) override { XF_HIP_CHECK(hipEventSynchronize(static_cast<hipEvent_t>(e))); }
  // nullptr selects the null (default) stream, which is what torch reports as
  // its default current stream.
  void set_stream(void* s) override { stream_ = reinterpret_cast<hipStream_t>(s); }
  void* stream() const override { return stream_; }
  void bind_thread() override { XF_HIP_CHECK(hipSetDevice(device_)); }

  void table_clear(const TableView& t) override { hip::launch_table_clear(t, stream_); }
  void dedup(const u64* keys, int64_t nnz, ScratchView s, DedupOut o) override {
    hip::launch_dedup(keys, nnz, s, o, stream_);
  }
  void scratch_reset(ScratchView s, const u32* pos, const int64_t* n_dev, int64_t n_max) override {
    hip::launch_scratch_reset(s, pos, n_dev, n_max, stream_);
  }
  void table_pull(const PullArgs& a) override { hip::launch_table_pull(a, stream_); }
  void table_apply(const ApplyArgs& a) override { hip::launch_table_apply(a, stream_); }
  void forward_backward(const FwdArgs& a) override { hip::launch_forward_backward(a, stream_); }
  void slice_masks(const BatchView& b, const u32* pos, u32* tmask) override {
    hip::launch_slice_masks(b, pos, tmask, stream_);
  }
  void parse_text(const TextParseArgs& a) override { hip::launch_parse_text(a, stream_); }
  bool remaps_positions() const override { return true; }
  void remap_pos(u32* pos, int64_t nnz, const u32* inv, u32 none) override {
    hip::launch_remap_pos(pos, nnz, inv, none, stream_);
  }
  void bucket(const BucketArgs& a) override { hip::launch_bucket(a, stream_); }
  bool partitioned_dedup() const override { return true; }
  void partition_counts(const ScratchView& s, const u32* chunk_offsets, const int64_t* n_uniq,
                        int64_t* counts, int64_t seq) override {
    hip::launch_partition_counts(s, chunk_offsets, n_uniq, counts, seq, stream_);
  }
  bool owner_grouping() const override { return true; }
  void owner_group(const OwnerGroupArgs& a) override { hip::launch_owner_group(a, stream_); }
  void gather_grads(const GatherGradArgs& a) override { hip::launch_gather_grads(a, stream_); }
  bool csr_exchange() const override { return true; }
  void scan_u32(const u32* in, u32* out, const int64_t* n_dev, int64_t n_max) override {
    const size_t words = (size_t)(n_max / 4096 + 4);
    if (words > scan_tiles_words_) {  // (grow-only, stream-ordered: no host wait)
      if (scan_tiles_) free_stream(scan_tiles_);
      scan_tiles_words_ = words + words / 2;
      scan_tiles_ = static_cast<u32*>(alloc_stream(scan_tiles_words_ * sizeof(u32)));
    }
    hip::launch_scan_u32(in, out, n_dev, n_max, scan_tiles_, stream_);
  }
  void csr_pack(const u32* off, const u32* cnt, const void* src, const u32* doff,
                const int64_t* n_dev, int64_t n_max, void* dst, int entry_bytes) override {
    hip::launch_csr_pack(off, cnt, src, doff, n_dev, n_max, dst, entry_bytes, stream_);
  }
  void csr_totals(const int64_t* counts, int world, bool encoded, const u32* doff,
                  int64_t* totals) override {
    hip::launch_csr_totals(counts, world, encoded, doff, totals, stream_);
  }
  void scatter_rows(const float* src, float* dst, const u32* map, const int64_t* n_dev,
                    int64_t n_max, int width, float* zero_out, int zero_width) override {
    hip::launch_scatter_rows(src, dst, map, n_dev, n_max, width, zero_out, zero_width, stream_);
  }
  void gather_rows(const float* src, float* dst, const u32* map, const int64_t* n_dev,
                   int64_t n_max, int width, bool zero_src) override {
    hip::launch_gather_rows(src, dst, map, n_dev, n_max, width, zero_src, stream_);
  }
  void gather_u32(const u32* src, u32* dst, const u32* map, const int64_t* n_dev, int64_t n_max,
                  bool zero_src) override {
    hip::launch_gather_u32(src, dst, map, n_dev, n_max, zero_src, stream_);
  }
  void scatter_u32(const u32* src, u32* dst, const u32* map, const int64_t* n_dev,
                   int64_t n_max) override {
    hip::launch_scatter_u32(src, dst, map, n_dev, n_max, stream_);
  }
  void synth_batch(const SynthArgs& a) override { hip::launch_synth(a, stream_); }
  void unpack_block(const UnpackArgs& a) override { hip::launch_unpack_block(a, stream_); }
  void field_major(const void* src, void* dst, int64_t rows, int F, int elem_bytes,
                   bool widen) override {
    hip::launch_field_major(src, dst, rows, F, elem_bytes, widen, stream_);
  }
  int64_t table_export(const TableView& t, u64* keys_out, u32* words_out,
                       int64_t max_rows) override {
    hip::launch_table_export(t, keys_out, words_out, max_rows, counter_, stream_);
    unsigned long long n = 0;
    copy_d2h(&n, counter_, sizeof(n));
    return (int64_t)n;
  }
  void table_import(const TableView& t, const u64* keys, const u32* words, int64_t n) override {
    hip::launch_table_import(t, keys, words, n, stream_);
  }
  void table_prefill(const TableView& t, int64_t n, u64 seed) override {
    hip::launch_table_prefill(t, n, seed, stream_);
  }
  void table_split(const TableView& t, u64 s0, u64 k) override {
    const size_t words = (size_t)(((k << t.seg_log2) + 63) / 64);
    if (words > split_marks_words_) {
      if (split_marks_) (void)hipFree(split_marks_);
      split_marks_ = nullptr;
      XF_HIP_CHECK(hipMalloc(&split_marks_, words * sizeof(u64)));
      split_marks_words_ = words;
    }
    hip::launch_table_split(t, s0, k, split_marks_, stream_);
  }

  // ---- the table's address range (virtual memory management) ----
  // One range of the table's maximum size is reserved; memory is created and
  // mapped behind it as the table grows, in chunks of at least 1/8 of what is
  // mapped (few mappings, <= 12.5 % slack).  A table that cannot grow, or
  // no VMM support (or XFLOW_TABLE_VMM=0): one hipMalloc, re-allocated and
  // copied on growth.  (The headline step runs ~1 % faster on hipMalloc
  // memory than on VMM-mapped memory: profiles/r4_table_segments.txt.)
  void* table_reserve(size_t max_bytes, bool growable) override {
    int vmm = 0;
    XF_HIP_CHECK(hipSetDevice(device_));
    (void)hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, device_);
    const char* env = std::getenv("XFLOW_TABLE_VMM");
    if ((env && env[0] == '0') || !growable) vmm = 0;
    vm_on_ = false;
    if (vmm) {
      vm_prop_ = hipMemAllocationProp{};
      vm_prop_.type = hipMemAllocationTypePinned;
      vm_prop_.location.type = hipMemLocationTypeDevice;
      vm_prop_.location.id = device_;
      size_t gran = 0;
      if (hipMemGetAllocationGranularity(&gran, &vm_prop_, hipMemAllocationGranularityRecommended) ==
              hipSuccess && gran > 0) {
        vm_gran_ = gran;
        vm_max_ = (max_bytes + gran - 1) / gran * gran;
        void* p = nullptr;
        if (hipMemAddressReserve(&p, vm_max_, gran, nullptr, 0) == hipSuccess) {
          vm_on_ = true;
          vm_base_ = p;
          vm_committed_ = 0;
          return p;
        }
      }
      (void)hipGetLastError();
    }
    fb_bytes_ = 0;
    fb_max_ = max_bytes;
    return nullptr;
  }
  void* table_commit(void* base, size_t bytes) override {
    if (vm_on_) {
      if (bytes <= vm_committed_) return base;
      if (bytes > vm_max_) throw std::runtime_error("xflow: table beyond its reserved range");
      size_t want = (bytes + vm_gran_ - 1) / vm_gran_ * vm_gran_;
      size_t ahead = (vm_committed_ / 8 + vm_gran_ - 1) / vm_gran_ * vm_gran_;
      if (vm_committed_ && want < vm_committed_ + ahead) want = vm_committed_ + ahead;
      if (want > vm_max_) want = vm_max_;
      {  // (the slack only when the device has room for it)
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && want - vm_committed_ + (512u << 20) > fr)
          want = (bytes + vm_gran_ - 1) / vm_gran_ * vm_gran_;
      }
      const size_t add = want - vm_committed_;
      char* at = static_cast<char*>(vm_base_) + vm_committed_;
      hipMemGenericAllocationHandle_t h;
      XF_HIP_CHECK(hipMemCreate(&h, add, &vm_prop_, 0));
      XF_HIP_CHECK(hipMemMap(at, add, 0, h, 0));
      hipMemAccessDesc acc{};
      acc.location = vm_prop_.location;
      acc.flags = hipMemAccessFlagsProtReadWrite;
      // (ROCm takes the access of a range only from the reservation's base:
      // a range starting inside it is refused -- tools/probe/vmm_probe.hip)
      XF_HIP_CHECK(hipMemSetAccess(vm_base_, want, &acc, 1));
      vm_chunks_.push_back(VmChunk{vm_committed_, add, h});
      vm_committed_ = want;
      return base;
    }
    if (bytes <= fb_bytes_) return base;
    // (no virtual memory: every growth re-allocates and copies, so grow
    // geometrically -- 1.5x, within the reservation and what is free next to
    // the live table -- instead of one copy of the table per paced split)
    if (base && fb_bytes_) {
      size_t want = fb_bytes_ + fb_bytes_ / 2;
      if (want > fb_max_) want = fb_max_;
      size_t fr = 0, tot = 0;
      if (want > bytes && hipMemGetInfo(&fr, &tot) == hipSuccess && want + (512u << 20) <= fr)
        bytes = want;
    }
    void* p = alloc(bytes);
    if (base && fb_bytes_) {
      copy_d2d(p, base, fb_bytes_);
      synchronize();
      free(base);
    }
    fb_bytes_ = bytes;
    return p;
  }
  void table_release(void* base) override {
    if (!vm_on_) {
      free(base);
      fb_bytes_ = 0;
      return;
    }
    (void)hipSetDevice(device_);
    (void)hipDeviceSynchronize();
    for (const VmChunk& c : vm_chunks_) {
      (void)hipMemUnmap(static_cast<char*>(vm_base_) + c.off, c.bytes);
      (void)hipMemRelease(c.h);
    }
    vm_chunks_.clear();
    (void)hipMemAddressFree(vm_base_, vm_max_);
    vm_on_ = false;
    vm_base_ = nullptr;
    vm_committed_ = 0;
  }
  size_t table_committed() const override { return vm_on_ ? vm_committed_ : fb_bytes_; }
  bool table_in_place() const override { return vm_on_; }

  EvalMetrics eval_metrics(const float* pctr, const float* labels, int64_t n) override {
    EvalMetrics m;
    hip::launch_eval_metrics(pctr, labels, n, &m, stream_);
    return m;
  }
  int64_t table_nonzero(const TableView& t, const OptSpec& o) override {
    hip::launch_table_nonzero(t, o, counter_, stream_);
    unsigned long long n = 0;
    copy_d2h(&n, counter_, sizeof(n));
    return (int64_t)n;
  }

 private:
  int device_;
  hipStream_t own_stream_ = nullptr;
  hipStream_t stream_ = nullptr;
  unsigned long long* counter_ = nullptr;
  hipStream_t copy_stream_ = nullptr;
  hipEvent_t ev_copied_[2] = {nullptr, nullptr}, ev_used_[2] = {nullptr, nullptr};
  void* pinned_[2] = {nullptr, nullptr};
  size_t pinned_cap_[2] = {0, 0};
  bool copied_pending_[2] = {false, false}, used_pending_[2] = {false, false};
  bool waited_used_[2] = {false, false};
  u64* split_marks_ = nullptr;
  size_t split_marks_words_ = 0;
  struct VmChunk {
    size_t off, bytes;
    hipMemGenericAllocationHandle_t h;
  };
  bool vm_on_ = false;
  void* vm_base_ = nullptr;
  size_t vm_max_ = 0, vm_gran_ = 0, vm_committed_ = 0, fb_bytes_ = 0, fb_max_ = 0;
  u32* scan_tiles_ = nullptr;
  size_t scan_tiles_words_ = 0;
  hipMemAllocationProp vm_prop_{};
  std::vector<VmChunk> vm_chunks_;
};

}  // namespace

std::unique_ptr<Backend> make_hip_backend(int device) {
  return std::unique_ptr<Backend>(new HipBackend(device));
}

bool hip_backend_available() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return false;
  return n > 0;
}

}  // namespace xflow
