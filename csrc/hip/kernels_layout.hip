// xflow-amd: batch layout kernels.
//
// Row-major fixed-width blocks ([rows][F], the .xfb / libffm reader layout)
// become field-major ([F][rows], BatchView::col_stride) on the device: the
// layout the dedup and the fused LR/FM/MVM kernels read coalesced.  torch's
// generic strided copy (x.view(rows, F).t().contiguous()) ran at ~0.6 TB/s
// (279 us per 262 144 x 39 block of u64 keys); this kernel stages a tile of
// kTileRows rows x F fields in LDS with coalesced global reads, then writes
// each field's kTileRows values as one contiguous run.
#include "kernels.h"
#include "hip_util.h"

namespace xflow {
namespace hip {

constexpr int kTileRows = 64;
constexpr int kMaxTileFields = 64;  // LDS: 64 x 65 x 8 B = 33 KB per workgroup

// TO != T: zero-extending copy (compact u32 .xfb keys -> u64 engine keys:
// half the H2D bytes of the streamed input path, widened in this pass)
template <typename T, typename TO = T>
__global__ void __launch_bounds__(kBlock) k_field_major(const T* __restrict__ src,
                                                        TO* __restrict__ dst, int64_t rows, int F) {
  // (+1 column of padding: consecutive rows of one field land in different banks)
  __shared__ T tile[kTileRows * (kMaxTileFields + 1)];
  const int64_t r0 = (int64_t)blockIdx.x * kTileRows;
  const int nr = (int)(rows - r0 < kTileRows ? rows - r0 : kTileRows);
  const int n = nr * F;
  const T* s = src + r0 * F;  // the tile's rows are one contiguous run
  for (int i = threadIdx.x; i < n; i += kBlock) {
    const int r = i / F, f = i - r * F;
    tile[r * (kMaxTileFields + 1) + f] = s[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < F * kTileRows; i += kBlock) {
    const int f = i / kTileRows, r = i - f * kTileRows;
    if (r < nr) dst[(int64_t)f * rows + r0 + r] = (TO)tile[r * (kMaxTileFields + 1) + f];
  }
}

void launch_field_major(const void* src, void* dst, int64_t rows, int F, int elem_bytes,
                        bool widen, hipStream_t st) {
  if (rows <= 0 || F <= 0) return;
  if (F > kMaxTileFields) throw std::runtime_error("field_major: at most 64 fields");
  const int64_t g = (rows + kTileRows - 1) / kTileRows;
  if (widen) {
    if (elem_bytes != 4) throw std::runtime_error("field_major: widen needs 4-byte elements");
    hipLaunchKernelGGL((k_field_major<u32, unsigned long long>), dim3((unsigned)g), dim3(kBlock),
                       0, st, static_cast<const u32*>(src), static_cast<unsigned long long*>(dst),
                       rows, F);
  } else if (elem_bytes == 8) {
    hipLaunchKernelGGL(k_field_major<unsigned long long>, dim3((unsigned)g), dim3(kBlock), 0, st,
                       static_cast<const unsigned long long*>(src),
                       static_cast<unsigned long long*>(dst), rows, F);
  } else if (elem_bytes == 4) {
    hipLaunchKernelGGL(k_field_major<u32>, dim3((unsigned)g), dim3(kBlock), 0, st,
                       static_cast<const u32*>(src), static_cast<u32*>(dst), rows, F);
  } else {
    throw std::runtime_error("field_major: 4- or 8-byte elements");
  }
  XF_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace xflow
