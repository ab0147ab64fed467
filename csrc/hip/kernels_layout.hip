// xflow-amd: batch layout kernels.
//
// Row-major fixed-width blocks ([rows][F], the .xfb / libffm reader layout)
// become field-major ([F][rows], BatchView::col_stride) on the device: the
// layout the dedup and the fused LR/FM/MVM kernels read coalesced.  torch's
// generic strided copy (x.view(rows, F).t().contiguous()) ran at ~0.6 TB/s
// (279 us per 262 144 x 39 block of u64 keys); this kernel stages a tile of
// kTileRows rows x F fields in LDS with coalesced global reads, then writes
// each field's kTileRows values as one contiguous run.
#include <algorithm>

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

// Packed v3 block -> the field-major batch (UnpackArgs).  blockIdx.y = field:
// one code width and one dictionary per workgroup row, coalesced code reads
// and key writes; the dictionary gathers hit small tables (a field is
// dictionary-coded only when it has <= 65536 distinct keys).
template <typename C>
__device__ __forceinline__ u64 packed_key(const uint8_t* col, int64_t r, const u64* dict) {
  const u64 c = (u64)reinterpret_cast<const C*>(col)[r];
  return dict ? dict[c] : c;
}

__global__ void __launch_bounds__(kBlock) k_unpack_block(UnpackArgs a) {
  const int f = blockIdx.y;
  const uint8_t* col = a.block + a.col_off[f];
  const u64* dict = a.dict[f];
  const int w = a.width[f];
  const int32_t fg = a.fgid_col[f];
  u64* out = a.keys + (int64_t)f * a.rows;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < a.rows; r += stride) {
    u64 k;
    if (w == 1) k = packed_key<uint8_t>(col, r, dict);
    else if (w == 2) k = packed_key<unsigned short>(col, r, dict);
    else if (w == 4) k = packed_key<u32>(col, r, dict);
    else k = packed_key<u64>(col, r, dict);
    out[r] = k;
    if (a.fgid) a.fgid[(int64_t)f * a.rows + r] = fg;
    if (f == 0) a.labels[r] = (float)a.block[r];
  }
}

void launch_unpack_block(const UnpackArgs& a, hipStream_t st) {
  if (a.rows <= 0 || a.F <= 0) return;
  if (a.F > kMaxPackedFields) throw std::runtime_error("unpack_block: at most 64 fields");
  for (int f = 0; f < a.F; ++f) {
    const int w = a.width[f];
    if ((w != 1 && w != 2 && w != 4 && w != 8) || (a.col_off[f] % w) != 0)
      throw std::runtime_error("unpack_block: code widths 1/2/4/8, aligned columns");
  }
  const int64_t gx = std::min<int64_t>((a.rows + kBlock - 1) / kBlock, 1024);
  hipLaunchKernelGGL(k_unpack_block, dim3((unsigned)gx, (unsigned)a.F), dim3(kBlock), 0, st, a);
  XF_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace xflow
