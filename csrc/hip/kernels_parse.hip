// xflow-amd: libffm text -> CSR batch on the device (gfx950).
//
// The reference parses every block of text on its training threads
// (/root/reference/src/io/load_data_from_disk.cc:103-210, the only loader it
// uses); csrc/io/reader.cpp does the same on the host at ~1.3 GB/s.  Here a
// block's bytes are uploaded as they are and tokenised where they will be
// used:
//
//   k_nl_count   newlines per 4 KB chunk (one dwordx4 per lane, exact SWAR
//                zero-byte count)
//   k_nl_scan    chunk offsets (one workgroup), line count, virtual last line
//   k_nl_write   every line's end offset, in order
//   k_line_count one lane per line: has a TAB (a row), feature tokens
//   k_scan_*     row index and occurrence offset of every line (u64 scan of
//                (row flag << 40 | tokens))
//   k_line_emit  one lane per row: label (atof > 1e-7), row_ptr, and per
//                token fgid = (int)atof(field) and key = std::hash<string> of
//                the feature text (libstdc++ _Hash_bytes: MurmurHash64A
//                variant, seed 0xc70f6907)
//
// Parse rules are reader.cpp's (themselves load_data_from_disk.cc's): lines
// end at '\n'; a line without '\t' is no row; tokens after the TAB are split
// at ' ' (empty ones skipped); a token without ':' is no feature; the key
// hashes the text between the first and second ':' (a 2-part token: to the
// end, trailing '\r' stripped); the value is never read.  Bit-equal keys,
// field ids, labels and row offsets (tests/test_gpu_parse.py).
#include "kernels.h"
#include "hip_util.h"

namespace xflow {
namespace hip {

namespace {

constexpr int kPBlock = 256;
constexpr int kChunkBytes = 16;                       // one dwordx4 per lane
constexpr int kWgBytes = kPBlock * kChunkBytes;       // 4 KB per workgroup

// exact number of '\n' bytes in a 32-bit word (no borrow false positives)
__device__ __forceinline__ u32 nl_in_word(u32 w) {
  const u32 x = w ^ 0x0A0A0A0Au;  // '\n' bytes -> 0
  u32 y = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  y = ~(y | x | 0x7F7F7F7Fu);     // high bit set exactly in the zero bytes
  return (u32)__popc(y);
}

__device__ __forceinline__ u32 nl_in_lane(const char* __restrict__ text, int64_t n, int64_t base) {
  if (base + kChunkBytes <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(text + base);
    return nl_in_word(v.x) + nl_in_word(v.y) + nl_in_word(v.z) + nl_in_word(v.w);
  }
  u32 c = 0;
  for (int64_t i = base; i < n; ++i) c += text[i] == '\n';
  return c;
}

__global__ void __launch_bounds__(kPBlock) k_nl_count(const char* __restrict__ text, int64_t n,
                                                      u32* __restrict__ wg_cnt) {
  const int64_t base = (int64_t)blockIdx.x * kWgBytes + (int64_t)threadIdx.x * kChunkBytes;
  u32 tot;
  (void)block_exclusive_scan<kPBlock>(nl_in_lane(text, n, base), &tot);
  if (threadIdx.x == 0) wg_cnt[blockIdx.x] = tot;
}

// one workgroup: exclusive offsets of the chunk counts (in place), the line
// count and -- for text not ending in '\n' -- the virtual end of its last line
__global__ void __launch_bounds__(1024) k_nl_scan(u32* __restrict__ wg_cnt, int nwg,
                                                  const char* __restrict__ text, int64_t n,
                                                  u32* __restrict__ line_end, int64_t max_lines,
                                                  long long* __restrict__ counts) {
  u32 carry = 0;
  for (int c0 = 0; c0 < nwg; c0 += 1024) {
    const int i = c0 + (int)threadIdx.x;
    const u32 v = i < nwg ? wg_cnt[i] : 0u;
    u32 t;
    const u32 ex = block_exclusive_scan<1024>(v, &t);
    if (i < nwg) wg_cnt[i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) {
    long long lines = carry;
    if (n > 0 && text[n - 1] != '\n') {
      if (lines < max_lines) line_end[lines] = (u32)n;
      ++lines;
    }
    if (lines > max_lines) counts[5] = 1;  // (more lines than the workspace holds)
    counts[4] = lines;
  }
}

__global__ void __launch_bounds__(kPBlock) k_nl_write(const char* __restrict__ text, int64_t n,
                                                      const u32* __restrict__ wg_off,
                                                      u32* __restrict__ line_end,
                                                      int64_t max_lines) {
  const int64_t base = (int64_t)blockIdx.x * kWgBytes + (int64_t)threadIdx.x * kChunkBytes;
  u32 tot;
  int64_t k = wg_off[blockIdx.x] + block_exclusive_scan<kPBlock>(nl_in_lane(text, n, base), &tot);
  const int64_t e = base + kChunkBytes < n ? base + kChunkBytes : n;
  for (int64_t i = base; i < e && k < max_lines; ++i)
    if (text[i] == '\n') line_end[k++] = (u32)i;
}

__device__ __forceinline__ bool is_space(char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

// atof of the NUL-terminated copy of [b, e) (reader.cpp range_atof: at most
// 63 characters): leading white space, sign, inf / nan, decimal digits with
// a fraction and an exponent.  Correctly rounded for up to 19 significant
// digits and |decimal exponent| <= 22 (exact powers of ten) -- every label
// and field id of CTR data; hexadecimal floats are not recognised (0).
__device__ double dev_atof(const char* __restrict__ b, const char* __restrict__ e) {
  if (e - b > 63) e = b + 63;
  const char* p = b;
  while (p < e && is_space(*p)) ++p;
  bool neg = false;
  if (p < e && (*p == '+' || *p == '-')) neg = *p++ == '-';
  if (e - p >= 3 && (p[0] | 32) == 'i' && (p[1] | 32) == 'n' && (p[2] | 32) == 'f')
    return neg ? -INFINITY : INFINITY;
  if (e - p >= 3 && (p[0] | 32) == 'n' && (p[1] | 32) == 'a' && (p[2] | 32) == 'n') return NAN;
  unsigned long long mant = 0;
  int digits = 0, ex = 0;
  bool any = false;
  for (; p < e && *p >= '0' && *p <= '9'; ++p) {
    any = true;
    if (digits < 19) {
      mant = mant * 10ull + (unsigned long long)(*p - '0');
      digits += mant != 0ull;
    } else {
      ++ex;
    }
  }
  if (p < e && *p == '.') {
    for (++p; p < e && *p >= '0' && *p <= '9'; ++p) {
      any = true;
      if (digits < 19) {
        mant = mant * 10ull + (unsigned long long)(*p - '0');
        digits += mant != 0ull;
        --ex;
      }
    }
  }
  if (!any) return 0.0;
  if (p < e && (*p | 32) == 'e') {
    const char* q = p + 1;
    bool eneg = false;
    if (q < e && (*q == '+' || *q == '-')) eneg = *q++ == '-';
    if (q < e && *q >= '0' && *q <= '9') {
      int v = 0;
      for (; q < e && *q >= '0' && *q <= '9'; ++q) v = v < 100000 ? v * 10 + (*q - '0') : v;
      ex += eneg ? -v : v;
    }
  }
  double r = (double)mant;
  if (mant != 0ull && ex != 0) {
    if (ex > 0 && ex <= 22) r *= exp10((double)ex);
    else if (ex < 0 && ex >= -22) r /= exp10((double)-ex);
    else r *= exp10((double)ex);
  }
  return neg ? -r : r;
}

// libstdc++ std::hash<std::string> on LP64: _Hash_bytes(p, n, 0xc70f6907)
__device__ __forceinline__ u64 std_hash_bytes(const char* __restrict__ p, int64_t n) {
  const u64 mul = (0xc6a4a793ull << 32) + 0x5bd1e995ull;
  auto shift_mix = [](u64 v) { return v ^ (v >> 47); };
  u64 h = 0xc70f6907ull ^ ((u64)n * mul);
  const int64_t n8 = n & ~(int64_t)7;
  for (int64_t i = 0; i < n8; i += 8) {
    u64 d = 0;
#pragma unroll
    for (int k = 7; k >= 0; --k) d = (d << 8) | (unsigned char)p[i + k];
    h ^= shift_mix(d * mul) * mul;
    h *= mul;
  }
  if (n & 7) {
    u64 d = 0;
    for (int64_t k = n - 1; k >= n8; --k) d = (d << 8) | (unsigned char)p[k];
    h ^= d;
    h *= mul;
  }
  h = shift_mix(h) * mul;
  return shift_mix(h);
}

// Sequential reader of a line's bytes from aligned 16-byte chunks held in
// registers, the next chunk loaded one ahead: a lane scanning its line byte by
// byte waits on one load per 16 bytes (latency hidden by the look-ahead)
// instead of one dependent byte load per byte.  Reads stay inside the text
// allocation: callers give >= 32 bytes of allocation beyond the block.
struct ByteStream {
  const char* __restrict__ t;
  int64_t base;  // 16-byte aligned offset of cur
  uint4 cur, nxt;
  __device__ __forceinline__ void start(const char* __restrict__ text, int64_t i) {
    t = text;
    base = i & ~(int64_t)15;
    cur = *reinterpret_cast<const uint4*>(t + base);
    nxt = *reinterpret_cast<const uint4*>(t + base + 16);
  }
  // byte i (i >= the previous i: sequential, forward)
  __device__ __forceinline__ char at(int64_t i) {
    while (i >= base + 16) {
      base += 16;
      cur = nxt;
      nxt = *reinterpret_cast<const uint4*>(t + base + 16);
    }
    const int o = (int)(i - base);
    const u32 w = o < 8 ? (o < 4 ? cur.x : cur.y) : (o < 12 ? cur.z : cur.w);
    return (char)(w >> ((o & 3) * 8));
  }
};

// [start, end) of line l (end: its '\n' or the text end)
__device__ __forceinline__ void line_span(const u32* __restrict__ line_end, int64_t l,
                                          int64_t& s, int64_t& e) {
  s = l == 0 ? 0 : (int64_t)line_end[l - 1] + 1;
  e = line_end[l];
}


// row flag << 40 | feature tokens of each line
constexpr int kTokBits = 40;

__global__ void __launch_bounds__(kPBlock) k_line_count(const char* __restrict__ text,
                                                        const u32* __restrict__ line_end,
                                                        const long long* __restrict__ counts,
                                                        unsigned long long* __restrict__ lv,
                                                        int64_t max_lines) {
  int64_t nl = counts[4];
  nl = nl < max_lines ? nl : max_lines;
  // (grid-stride: the grid is sized for the workspace bound, the lines are
  // counted on the device)
  for (int64_t l = (int64_t)blockIdx.x * kPBlock + threadIdx.x; l < nl;
       l += (int64_t)gridDim.x * kPBlock) {
  int64_t s, e;
  line_span(line_end, l, s, e);
  // one forward pass: the first TAB starts the tokens; a token (a run
  // between ' ') counts when it holds a ':'
  ByteStream bs;
  bs.start(text, s);
  bool row = false, colon = false;
  unsigned long long tok = 0;
  for (int64_t i = s; i < e; ++i) {
    const char c = bs.at(i);
    if (!row) {
      row = c == '\t';
      continue;
    }
    if (c == ' ') {
      tok += colon;
      colon = false;
    } else {
      colon |= c == ':';
    }
  }
  tok += colon;
  lv[l] = row ? ((1ull << kTokBits) | tok) : 0ull;
  }
}

// exclusive scan of n u64 values in place: per-workgroup totals, one
// workgroup over the totals, then each workgroup's own scan
constexpr int kScanPer = 4;  // values per lane
constexpr int kScanWg = kPBlock * kScanPer;

__device__ __forceinline__ unsigned long long block_excl_u64(unsigned long long v,
                                                              unsigned long long* total) {
  __shared__ unsigned long long wsum[kPBlock / kWave];
  const int lane = threadIdx.x % kWave, w = threadIdx.x / kWave;
  unsigned long long incl = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const unsigned long long t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  if (lane == kWave - 1) wsum[w] = incl;
  __syncthreads();
  unsigned long long off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kPBlock / kWave; ++i) {
    off += i < w ? wsum[i] : 0ull;
    tot += wsum[i];
  }
  __syncthreads();
  *total = tot;
  return off + incl - v;
}

__global__ void __launch_bounds__(kPBlock) k_scan_reduce(const unsigned long long* __restrict__ v,
                                                         const long long* __restrict__ counts,
                                                         int64_t max_n,
                                                         unsigned long long* __restrict__ wg) {
  int64_t n = counts[4];
  n = n < max_n ? n : max_n;
  for (int64_t c = blockIdx.x; c * kScanWg < n; c += gridDim.x) {  // (block-uniform)
    const int64_t i0 = c * kScanWg + (int64_t)threadIdx.x * kScanPer;
    unsigned long long s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) s += i0 + k < n ? v[i0 + k] : 0ull;
    unsigned long long tot;
    (void)block_excl_u64(s, &tot);
    if (threadIdx.x == 0) wg[c] = tot;
  }
}

__global__ void __launch_bounds__(kPBlock) k_scan_top(unsigned long long* __restrict__ wg, int64_t max_n,
                                                      long long* __restrict__ counts) {
  int64_t n = counts[4];
  n = n < max_n ? n : max_n;
  const int nwg = (int)((n + kScanWg - 1) / kScanWg);  // (the chunks that hold lines)
  unsigned long long carry = 0;
  for (int c0 = 0; c0 < nwg; c0 += kPBlock) {
    const int i = c0 + (int)threadIdx.x;
    const unsigned long long x = i < nwg ? wg[i] : 0ull;
    unsigned long long t;
    const unsigned long long ex = block_excl_u64(x, &t);
    if (i < nwg) wg[i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) {
    counts[0] = (long long)(carry >> kTokBits);                   // rows
    counts[1] = (long long)(carry & ((1ull << kTokBits) - 1ull));  // occurrences
  }
}

__global__ void __launch_bounds__(kPBlock) k_scan_apply(unsigned long long* __restrict__ v,
                                                        const long long* __restrict__ counts,
                                                        int64_t max_n,
                                                        const unsigned long long* __restrict__ wg) {
  int64_t n = counts[4];
  n = n < max_n ? n : max_n;
  for (int64_t c = blockIdx.x; c * kScanWg < n; c += gridDim.x) {  // (block-uniform)
    const int64_t i0 = c * kScanWg + (int64_t)threadIdx.x * kScanPer;
    unsigned long long x[kScanPer], s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      x[k] = i0 + k < n ? v[i0 + k] : 0ull;
      s += x[k];
    }
    unsigned long long tot;
    unsigned long long off = wg[c] + block_excl_u64(s, &tot);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      if (i0 + k < n) {
        const unsigned long long own = x[k];
        v[i0 + k] = off;  // exclusive prefix; (own's flag tells a row apart)
        off += own;
        if (!(own >> kTokBits)) v[i0 + k] |= 1ull << 63;  // no row
      }
    }
  }
}

__global__ void __launch_bounds__(kPBlock) k_line_emit(const char* __restrict__ text,
                                                       const u32* __restrict__ line_end,
                                                       const unsigned long long* __restrict__ lv,
                                                       TextParseArgs a) {
  int64_t nl = a.counts[4];
  nl = nl < a.max_lines ? nl : a.max_lines;
  const bool rows_ok = a.counts[0] <= a.max_rows && a.counts[1] <= a.max_nnz && a.counts[5] == 0;
  int mn = 0x7FFFFFFF, mx = 0;
  for (int64_t l = (int64_t)blockIdx.x * kPBlock + threadIdx.x; l < nl && rows_ok;
       l += (int64_t)gridDim.x * kPBlock) {
    if (lv[l] >> 63) continue;  // (no row)
    const unsigned long long off = lv[l];
    const int64_t row = (int64_t)(off >> kTokBits);
    int64_t o = (int64_t)(off & ((1ull << kTokBits) - 1ull));
    const int64_t o0 = o;
    int64_t s, e;
    line_span(line_end, l, s, e);
    ByteStream bs;
    bs.start(text, s);
    int64_t i = s;
    while (i < e && bs.at(i) != '\t') ++i;  // (a row: there is a TAB)
    a.labels[row] = dev_atof(text + s, text + i) > 0.0000001 ? 1.0f : 0.0f;
    // One forward pass over the tokens, from registers: a token ends at ' '
    // or the line end; part 0 (before the first ':') is the field id -- an
    // optionally signed decimal integer is accumulated on the fly, anything
    // else takes atof from memory --, part 1 (to the second ':') the feature
    // text, kept in two 64-bit words up to 16 bytes and hashed from them
    // (longer: hashed from memory), part 2 (the value) is ignored.
    int64_t q = ++i, c1 = -1;
    int part = 0, flen = 0;
    long long fval = 0;
    bool fneg = false, fsign = false, fdig = false, fslow = false;
    u64 w0 = 0, w1 = 0;
    for (; i <= e; ++i) {
      const char c = i < e ? bs.at(i) : ' ';
      if (c == ' ') {
        if (c1 >= 0) {  // a feature token (empty tokens have no ':')
          int n = flen;
          const int64_t fb = c1 + 1;
          auto byte_at = [&](int j) -> char {
            return (char)((j < 8 ? w0 >> (8 * j) : w1 >> (8 * (j - 8))) & 0xFF);
          };
          if (part == 1) {  // 2-part token: trailing '\r' (a CRLF line end) stripped
            if (n <= 16) {
              while (n > 0 && byte_at(n - 1) == '\r') --n;
            } else {
              while (n > 0 && text[fb + n - 1] == '\r') --n;
            }
          }
          u64 key;
          if (n <= 16) {
            const u64 mul = (0xc6a4a793ull << 32) + 0x5bd1e995ull;
            auto shift_mix = [](u64 v) { return v ^ (v >> 47); };
            u64 h = 0xc70f6907ull ^ ((u64)n * mul);
            if (n >= 8) {
              h ^= shift_mix(w0 * mul) * mul;
              h *= mul;
            }
            if (n >= 16) {
              h ^= shift_mix(w1 * mul) * mul;
              h *= mul;
            }
            const int rem = n & 7;
            if (rem) {
              h ^= (n >= 8 ? w1 : w0) & ((1ull << (8 * rem)) - 1ull);
              h *= mul;
            }
            h = shift_mix(h) * mul;
            key = shift_mix(h);
          } else {
            key = std_hash_bytes(text + fb, n);
          }
          a.fgid[o] = fslow ? (int32_t)dev_atof(text + q, text + c1)
                            : (int32_t)(fneg ? -fval : fval);
          a.keys[o] = key;
          ++o;
        }
        q = i + 1;
        c1 = -1;
        part = flen = 0;
        fval = 0;
        fneg = fsign = fdig = fslow = false;
        w0 = w1 = 0;
        continue;
      }
      if (part == 0) {
        if (c == ':') {
          part = 1;
          c1 = i;
        } else if (c >= '0' && c <= '9') {
          if (!fslow) {
            fval = fval * 10 + (c - '0');
            fslow = fval > 0x7FFFFFFFll;  // (beyond int32: atof from memory)
          }
          fdig = true;
        } else if ((c == '-' || c == '+') && !fdig && !fsign) {
          fsign = true;
          fneg = c == '-';
        } else if (!(is_space(c) && !fdig && !fsign)) {
          fslow = true;  // fraction, exponent, text...: atof from memory
        }
      } else if (part == 1) {
        if (c == ':') {
          part = 2;
        } else {
          if (flen < 8) w0 |= (u64)(unsigned char)c << (8 * flen);
          else if (flen < 16) w1 |= (u64)(unsigned char)c << (8 * (flen - 8));
          ++flen;
        }
      }
    }
    a.row_ptr[row + 1] = (int32_t)o;
    const long long rows = a.counts[0];
    if (row + 1 == rows - rows % a.row_mod) a.counts[6] = o;  // (the used rows' end)
    mn = min(mn, (int)(o - o0));
    mx = max(mx, (int)(o - o0));
  }
  // the rows' shortest / longest feature counts (fixed-width blocks go
  // field-major on the device)
  __shared__ int s_mn[kPBlock / kWave], s_mx[kPBlock / kWave];
  int wmn = mn, wmx = mx;
#pragma unroll
  for (int o2 = kWave / 2; o2 > 0; o2 >>= 1) {
    wmn = min(wmn, __shfl_xor(wmn, o2));
    wmx = max(wmx, __shfl_xor(wmx, o2));
  }
  if (threadIdx.x % kWave == 0) {
    s_mn[threadIdx.x / kWave] = wmn;
    s_mx[threadIdx.x / kWave] = wmx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int bmn = 0x7FFFFFFF, bmx = 0;
#pragma unroll
    for (int w = 0; w < kPBlock / kWave; ++w) {
      bmn = min(bmn, s_mn[w]);
      bmx = max(bmx, s_mx[w]);
    }
    if (bmx > 0 || bmn != 0x7FFFFFFF) {
      atomicMin(reinterpret_cast<long long*>(&a.counts[2]), (long long)bmn);
      atomicMax(reinterpret_cast<long long*>(&a.counts[3]), (long long)bmx);
    }
  }
}

__global__ void k_parse_init(long long* counts, int32_t* row_ptr) {
  counts[0] = counts[1] = counts[4] = counts[5] = counts[6] = 0;
  counts[2] = 0x7FFFFFFFll;
  counts[3] = 0;
  row_ptr[0] = 0;
}

}  // namespace

void launch_parse_text(const TextParseArgs& a, hipStream_t st) {
  if (a.n < 0 || a.n > 0xFFFFFFFFll) throw std::runtime_error("parse_text: block of 0 .. 4 GB");
  if (a.row_mod < 1) throw std::runtime_error("parse_text: row_mod >= 1");
  if (reinterpret_cast<uintptr_t>(a.text) & 15) throw std::runtime_error("parse_text: text must be 16-byte aligned");
  const int64_t nwg = (a.n + kWgBytes - 1) / kWgBytes;
  const int64_t max_lines = a.max_lines;
  if (a.ws_words < text_ws_words(a.n) || a.max_lines < text_max_lines(a.n))
    throw std::runtime_error("parse_text: workspace too small");
  // workspace: chunk counts | line ends | per-line values | scan totals
  u32* wg_cnt = reinterpret_cast<u32*>(a.ws);
  u32* line_end = wg_cnt + ((nwg + 3) & ~3ll);
  unsigned long long* lv = reinterpret_cast<unsigned long long*>(line_end + ((max_lines + 1 + 3) & ~3ll));
  unsigned long long* swg = lv + max_lines;
  hipLaunchKernelGGL(k_parse_init, dim3(1), dim3(1), 0, st, a.counts, a.row_ptr);
  if (a.n > 0) {
    hipLaunchKernelGGL(k_nl_count, dim3((unsigned)nwg), dim3(kPBlock), 0, st, a.text, a.n, wg_cnt);
    hipLaunchKernelGGL(k_nl_scan, dim3(1), dim3(1024), 0, st, wg_cnt, (int)nwg, a.text, a.n, line_end,
                       max_lines, a.counts);
    hipLaunchKernelGGL(k_nl_write, dim3((unsigned)nwg), dim3(kPBlock), 0, st, a.text, a.n, wg_cnt,
                       line_end, max_lines);
    // grid-stride kernels: at most 8 K workgroups (the lines are counted on the device)
    const unsigned lg = (unsigned)std::min<int64_t>((max_lines + kPBlock - 1) / kPBlock, 8192);
    hipLaunchKernelGGL(k_line_count, dim3(lg), dim3(kPBlock), 0, st, a.text, line_end, a.counts, lv,
                       max_lines);
    const unsigned sw = (unsigned)std::min<int64_t>((max_lines + kScanWg - 1) / kScanWg, 4096);
    hipLaunchKernelGGL(k_scan_reduce, dim3(sw), dim3(kPBlock), 0, st, lv, a.counts, max_lines, swg);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kPBlock), 0, st, swg, max_lines, a.counts);
    hipLaunchKernelGGL(k_scan_apply, dim3(sw), dim3(kPBlock), 0, st, lv, a.counts, max_lines, swg);
    hipLaunchKernelGGL(k_line_emit, dim3(lg), dim3(kPBlock), 0, st, a.text, line_end, lv, a);
  }
  XF_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace xflow
