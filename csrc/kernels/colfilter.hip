// colfilter.hip — columnar predicate evaluation + selection compaction.
//
// PG-Strom-style scan (BASELINE config 5): after an Arrow column lands in HBM
// (and is decompressed), evaluate lo <= v <= hi for every row and produce an
// Arrow-compatible selection bitmap (LSB-first, 64 rows per word) plus the
// selected-row count.  One lane per row, one wavefront per 64-row word: the
// predicate's __ballot IS the bitmap word, ANDed with the validity word, so
// the bitmap is written with one 8-byte store per wave and no atomics on the
// data path (one count atomic per workgroup).
//
// bitmap_to_indices turns the bitmap into a dense, ordered row-index list
// (three launches: per-block popcounts, single-block exclusive scan,
// per-block LDS scan + write), deterministic regardless of scheduling.
// Measured alternatives (2M words, 10% selected; profiles/r1t/): a one-launch
// decoupled look-back scan took 98 us (the status chain crosses the 8 XCD
// L2s) and a wave-wide bit-parallel emit 48 us (one 64-lane store
// instruction per word, mostly inactive lanes) vs 6 + 12 + 40 us here.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <mutex>
#include <utility>

#include "strom/strom.h"

namespace {

// Each wave takes U consecutive 64-row words per trip and issues all their
// loads before the first compare: U rows per lane in flight instead of one
// (round 2 trace: 3.75 TB/s with one load in flight per wave).
constexpr uint32_t kU = 4;

template <typename T>
__global__ __launch_bounds__(256) void filter_kernel(const T *__restrict__ v,
                                                     const uint64_t *__restrict__ valid,
                                                     uint64_t n, T lo, T hi,
                                                     uint64_t *__restrict__ bitmap,
                                                     unsigned long long *__restrict__ count) {
  __shared__ uint32_t wave_cnt[4];
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t nwords = (n + 63) / 64;
  uint32_t local = 0;
  const uint64_t step = (uint64_t)gridDim.x * 4 * kU;
  for (uint64_t w0 = ((uint64_t)blockIdx.x * 4 + wid) * kU; w0 < nwords; w0 += step) {
    T x[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint64_t i = (w0 + u) * 64 + lane;
      x[u] = i < n ? __builtin_nontemporal_load(v + i) : (T)0;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint64_t w = w0 + u;
      if (w >= nwords) break;
      const uint64_t i = w * 64 + lane;
      uint64_t word = __ballot(i < n && x[u] >= lo && x[u] <= hi);
      if (valid) word &= valid[w];
      if (lane == 0) bitmap[w] = word;
      local += __popcll(word);
    }
  }
  if (lane == 0) wave_cnt[wid] = local;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicAdd(count, (unsigned long long)(wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3]));
}

constexpr uint32_t kWordsPerBlock = 256;

__global__ __launch_bounds__(256) void block_popc_kernel(const uint64_t *__restrict__ bm,
                                                         uint64_t nwords,
                                                         uint32_t *__restrict__ block_cnt) {
  __shared__ uint32_t s[4];
  uint64_t w = (uint64_t)blockIdx.x * kWordsPerBlock + threadIdx.x;
  uint32_t c = w < nwords ? __popcll(bm[w]) : 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) block_cnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// exclusive scan of block counts in one workgroup (sequential chunks per thread)
__global__ __launch_bounds__(1024) void scan_blocks_kernel(uint32_t *__restrict__ cnt, uint32_t nb,
                                                           unsigned long long *__restrict__ total) {
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (nb + 1023) / 1024;
  const uint32_t lo = min(nb, t * per), hi = min(nb, lo + per);
  uint64_t s = 0;
  for (uint32_t i = lo; i < hi; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    uint64_t add = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += add;
    __syncthreads();
  }
  uint64_t run = t ? part[t - 1] : 0;
  for (uint32_t i = lo; i < hi; ++i) {
    uint32_t c = cnt[i];
    cnt[i] = (uint32_t)run;
    run += c;
  }
  if (t == 1023) *total = part[1023];
}

__global__ __launch_bounds__(256) void emit_indices_kernel(const uint64_t *__restrict__ bm,
                                                           uint64_t nwords, uint64_t n,
                                                           const uint32_t *__restrict__ base,
                                                           uint32_t *__restrict__ out) {
  __shared__ uint32_t s[256];
  uint64_t w = (uint64_t)blockIdx.x * kWordsPerBlock + threadIdx.x;
  uint64_t word = w < nwords ? bm[w] : 0;
  if (w == nwords - 1 && (n & 63)) word &= (1ull << (n & 63)) - 1;
  uint32_t c = __popcll(word);
  s[threadIdx.x] = c;
  __syncthreads();
  for (uint32_t off = 1; off < 256; off <<= 1) {
    uint32_t add = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
    __syncthreads();
    s[threadIdx.x] += add;
    __syncthreads();
  }
  uint32_t pos = base[blockIdx.x] + s[threadIdx.x] - c;
  while (word) {
    uint32_t b = __ffsll((unsigned long long)word) - 1;
    out[pos++] = (uint32_t)(w * 64 + b);
    word &= word - 1;
  }
}

// ---------------------------------------------------------------- batched
// batch of bitmap word w: the last b with word_base <= w (uniform per wave)
template <typename B>
__device__ __forceinline__ uint32_t batch_of(const B *b, uint32_t nb, uint64_t w) {
  uint32_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (b[mid].word_base <= w) lo = mid;
    else hi = mid;
  }
  return lo;
}

// combine: AND the predicate into the existing bitmap (a qualifier list:
// the first column writes the words, later ones narrow them); the count is
// of the combined words, so the last qualifier's count is the selection's
template <typename T>
__global__ __launch_bounds__(256) void filter_batched_kernel(const strom_filter_batch *__restrict__ bt,
                                                             uint32_t nb, uint64_t nwords, T lo,
                                                             T hi, uint64_t *__restrict__ bitmap,
                                                             unsigned long long *__restrict__ count,
                                                             int combine) {
  __shared__ uint32_t wave_cnt[4];
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t local = 0;
  const uint64_t step = (uint64_t)gridDim.x * 4 * kU;
  for (uint64_t w0 = ((uint64_t)blockIdx.x * 4 + wid) * kU; w0 < nwords; w0 += step) {
    // U words per trip, all loads issued first (as filter_kernel)
    T x[kU];
    uint32_t bi[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint64_t w = w0 + u;
      x[u] = (T)0;
      bi[u] = 0;
      if (w < nwords) {
        bi[u] = batch_of(bt, nb, w);
        const strom_filter_batch &b = bt[bi[u]];
        const uint64_t i = (w - b.word_base) * 64 + lane;
        if (i < b.nrows) x[u] = ((const T *)b.values)[i];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint64_t w = w0 + u;
      if (w >= nwords) break;
      const strom_filter_batch b = bt[bi[u]];
      const uint64_t k = w - b.word_base;           // word within the batch
      const uint64_t i = k * 64 + lane;
      uint64_t word = __ballot(i < b.nrows && x[u] >= lo && x[u] <= hi);
      if (b.valid && k * 64 < b.nrows) word &= ((const uint64_t *)b.valid)[k];
      if (combine) word &= bitmap[w];                 // uniform load, one per wave
      if (lane == 0) bitmap[w] = word;
      local += __popcll(word);
    }
  }
  if (lane == 0) wave_cnt[wid] = local;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicAdd(count, (unsigned long long)(wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3]));
}

// like scan_blocks_kernel, offset by the running output cursor, which it
// then advances (one workgroup: every thread reads the cursor before the
// first barrier, thread 1023 writes it after the last)
__global__ __launch_bounds__(1024) void scan_blocks_cursor_kernel(uint64_t *__restrict__ cnt,
                                                                  uint32_t nb,
                                                                  unsigned long long *__restrict__ cursor) {
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t base = *cursor;
  const uint32_t per = (nb + 1023) / 1024;
  const uint32_t lo = min(nb, t * per), hi = min(nb, lo + per);
  uint64_t s = 0;
  for (uint32_t i = lo; i < hi; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    uint64_t add = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += add;
    __syncthreads();
  }
  uint64_t run = base + (t ? part[t - 1] : 0);
  for (uint32_t i = lo; i < hi; ++i) {
    const uint64_t c = cnt[i];
    cnt[i] = run;
    run += c;
  }
  if (t == 1023) *cursor = base + part[1023];
}

__global__ __launch_bounds__(256) void block_popc64_kernel(const uint64_t *__restrict__ bm,
                                                           uint64_t nwords,
                                                           uint64_t *__restrict__ block_cnt) {
  __shared__ uint32_t s[4];
  uint64_t w = (uint64_t)blockIdx.x * kWordsPerBlock + threadIdx.x;
  uint32_t c = w < nwords ? __popcll(bm[w]) : 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) block_cnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// W: bytes per projected value (0: no projection).  With a projection the
// selected rows' values of another column (its own per-batch pointers in
// `pt`, same batches) are gathered next to the row ids, plus a 0/1 validity
// byte when that column has nulls: PG-Strom's projection of the qualifying
// tuples, done while the ids are written.
template <uint32_t W>
__global__ __launch_bounds__(256) void emit_rows_kernel(const uint64_t *__restrict__ bm,
                                                        uint64_t nwords,
                                                        const strom_filter_batch *__restrict__ bt,
                                                        uint32_t nb,
                                                        const uint64_t *__restrict__ base,
                                                        int64_t *__restrict__ out,
                                                        const strom_filter_batch *__restrict__ pt,
                                                        void *__restrict__ pout,
                                                        uint8_t *__restrict__ pvalid) {
  __shared__ uint32_t s[256];
  const uint64_t w = (uint64_t)blockIdx.x * kWordsPerBlock + threadIdx.x;
  uint64_t word = w < nwords ? bm[w] : 0;
  const uint32_t c = __popcll(word);
  s[threadIdx.x] = c;
  __syncthreads();
  for (uint32_t off = 1; off < 256; off <<= 1) {
    uint32_t add = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
    __syncthreads();
    s[threadIdx.x] += add;
    __syncthreads();
  }
  if (!word) return;
  uint64_t pos = base[blockIdx.x] + s[threadIdx.x] - c;
  const uint32_t bi = batch_of(bt, nb, w);
  const strom_filter_batch b = bt[bi];
  const uint64_t local0 = (w - b.word_base) * 64;
  const int64_t row0 = (int64_t)(b.row_base + local0);
  const uint8_t *pv = nullptr, *pval = nullptr;
  if (W) {
    pv = (const uint8_t *)pt[bi].values;
    pval = (const uint8_t *)pt[bi].valid;
  }
  while (word) {
    const uint32_t bit = __ffsll((unsigned long long)word) - 1;
    out[pos] = row0 + bit;
    if (W) {
      const uint64_t r = local0 + bit;
      if (W == 16) {
        ((uint64_t *)pout)[2 * pos] = ((const uint64_t *)pv)[2 * r];
        ((uint64_t *)pout)[2 * pos + 1] = ((const uint64_t *)pv)[2 * r + 1];
      } else if (W == 8) ((uint64_t *)pout)[pos] = ((const uint64_t *)pv)[r];
      else if (W == 4) ((uint32_t *)pout)[pos] = ((const uint32_t *)pv)[r];
      else if (W == 2) ((uint16_t *)pout)[pos] = ((const uint16_t *)pv)[r];
      else ((uint8_t *)pout)[pos] = pv[r];
      if (pvalid) pvalid[pos] = pval ? (pval[r >> 3] >> (r & 7)) & 1 : 1;
    }
    ++pos;
    word &= word - 1;
  }
}

// ------------------------------------------------------------ string projection
// A selected row's characters (offsets OT of a utf8/binary column, the
// characters in aux): a malformed offset pair gives an empty string, never
// a read outside the buffer (as the qualifier kernel).
template <typename OT>
__device__ __forceinline__ void str_span(const strom_qual_batch &b, uint64_t r, uint64_t &s,
                                         uint32_t &len) {
  const int64_t a = (int64_t)((const OT *)b.values)[r];
  const int64_t e = (int64_t)((const OT *)b.values)[r + 1];
  const bool ok = a >= 0 && e >= a && (uint64_t)e <= b.aux_len;
  s = ok ? (uint64_t)a : 0;
  len = ok ? (uint32_t)(e - a) : 0;
}

// per 256-word block: characters of the selected rows (the weights of the
// character cursor scan, as block_popc64_kernel's counts are of the rows)
template <typename OT>
__global__ __launch_bounds__(256) void block_chars_kernel(const uint64_t *__restrict__ bm,
                                                          uint64_t nwords,
                                                          const strom_qual_batch *__restrict__ pt,
                                                          uint32_t nb,
                                                          uint64_t *__restrict__ block_sum) {
  __shared__ uint64_t red[256];
  const uint64_t w = (uint64_t)blockIdx.x * kWordsPerBlock + threadIdx.x;
  uint64_t word = w < nwords ? bm[w] : 0, sum = 0;
  if (word) {
    const strom_qual_batch b = pt[batch_of(pt, nb, w)];
    const uint64_t local0 = (w - b.word_base) * 64;
    while (word) {
      const uint32_t bit = __ffsll((unsigned long long)word) - 1;
      uint64_t st;
      uint32_t len;
      str_span<OT>(b, local0 + bit, st, len);
      sum += len;
      word &= word - 1;
    }
  }
  red[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) block_sum[blockIdx.x] = red[0];
}

// row ids (as emit_rows_kernel) + each selected row's characters appended
// at the character cursor: poff[pos] = its start, the bytes in pchars
template <typename OT>
__global__ __launch_bounds__(256) void emit_str_kernel(const uint64_t *__restrict__ bm,
                                                       uint64_t nwords,
                                                       const strom_qual_batch *__restrict__ pt,
                                                       uint32_t nb,
                                                       const uint64_t *__restrict__ rbase,
                                                       const uint64_t *__restrict__ cbase,
                                                       int64_t *__restrict__ out,
                                                       int64_t *__restrict__ poff,
                                                       uint8_t *__restrict__ pchars,
                                                       uint8_t *__restrict__ pvalid) {
  __shared__ uint32_t rs[256];
  __shared__ uint64_t cs[256];
  const uint64_t w = (uint64_t)blockIdx.x * kWordsPerBlock + threadIdx.x;
  uint64_t word = w < nwords ? bm[w] : 0;
  const uint32_t c = __popcll(word);
  uint64_t chars = 0;
  strom_qual_batch b{};
  uint64_t local0 = 0;
  if (word) {
    b = pt[batch_of(pt, nb, w)];
    local0 = (w - b.word_base) * 64;
    for (uint64_t x = word; x; x &= x - 1) {
      uint64_t st;
      uint32_t len;
      str_span<OT>(b, local0 + (__ffsll((unsigned long long)x) - 1), st, len);
      chars += len;
    }
  }
  rs[threadIdx.x] = c;
  cs[threadIdx.x] = chars;
  __syncthreads();
  for (uint32_t off = 1; off < 256; off <<= 1) {
    const uint32_t ra = threadIdx.x >= off ? rs[threadIdx.x - off] : 0;
    const uint64_t ca = threadIdx.x >= off ? cs[threadIdx.x - off] : 0;
    __syncthreads();
    rs[threadIdx.x] += ra;
    cs[threadIdx.x] += ca;
    __syncthreads();
  }
  if (!word) return;
  uint64_t pos = rbase[blockIdx.x] + rs[threadIdx.x] - c;
  uint64_t cp = cbase[blockIdx.x] + cs[threadIdx.x] - chars;
  const int64_t row0 = (int64_t)(b.row_base + local0);
  const uint8_t *val = (const uint8_t *)b.valid;
  while (word) {
    const uint32_t bit = __ffsll((unsigned long long)word) - 1;
    const uint64_t r = local0 + bit;
    uint64_t st;
    uint32_t len;
    str_span<OT>(b, r, st, len);
    out[pos] = row0 + bit;
    poff[pos] = (int64_t)cp;
    const uint8_t *src = (const uint8_t *)b.aux + st;
    for (uint32_t k = 0; k < len; ++k) pchars[cp + k] = src[k];
    if (pvalid) pvalid[pos] = val ? (val[r >> 3] >> (r & 7)) & 1 : 1;
    cp += len;
    ++pos;
    word &= word - 1;
  }
}

template <typename T>
int launch_filter_batched(const strom_filter_batch *bt, uint32_t nb, uint64_t nwords, double lo,
                          double hi, uint64_t *bm, uint64_t *cnt, int combine, hipStream_t st) {
  uint64_t g = (nwords + 4 * kU - 1) / (4 * kU);
  uint32_t grid = (uint32_t)(g > 8192 ? 8192 : (g ? g : 1));
  hipLaunchKernelGGL(filter_batched_kernel<T>, dim3(grid), dim3(256), 0, st, bt, nb, nwords, (T)lo,
                     (T)hi, bm, (unsigned long long *)cnt, combine);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

template <typename T>
int launch_filter(const void *v, const uint8_t *valid, uint64_t n, double lo, double hi,
                  uint64_t *bm, uint64_t *cnt, hipStream_t st) {
  uint64_t words = (n + 63) / 64;
  uint64_t g = (words + 4 * kU - 1) / (4 * kU);
  uint32_t grid = (uint32_t)(g > 4096 ? 4096 : (g ? g : 1));
  (void)hipMemsetAsync(cnt, 0, sizeof(uint64_t), st);
  hipLaunchKernelGGL(filter_kernel<T>, dim3(grid), dim3(256), 0, st, (const T *)v,
                     (const uint64_t *)valid, n, (T)lo, (T)hi, bm, (unsigned long long *)cnt);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}


// ------------------------------------------------------------ qualifiers
// General predicates of an Arrow scan (strom_column_qual): one lane per row,
// one wave per 64-row word, as filter_batched_kernel, with the predicate's
// constants (ranges, string constants, a dictionary lookup table) staged
// once per workgroup in LDS.  The written word is
// (pred | or_src[w]) & (and_dst ? bitmap[w] : ~0): a CNF qualifier list is a
// chain of launches, ORs inside a clause and ANDs across clauses, no
// per-clause bitmaps beyond one scratch.
enum QKind { QK_RANGE, QK_LUT, QK_STR, QK_VALID };

template <typename T> struct CmpOf { typedef int64_t type; };
template <> struct CmpOf<uint64_t> { typedef uint64_t type; };
template <> struct CmpOf<float> { typedef double type; };
template <> struct CmpOf<double> { typedef double type; };

struct BitT {};   // STROM_COL_BOOL: one bit per row
template <> struct CmpOf<BitT> { typedef int64_t type; };
struct Dec128T {};   // STROM_COL_DEC128: 16-byte little-endian two's complement
template <> struct CmpOf<Dec128T> { typedef __int128 type; };

template <typename T>
__device__ __forceinline__ typename CmpOf<T>::type qload(const strom_qual_batch &b, uint64_t i) {
  return (typename CmpOf<T>::type)((const T *)b.values)[i];
}
template <>
__device__ __forceinline__ int64_t qload<BitT>(const strom_qual_batch &b, uint64_t i) {
  return (((const uint8_t *)b.values)[i >> 3] >> (i & 7)) & 1;
}
template <>
__device__ __forceinline__ __int128 qload<Dec128T>(const strom_qual_batch &b, uint64_t i) {
  const uint64_t *p = (const uint64_t *)b.values + 2 * i;   // Arrow buffers: 8-byte aligned
  return (__int128)(((unsigned __int128)(uint64_t)p[1] << 64) | p[0]);
}

// sorted disjoint inclusive ranges in LDS: linear for a few, else a binary
// search for the first range whose hi >= x (NaN: no range)
template <typename CT>
__device__ __forceinline__ bool in_ranges(CT x, const CT *r, uint32_t n) {
  if (n <= 8) {
    bool h = false;
    for (uint32_t k = 0; k < n; ++k) h |= (x >= r[2 * k]) & (x <= r[2 * k + 1]);
    return h;
  }
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (r[2 * mid + 1] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && r[2 * lo] <= x;
}

template <typename CT> __device__ __forceinline__ bool is_nan(CT) { return false; }
template <> __device__ __forceinline__ bool is_nan<double>(double x) { return x != x; }

// len bytes at global p == the LDS constant c (4-aligned).  Whole dwords:
// aligned loads funnel-shifted into place (v_alignbyte), never reading a
// dword that holds no byte of the string, so no access past the buffer.
__device__ __forceinline__ bool str_eq(const uint8_t *p, const uint32_t *c, uint32_t len) {
  if (!len) return true;
  const uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  const uint32_t *last = (const uint32_t *)((a + len - 1) & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  uint32_t cur = *w;
  for (uint32_t j = 0; j < len; j += 4) {
    const uint32_t *nx = w + 1 <= last ? w + 1 : last;
    const uint32_t nxt = *nx;
    const uint32_t v = __builtin_amdgcn_alignbyte(nxt, cur, sh);
    const uint32_t rem = len - j;
    const uint32_t m = rem >= 4 ? ~0u : (1u << (8 * rem)) - 1;
    if ((v ^ c[j >> 2]) & m) return false;
    cur = nxt;
    ++w;
  }
  return true;
}

// bytewise-lexicographic compare of len bytes at global p with the LDS
// constant c of clen bytes: <0, 0, >0 (dwords compared big-endian)
__device__ __forceinline__ int str_cmp(const uint8_t *p, uint32_t len, const uint32_t *c,
                                       uint32_t clen) {
  const uint32_t n = len < clen ? len : clen;
  if (n) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t *last = (const uint32_t *)((a + n - 1) & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t cur = *w;
    for (uint32_t j = 0; j < n; j += 4) {
      const uint32_t *nx = w + 1 <= last ? w + 1 : last;
      const uint32_t nxt = *nx;
      const uint32_t rem = n - j;
      const uint32_t m = rem >= 4 ? ~0u : (1u << (8 * rem)) - 1;
      const uint32_t v = __builtin_amdgcn_alignbyte(nxt, cur, sh) & m;
      const uint32_t k = c[j >> 2] & m;
      if (v != k) return __builtin_bswap32(v) < __builtin_bswap32(k) ? -1 : 1;
      cur = nxt;
      ++w;
    }
  }
  return len < clen ? -1 : (len > clen ? 1 : 0);
}

// one bound of a string range: offs (start, len, mode); mode 0 unbounded
__device__ __forceinline__ bool str_bound(const uint8_t *p, uint32_t len, const uint32_t *qs,
                                          const uint32_t *b, bool upper) {
  const uint32_t mode = b[2];
  if (!mode) return true;
  const int r = str_cmp(p, len, qs + b[0] / 4, b[1]);
  if (upper) return mode == 1 ? r <= 0 : r < 0;
  return mode == 1 ? r >= 0 : r > 0;
}

template <typename T, int K>
__global__ __launch_bounds__(256) void qual_kernel(strom_col_qual q,
                                                   const strom_qual_batch *__restrict__ bt,
                                                   uint32_t nb, uint64_t nwords,
                                                   uint64_t *__restrict__ bitmap,
                                                   const uint64_t *__restrict__ or_src, int and_dst,
                                                   unsigned long long *__restrict__ count) {
  typedef typename CmpOf<T>::type CT;
  extern __shared__ __attribute__((aligned(16))) uint32_t qs[];
  __shared__ uint32_t wave_cnt[4];
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // constants -> LDS (consts, then the string (start, len) pairs)
  const uint32_t cw = (uint32_t)(q.const_bytes / 4), ow = (uint32_t)(q.offs_bytes / 4);
  if (K != QK_VALID) {
    for (uint32_t k = threadIdx.x; k < cw; k += 256) qs[k] = ((const uint32_t *)q.consts)[k];
    if (K == QK_STR)
      for (uint32_t k = threadIdx.x; k < ow; k += 256) qs[cw + k] = ((const uint32_t *)q.offs)[k];
  }
  __syncthreads();
  const bool neg = q.flags & STROM_QUAL_NEGATE;
  const bool nan_hit = q.flags & STROM_QUAL_NAN;
  uint32_t local = 0;
  constexpr uint32_t U = K == QK_STR ? 1 : kU;
  const uint64_t step = (uint64_t)gridDim.x * 4 * U;
  for (uint64_t w0 = ((uint64_t)blockIdx.x * 4 + wid) * U; w0 < nwords; w0 += step) {
    // pass 1: batch lookup + every lane's load of U words issued before the
    // first compare (kU rows per lane in flight, as filter_batched_kernel)
    bool hit[U];
    uint32_t bi[U];
    CT x[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t w = w0 + u;
      hit[u] = false;
      bi[u] = 0;
      x[u] = 0;
      if (w >= nwords) continue;
      uint32_t lo = 0, hi = nb;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (bt[mid].word_base <= w) lo = mid;
        else hi = mid;
      }
      bi[u] = lo;
      const strom_qual_batch &b = bt[lo];
      const uint64_t i = (w - b.word_base) * 64 + lane;
      if constexpr (K == QK_RANGE || K == QK_LUT)
        if (i < b.nrows) x[u] = qload<T>(b, i);
    }
    // pass 2: the predicate
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t w = w0 + u;
      if (w >= nwords) break;
      const strom_qual_batch &b = bt[bi[u]];
      const uint64_t i = (w - b.word_base) * 64 + lane;
      if (i >= b.nrows || K == QK_VALID) continue;
      if constexpr (K == QK_RANGE) {
        hit[u] = in_ranges<CT>(x[u], (const CT *)qs, q.nconst) || (nan_hit && is_nan<CT>(x[u]));
      } else if constexpr (K == QK_LUT) {
        const int64_t v = (int64_t)x[u];
        hit[u] = (uint64_t)v < q.nconst && ((qs[v >> 5] >> (v & 31)) & 1);
      } else {   // QK_STR: T is the offset type
        const int64_t s = (int64_t)((const T *)b.values)[i];
        const int64_t e = (int64_t)((const T *)b.values)[i + 1];
        // a malformed offset pair (file data) never matches and is never
        // followed outside the character buffer
        if (s < 0 || e < s || (uint64_t)e > b.aux_len) continue;
        const uint32_t len = (uint32_t)(e - s);
        const uint8_t *p = (const uint8_t *)b.aux + s;
        const uint32_t *offs = qs + cw;
        bool h = false;
        if (q.op == STROM_QOP_STR_RANGES) {
          for (uint32_t k = 0; k < q.nconst && !h; ++k)
            h = str_bound(p, len, qs, offs + 6 * k, false) &&
                str_bound(p, len, qs, offs + 6 * k + 3, true);
        } else {
          const bool prefix = q.op == STROM_QOP_STR_PREFIX;
          for (uint32_t k = 0; k < q.nconst && !h; ++k) {
            const uint32_t cl = offs[2 * k + 1];
            if (prefix ? len >= cl : len == cl) h = str_eq(p, qs + offs[2 * k] / 4, cl);
          }
        }
        hit[u] = h;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t w = w0 + u;
      if (w >= nwords) break;
      const strom_qual_batch &b = bt[bi[u]];
      const uint64_t k = w - b.word_base;
      const uint64_t i = k * 64 + lane;
      const uint64_t vword = b.valid ? ((const uint64_t *)b.valid)[k] : ~0ull;
      uint64_t word;
      if (K == QK_VALID) word = __ballot(i < b.nrows && (((vword >> lane) & 1) != neg));
      else word = __ballot(i < b.nrows && (hit[u] != neg)) & vword;
      if (or_src) word |= or_src[w];
      if (and_dst) word &= bitmap[w];
      if (lane == 0) bitmap[w] = word;
      local += __popcll(word);
    }
  }
  if (lane == 0) wave_cnt[wid] = local;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicAdd(count, (unsigned long long)(wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3]));
}

template <typename T, int K>
int launch_qual(const strom_col_qual &q, const strom_qual_batch *bt, uint32_t nb, uint64_t nwords,
                uint64_t *bm, const uint64_t *orv, int and_dst, uint64_t *cnt, hipStream_t st) {
  const uint32_t U = K == QK_STR ? 1 : kU;
  uint64_t g = (nwords + 4 * U - 1) / (4 * U);
  uint32_t grid = (uint32_t)(g > 8192 ? 8192 : (g ? g : 1));
  const size_t lds = K == QK_VALID ? 0 : (size_t)(q.const_bytes + (K == QK_STR ? q.offs_bytes : 0));
  hipLaunchKernelGGL((qual_kernel<T, K>), dim3(grid), dim3(256), lds, st, q, bt, nb, nwords, bm, orv,
                     and_dst, (unsigned long long *)cnt);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

template <int K>
int qual_by_type(const strom_col_qual &q, const strom_qual_batch *bt, uint32_t nb, uint64_t nw,
                 uint64_t *bm, const uint64_t *orv, int and_dst, uint64_t *cnt, hipStream_t st) {
  switch (q.type) {
    case STROM_COL_I8: return launch_qual<int8_t, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
    case STROM_COL_I16: return launch_qual<int16_t, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
    case STROM_COL_I32: return launch_qual<int32_t, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
    case STROM_COL_I64: return launch_qual<int64_t, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
    case STROM_COL_U8: return launch_qual<uint8_t, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
    case STROM_COL_U16: return launch_qual<uint16_t, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
    case STROM_COL_U32: return launch_qual<uint32_t, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
    case STROM_COL_U64: return launch_qual<uint64_t, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
    default: break;
  }
  if constexpr (K == QK_RANGE) {
    switch (q.type) {
      case STROM_COL_F32: return launch_qual<float, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
      case STROM_COL_F64: return launch_qual<double, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
      case STROM_COL_BOOL: return launch_qual<BitT, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
      case STROM_COL_DEC128: return launch_qual<Dec128T, K>(q, bt, nb, nw, bm, orv, and_dst, cnt, st);
      default: break;
    }
  }
  return -22;
}


// Block-count scratch of the emit launches, kept per (device, stream) and
// grown on demand.  Stream-ordered reuse on one stream is safe; hipMallocAsync
// / hipFreeAsync were not free: the host blocked in them until the stream's
// queued work had drained (r5 Arrow ZSTD timeline: group k+1's emit waited
// ~20 ms for its own decode, so the next group's launches queued late).
struct ColScratch {
  void *p = nullptr;
  size_t bytes = 0;
  uint64_t used = 0;                  // LRU clock
};
std::mutex g_cs_mu;
std::map<std::pair<int, void *>, ColScratch> g_cs;
uint64_t g_cs_clock = 0;
constexpr size_t kColScratchKeep = 64;   // streams kept (a caller cycling through
                                         // more evicts the least recently used)

// under g_cs_mu, held by the caller through its launches
void *col_scratch(hipStream_t st, size_t bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const std::pair<int, void *> key{dev, (void *)st};
  if (!g_cs.count(key) && g_cs.size() >= kColScratchKeep) {
    auto lru = g_cs.begin();
    for (auto j = g_cs.begin(); j != g_cs.end(); ++j)
      if (j->second.used < lru->second.used) lru = j;
    // its stream may still read it (hipFree waits for the device's work)
    if (lru->second.p) (void)hipFree(lru->second.p);
    g_cs.erase(lru);
  }
  ColScratch &c = g_cs[key];
  c.used = ++g_cs_clock;
  auto &e = c;
  if (e.bytes < bytes) {
    // the old buffer may still be read by this stream's queued launches
    if (e.p && (hipStreamSynchronize(st) != hipSuccess || hipFree(e.p) != hipSuccess))
      return nullptr;
    e.p = nullptr;
    e.bytes = 0;
    const size_t want = bytes < (64u << 10) ? (64u << 10) : bytes;
    void *p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess) return nullptr;
    e.p = p;
    e.bytes = want;
  }
  return e.p;
}

}  // namespace

extern "C" int strom_column_filter(int type, const void *d_values, const uint8_t *d_valid,
                                   uint64_t n, double lo, double hi, uint64_t *d_bitmap,
                                   uint64_t *d_count, void *stream) {
  if (!n) return 0;
  if (((uintptr_t)d_valid & 7) || ((uintptr_t)d_bitmap & 7)) return -22;
  hipStream_t st = (hipStream_t)stream;
  switch (type) {
    case STROM_COL_I32: return launch_filter<int32_t>(d_values, d_valid, n, lo, hi, d_bitmap, d_count, st);
    case STROM_COL_I64: return launch_filter<int64_t>(d_values, d_valid, n, lo, hi, d_bitmap, d_count, st);
    case STROM_COL_F32: return launch_filter<float>(d_values, d_valid, n, lo, hi, d_bitmap, d_count, st);
    case STROM_COL_F64: return launch_filter<double>(d_values, d_valid, n, lo, hi, d_bitmap, d_count, st);
    default: return -22;
  }
}

// d_out needs room for every selected row; d_count receives the total.
// The block counts live in the library-kept per-stream scratch (col_scratch).
extern "C" int strom_bitmap_to_indices(const uint64_t *d_bitmap, uint64_t n, uint32_t *d_out,
                                       uint64_t *d_count, void *stream) {
  if (!n) return 0;
  if (n > 0xffffffffull) return -75;  // row indices are 32-bit
  hipStream_t st = (hipStream_t)stream;
  uint64_t words = (n + 63) / 64;
  uint32_t nb = (uint32_t)((words + kWordsPerBlock - 1) / kWordsPerBlock);
  std::lock_guard<std::mutex> g(g_cs_mu);
  uint32_t *cnt = (uint32_t *)col_scratch(st, sizeof(uint32_t) * nb);
  if (!cnt) return -12;
  hipLaunchKernelGGL(block_popc_kernel, dim3(nb), dim3(256), 0, st, d_bitmap, words, cnt);
  hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(1024), 0, st, cnt, nb,
                     (unsigned long long *)d_count);
  hipLaunchKernelGGL(emit_indices_kernel, dim3(nb), dim3(256), 0, st, d_bitmap, words, n, cnt, d_out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int strom_column_filter_batched2(int type, const strom_filter_batch *d_batches,
                                            uint32_t nbatches, uint64_t nwords, double lo,
                                            double hi, uint64_t *d_bitmap, uint64_t *d_count,
                                            int combine, void *stream) {
  if (!nbatches || !nwords) return 0;
  if (!d_batches || !d_bitmap || !d_count || ((uintptr_t)d_bitmap & 7)) return -22;
  hipStream_t st = (hipStream_t)stream;
  switch (type) {
    case STROM_COL_I32: return launch_filter_batched<int32_t>(d_batches, nbatches, nwords, lo, hi, d_bitmap, d_count, combine, st);
    case STROM_COL_I64: return launch_filter_batched<int64_t>(d_batches, nbatches, nwords, lo, hi, d_bitmap, d_count, combine, st);
    case STROM_COL_F32: return launch_filter_batched<float>(d_batches, nbatches, nwords, lo, hi, d_bitmap, d_count, combine, st);
    case STROM_COL_F64: return launch_filter_batched<double>(d_batches, nbatches, nwords, lo, hi, d_bitmap, d_count, combine, st);
    default: return -22;
  }
}

extern "C" int strom_column_filter_batched(int type, const strom_filter_batch *d_batches,
                                           uint32_t nbatches, uint64_t nwords, double lo,
                                           double hi, uint64_t *d_bitmap, uint64_t *d_count,
                                           void *stream) {
  return strom_column_filter_batched2(type, d_batches, nbatches, nwords, lo, hi, d_bitmap,
                                      d_count, 0, stream);
}

extern "C" int strom_bitmap_to_rows_proj(const uint64_t *d_bitmap, uint64_t nwords,
                                         const strom_filter_batch *d_batches, uint32_t nbatches,
                                         int64_t *d_out, uint64_t *d_total,
                                         const strom_filter_batch *d_proj, uint32_t width,
                                         void *d_pout, uint8_t *d_pvalid, void *stream) {
  if (!nwords || !nbatches) return 0;
  if (!d_bitmap || !d_batches || !d_out || !d_total) return -22;
  if (d_proj && ((width != 1 && width != 2 && width != 4 && width != 8 && width != 16) || !d_pout))
    return -22;
  hipStream_t st = (hipStream_t)stream;
  const uint64_t nb64 = (nwords + kWordsPerBlock - 1) / kWordsPerBlock;
  if (nb64 > 0xffffffffull) return -75;
  const uint32_t nb = (uint32_t)nb64;
  std::lock_guard<std::mutex> g(g_cs_mu);
  uint64_t *cnt = (uint64_t *)col_scratch(st, sizeof(uint64_t) * nb);
  if (!cnt) return -12;
  hipLaunchKernelGGL(block_popc64_kernel, dim3(nb), dim3(256), 0, st, d_bitmap, nwords, cnt);
  hipLaunchKernelGGL(scan_blocks_cursor_kernel, dim3(1), dim3(1024), 0, st, cnt, nb,
                     (unsigned long long *)d_total);
  if (!d_proj)
    hipLaunchKernelGGL(emit_rows_kernel<0>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords, d_batches,
                       nbatches, cnt, d_out, nullptr, nullptr, nullptr);
  else if (width == 16)
    hipLaunchKernelGGL(emit_rows_kernel<16>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords, d_batches,
                       nbatches, cnt, d_out, d_proj, d_pout, d_pvalid);
  else if (width == 8)
    hipLaunchKernelGGL(emit_rows_kernel<8>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords, d_batches,
                       nbatches, cnt, d_out, d_proj, d_pout, d_pvalid);
  else if (width == 4)
    hipLaunchKernelGGL(emit_rows_kernel<4>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords, d_batches,
                       nbatches, cnt, d_out, d_proj, d_pout, d_pvalid);
  else if (width == 2)
    hipLaunchKernelGGL(emit_rows_kernel<2>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords, d_batches,
                       nbatches, cnt, d_out, d_proj, d_pout, d_pvalid);
  else
    hipLaunchKernelGGL(emit_rows_kernel<1>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords, d_batches,
                       nbatches, cnt, d_out, d_proj, d_pout, d_pvalid);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int strom_bitmap_to_rows(const uint64_t *d_bitmap, uint64_t nwords,
                                    const strom_filter_batch *d_batches, uint32_t nbatches,
                                    int64_t *d_out, uint64_t *d_total, void *stream) {
  return strom_bitmap_to_rows_proj(d_bitmap, nwords, d_batches, nbatches, d_out, d_total, nullptr,
                                   0, nullptr, nullptr, stream);
}

extern "C" int strom_column_qual(const strom_col_qual *q, const strom_qual_batch *d_batches,
                                 uint32_t nbatches, uint64_t nwords, uint64_t *d_bitmap,
                                 const uint64_t *d_or, int and_dst, uint64_t *d_count,
                                 void *stream) {
  if (!q) return -22;
  if (!nbatches || !nwords) return 0;
  if (!d_batches || !d_bitmap || !d_count || ((uintptr_t)d_bitmap & 7)) return -22;
  hipStream_t st = (hipStream_t)stream;
  const bool str = q->type == STROM_COL_STR32 || q->type == STROM_COL_STR64;
  // constants must fit the LDS staging and be whole dwords
  if (q->op != STROM_QOP_VALID) {
    if (!q->consts || (q->const_bytes & 3) || (q->consts & 3)) return -22;
    if (q->const_bytes + (str ? q->offs_bytes : 0) > (64u << 10)) return -7;
  }
  switch (q->op) {
    case STROM_QOP_RANGES: {
      const uint64_t need = (q->type == STROM_COL_DEC128 ? 32ull : 16ull) * q->nconst;
      if (str || q->const_bytes < need) return -22;
      return qual_by_type<QK_RANGE>(*q, d_batches, nbatches, nwords, d_bitmap, d_or, and_dst, d_count, st);
    }
    case STROM_QOP_LUT:
      if (str || q->type == STROM_COL_BOOL || q->type == STROM_COL_F32 || q->type == STROM_COL_F64 ||
          q->const_bytes * 8 < q->nconst)
        return -22;
      return qual_by_type<QK_LUT>(*q, d_batches, nbatches, nwords, d_bitmap, d_or, and_dst, d_count, st);
    case STROM_QOP_STR_IN:
    case STROM_QOP_STR_PREFIX:
    case STROM_QOP_STR_RANGES: {
      const uint64_t per = q->op == STROM_QOP_STR_RANGES ? 24 : 8;
      if (!str || !q->offs || (q->offs & 3) || q->offs_bytes < per * q->nconst || (q->offs_bytes & 3))
        return -22;
      // every constant inside the blob (checked on the host copy by the
      // caller's contract: the (start, len) pairs are read from device
      // memory, so only the sizes can be checked here)
      if (q->type == STROM_COL_STR32)
        return launch_qual<int32_t, QK_STR>(*q, d_batches, nbatches, nwords, d_bitmap, d_or, and_dst, d_count, st);
      return launch_qual<int64_t, QK_STR>(*q, d_batches, nbatches, nwords, d_bitmap, d_or, and_dst, d_count, st);
    }
    case STROM_QOP_VALID:
      return launch_qual<int32_t, QK_VALID>(*q, d_batches, nbatches, nwords, d_bitmap, d_or, and_dst, d_count, st);
    default:
      return -22;
  }
}

// bitmap_to_rows with a utf8/binary column projected: d_strtab (the same
// batches as strom_qual_batch rows: offsets in values, characters in aux),
// owidth 4 or 8 (offset width); each selected row's characters are appended
// at the device cursor *d_char_cursor in d_pchars (the caller sizes it for
// the column's characters) and its start written to d_poff[pos].
extern "C" int strom_bitmap_to_rows_str(const uint64_t *d_bitmap, uint64_t nwords,
                                        const strom_filter_batch *d_batches, uint32_t nbatches,
                                        int64_t *d_out, uint64_t *d_total,
                                        const strom_qual_batch *d_strtab, uint32_t owidth,
                                        int64_t *d_poff, uint8_t *d_pchars, uint8_t *d_pvalid,
                                        uint64_t *d_char_cursor, void *stream) {
  if (!nwords || !nbatches) return 0;
  if (!d_bitmap || !d_batches || !d_out || !d_total || !d_strtab || !d_poff || !d_pchars ||
      !d_char_cursor || (owidth != 4 && owidth != 8))
    return -22;
  hipStream_t st = (hipStream_t)stream;
  const uint64_t nb64 = (nwords + kWordsPerBlock - 1) / kWordsPerBlock;
  if (nb64 > 0xffffffffull) return -75;
  const uint32_t nb = (uint32_t)nb64;
  std::lock_guard<std::mutex> g(g_cs_mu);
  uint64_t *cnt = (uint64_t *)col_scratch(st, sizeof(uint64_t) * 2 * nb);
  if (!cnt) return -12;
  uint64_t *ccnt = cnt + nb;
  hipLaunchKernelGGL(block_popc64_kernel, dim3(nb), dim3(256), 0, st, d_bitmap, nwords, cnt);
  if (owidth == 4)
    hipLaunchKernelGGL(block_chars_kernel<int32_t>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords,
                       d_strtab, nbatches, ccnt);
  else
    hipLaunchKernelGGL(block_chars_kernel<int64_t>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords,
                       d_strtab, nbatches, ccnt);
  hipLaunchKernelGGL(scan_blocks_cursor_kernel, dim3(1), dim3(1024), 0, st, cnt, nb,
                     (unsigned long long *)d_total);
  hipLaunchKernelGGL(scan_blocks_cursor_kernel, dim3(1), dim3(1024), 0, st, ccnt, nb,
                     (unsigned long long *)d_char_cursor);
  if (owidth == 4)
    hipLaunchKernelGGL(emit_str_kernel<int32_t>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords,
                       d_strtab, nbatches, cnt, ccnt, d_out, d_poff, d_pchars, d_pvalid);
  else
    hipLaunchKernelGGL(emit_str_kernel<int64_t>, dim3(nb), dim3(256), 0, st, d_bitmap, nwords,
                       d_strtab, nbatches, cnt, ccnt, d_out, d_poff, d_pchars, d_pvalid);
  (void)d_batches;
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
