// crc32c.hip — CRC32C (Castagnoli) of HBM-resident data on CDNA4.
//
// Replaces the reference's verify path (nvme_test -c: DtoH readback +
// memcmp, utils/nvme_test.c:226-267) with an on-GPU checksum: the host
// computes the same CRC of the file with strom_crc32c_host and compares
// 4 bytes instead of reading the whole segment back over PCIe.
//
// Layout of the work (one wavefront per chunk, 64-wide, grid-stride):
//   the chunk is viewed as rows of 1 KiB = 64 lanes x 16 B (one
//   global_load_dwordx4 per lane per row, fully coalesced, 8 rows in flight
//   per lane).  Lane l keeps a running raw CRC A_l of its column:
//   A_l <- shift1K(A_l) ^ R(piece), where
//     R()      = zero-init CRC of a 16-byte piece, slicing-by-4 (4 word steps
//                of 4 table lookups, tables T0..T3);
//     shift1K  = "append 1024 zero bytes", 4 lookups (tables X0..X3).
//   The 8 tables sit in LDS as 16 lane-indexed copies (entry b of copy c at
//   word b*16 + c): lanes l and l+16 share a copy and collide only when
//   their entries have the same parity, so a ds_read_b32 takes at most two
//   passes whatever the data, where round 1's single copy of 20 tables
//   (slicing-by-16) took ~4 on random bytes (14x more bank-conflict cycles
//   than LDS instructions on its worst input, profiles/r1i).  (A VALU-only
//   shift1K — 32 masked xors — measured slower: 2.8 vs 3.7 TB/s, r2.)
//   128 KiB of LDS, one workgroup of up to 16 waves per CU.
//   Columns are then aligned with one GF(2) multiply by x^(8*16*(63-l)) mod
//   P and folded with a 6-step xor butterfly — no cross-lane ordering, no
//   serial dependency across lanes.  CRC linearity also turns the 0xFFFFFFFF
//   initial value into an xor of the first data word.
// A second kernel folds per-chunk CRCs into the CRC of the whole buffer
// (zlib crc32_combine algebra: crc(A|B) = shift(crc(A), |B|) ^ crc(B)).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "strom/strom.h"

namespace {

constexpr uint32_t kPoly = 0x82F63B78u;

// reflected GF(2) product mod P: bit 31 is x^0
__host__ __device__ constexpr uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & (0x80000000u >> i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : (b >> 1);
  }
  return p;
}

struct CrcTables {
  uint32_t T[16][256];   // T[k][b] = R(b followed by k zero bytes)
  uint32_t X[4][256];    // X[k][b] = shift(b << 8k, 1024 bytes)
  uint32_t sh16[64];     // x^(8*16*m) mod P
  uint32_t x2n[64];      // x^(2^k) mod P
};

constexpr uint32_t xpow8n_c(const uint32_t *x2n, uint64_t n) {
  uint32_t p = 0x80000000u;
  int k = 3;
  while (n) {
    if (n & 1) p = multmodp(x2n[k], p);
    n >>= 1;
    ++k;
  }
  return p;
}

constexpr CrcTables make_tables() {
  CrcTables t{};
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
    t.T[0][b] = c;
  }
  for (int k = 1; k < 16; ++k)
    for (uint32_t b = 0; b < 256; ++b)
      t.T[k][b] = (t.T[k - 1][b] >> 8) ^ t.T[0][t.T[k - 1][b] & 0xff];
  t.x2n[0] = 0x40000000u;  // x^1
  for (int k = 1; k < 64; ++k) t.x2n[k] = multmodp(t.x2n[k - 1], t.x2n[k - 1]);
  const uint32_t k1k = xpow8n_c(t.x2n, 1024);
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) t.X[k][b] = multmodp(k1k, b << (8 * k));
  for (int m = 0; m < 64; ++m) t.sh16[m] = xpow8n_c(t.x2n, 16ull * m);
  return t;
}

__constant__ CrcTables g_crc = make_tables();

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ uint32_t xpow8n(uint64_t n) {
  uint32_t p = 0x80000000u;
  int k = 3;
  while (n) {
    if (n & 1) p = multmodp(g_crc.x2n[k], p);
    n >>= 1;
    ++k;
  }
  return p;
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int kCopies = 16;                    // lanes l and l+16 share a copy
constexpr int kTables = 8;                     // T0..T3 (slicing-by-4), X0..X3 (shift1K)
constexpr int kLdsWords = kTables * 256 * kCopies;   // 128 KiB

// table k (0..3 = T, 4..7 = X), entry b, from this lane's copy
__device__ __forceinline__ uint32_t tab(const uint32_t *lds, uint32_t k, uint32_t b, uint32_t cp) {
  return lds[((k << 8) + b) * kCopies + cp];
}

// zero-init CRC of a 16-byte piece (words in memory order)
__device__ __forceinline__ uint32_t r16(const uint32_t *lds, uint32_t cp, uint4 w) {
  const uint32_t v[4] = {w.x, w.y, w.z, w.w};
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = c ^ v[i];
    c = tab(lds, 3, x & 0xff, cp) ^ tab(lds, 2, (x >> 8) & 0xff, cp) ^
        tab(lds, 1, (x >> 16) & 0xff, cp) ^ tab(lds, 0, x >> 24, cp);
  }
  return c;
}

// append 1024 zero bytes
__device__ __forceinline__ uint32_t shift1k(const uint32_t *lds, uint32_t cp, uint32_t a) {
  return tab(lds, 4, a & 0xff, cp) ^ tab(lds, 5, (a >> 8) & 0xff, cp) ^
         tab(lds, 6, (a >> 16) & 0xff, cp) ^ tab(lds, 7, a >> 24, cp);
}

// append b (< 16) zero bytes
__device__ __forceinline__ uint32_t zshift(const uint32_t *lds, uint32_t cp, uint32_t a, uint32_t b) {
  for (uint32_t j = 0; j < b; ++j) a = (a >> 8) ^ tab(lds, 0, a & 0xff, cp);
  return a;
}

constexpr int kWaves = 16;                  // 1024-thread workgroups
constexpr int kRows = 8;                    // rows in flight per lane

// CRC register state after the bytes p[0, L) (init = ~0 when `first`, else
// 0 — the caller combines parts with crc(A|B) = shift(crc(A), |B|) ^ crc(B))
// computed by one wave; every lane returns the same value.
__device__ uint32_t wave_crc(const uint32_t *lds, uint32_t lane, uint32_t cp, const uint8_t *p,
                             uint32_t L, bool first) {
  if (L < 4) {
    uint32_t st = first ? 0xffffffffu : 0u;
    for (uint32_t j = 0; j < L; ++j) st = (st >> 8) ^ tab(lds, 0, (st ^ p[j]) & 0xff, cp);
    return st;
  }
  const uint32_t nfull = L >> 10;
  uint32_t a = 0;
  uint32_t r = 0;
  for (; r + kRows <= nfull; r += kRows) {
    uint4 w[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const v4u x = __builtin_nontemporal_load((const v4u *)(p + (uint64_t)(r + k) * 1024 + lane * 16));
      w[k] = make_uint4(x[0], x[1], x[2], x[3]);
    }
    if (first && r == 0 && lane == 0) w[0].x ^= 0xffffffffu;
    uint32_t rr[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) rr[k] = r16(lds, cp, w[k]);
#pragma unroll
    for (int k = 0; k < kRows; ++k) a = shift1k(lds, cp, a) ^ rr[k];
  }
  for (; r < nfull; ++r) {
    uint4 w = *(const uint4 *)(p + (uint64_t)r * 1024 + lane * 16);
    if (first && r == 0 && lane == 0) w.x ^= 0xffffffffu;
    a = shift1k(lds, cp, a) ^ r16(lds, cp, w);
  }
  const uint32_t full = nfull ? wave_xor(multmodp(g_crc.sh16[63 - lane], a)) : 0u;
  const uint32_t rest = L - nfull * 1024;
  if (!rest) return full;
  const uint32_t q = rest >> 4, b = rest & 15;
  const uint8_t *rp = p + (uint64_t)nfull * 1024;
  const bool head = first && nfull == 0;
  uint32_t contrib = 0;
  if (lane < q) {
    uint4 w = *(const uint4 *)(rp + lane * 16);
    if (head && lane == 0) w.x ^= 0xffffffffu;
    contrib = zshift(lds, cp, multmodp(g_crc.sh16[q - 1 - lane], r16(lds, cp, w)), b);
  } else if (lane == q && b) {
    uint32_t st = 0;
    for (uint32_t j = 0; j < b; ++j) {
      uint32_t byte = rp[lane * 16 + j];
      if (head && q == 0 && j < 4) byte ^= 0xffu;
      st = (st >> 8) ^ tab(lds, 0, (st ^ byte) & 0xff, cp);
    }
    contrib = st;
  }
  contrib = wave_xor(contrib);
  return zshift(lds, cp, multmodp(g_crc.sh16[q], full), b) ^ contrib;
}

// Two schedules over the same per-wave body:
//   split = 0: one wave per chunk, grid-stride over chunks (many chunks);
//   split = 1: one workgroup per chunk, each wave CRCs a contiguous 1-KiB-
//              aligned part and the parts are folded in LDS (few, large
//              chunks: 1 MiB chunks over 1 GiB are only 4 waves per CU in
//              wave mode).
__global__ __launch_bounds__(1024) void crc32c_chunks_kernel(const uint8_t *__restrict__ in,
                                                             uint64_t n, uint32_t chunk,
                                                             uint32_t nchunks, int split,
                                                             uint32_t *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t parts[kWaves];
  // fill: table word e = k*256 + b is loaded once and stored as its 16
  // contiguous copies (4 x ds_write_b128)
  for (uint32_t e = threadIdx.x; e < kTables * 256; e += blockDim.x) {
    const uint32_t v = e < 1024 ? g_crc.T[e >> 8][e & 255] : g_crc.X[(e >> 8) - 4][e & 255];
    const uint4 q = make_uint4(v, v, v, v);
    uint4 *dst = (uint4 *)(lds + e * kCopies);
#pragma unroll
    for (int j = 0; j < kCopies / 4; ++j) dst[j] = q;
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, cp = lane & 15, wv = threadIdx.x >> 6;
  const uint32_t wpb = blockDim.x >> 6;
  if (!split) {
    const uint32_t nwaves = gridDim.x * wpb;
    for (uint32_t c = blockIdx.x * wpb + wv; c < nchunks; c += nwaves) {
      const uint64_t base = (uint64_t)c * chunk;
      const uint32_t L = (uint32_t)min<uint64_t>(chunk, n - base);
      const uint32_t crc = ~wave_crc(lds, lane, cp, in + base, L, true);
      if (lane == 0) out[c] = crc;
    }
    return;
  }
  for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {   // uniform per workgroup
    const uint64_t base = (uint64_t)c * chunk;
    const uint32_t L = (uint32_t)min<uint64_t>(chunk, n - base);
    const uint32_t plen = (((L + wpb - 1) / wpb) + 1023u) & ~1023u;
    const uint32_t lo = min(L, wv * plen), hi = min(L, lo + plen);
    uint32_t v = hi > lo ? wave_crc(lds, lane, cp, in + base + lo, hi - lo, wv == 0) : 0u;
    if (hi > lo && hi < L) v = multmodp(xpow8n(L - hi), v);
    if (lane == 0) parts[wv] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t r = 0;
      for (uint32_t k = 0; k < wpb; ++k) r ^= parts[k];
      out[c] = ~r;
    }
    __syncthreads();
  }
}

// Fold per-chunk CRCs: one workgroup of 1024 threads.  Each thread folds a
// contiguous run of chunks (Horner; the fixed per-chunk shift as 4 byte
// lookups, one table entry built per thread), then shifts its run's CRC
// past every byte after the run, x^(8 * bytes after) — independent per
// thread, no serial tree of shifts — and the runs are xor-reduced
// (crc(A|B) = shift(crc(A), |B|) ^ crc(B), zlib's crc32_combine algebra).
__global__ __launch_bounds__(1024) void crc32c_combine_kernel(const uint32_t *__restrict__ crcs,
                                                              uint32_t nchunks, uint32_t chunk,
                                                              uint64_t nbytes,
                                                              uint32_t *__restrict__ out) {
  __shared__ uint32_t xk[4][256];      // xk[j][v] = (v << 8j) * x^(8 chunk) mod P
  __shared__ uint32_t part[16];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (nchunks + 1023) / 1024;
  const uint32_t lo = min(nchunks, t * per), hi = min(nchunks, lo + per);
  xk[t >> 8][t & 255] = multmodp(xpow8n(chunk), (t & 255) << (8 * (t >> 8)));
  __syncthreads();
  uint32_t acc = 0;
  // full chunks 8 at a time with their CRC loads in flight together (one
  // dependent load per chunk was most of this kernel's time)
  const uint32_t full_hi = min<uint64_t>(hi, nbytes / chunk);   // chunks before a partial tail
  uint32_t i = lo;
  for (; i + 8 <= full_hi; i += 8) {
    uint32_t c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = crcs[i + k];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      acc = (xk[0][acc & 255] ^ xk[1][(acc >> 8) & 255] ^ xk[2][(acc >> 16) & 255] ^
             xk[3][acc >> 24]) ^ c[k];
  }
  for (; i < hi; ++i) {
    const uint64_t li = min<uint64_t>(chunk, nbytes - (uint64_t)i * chunk);
    const uint32_t sh = li == chunk ? xk[0][acc & 255] ^ xk[1][(acc >> 8) & 255] ^
                                          xk[2][(acc >> 16) & 255] ^ xk[3][acc >> 24]
                                    : multmodp(xpow8n(li), acc);
    acc = sh ^ crcs[i];
  }
  if (hi > lo) {
    const uint64_t after = nbytes - min<uint64_t>(nbytes, (uint64_t)hi * chunk);
    if (after) acc = multmodp(xpow8n(after), acc);
  }
  acc = wave_xor(acc);
  if ((t & 63) == 0) part[t >> 6] = acc;
  __syncthreads();
  if (t == 0) {
    uint32_t r = 0;
    for (uint32_t k = 0; k < (blockDim.x >> 6); ++k) r ^= part[k];
    out[0] = r;
  }
}

}  // namespace

extern "C" int strom_crc32c_chunks(const void *d_in, uint64_t nbytes, uint32_t chunk,
                                   uint32_t *d_out, void *stream) {
  if (!d_in || !d_out || chunk == 0 || (chunk & 15) || ((uintptr_t)d_in & 15)) return -22;
  if (nbytes == 0) return 0;
  uint64_t nch = (nbytes + chunk - 1) / chunk;
  if (nch > 0xffffffffull) return -22;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void *)crc32c_chunks_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kLdsWords * 4);
    attr_set = true;
  }
  // one workgroup per CU holds the 128 KiB tables.  Enough chunks for 8+
  // waves per CU: one wave per chunk, up to 16 waves per workgroup; fewer,
  // larger chunks: a 16-wave workgroup per chunk.
  const bool split = nch < 256ull * 8 && chunk >= 16384;
  uint32_t wpb, grid;
  if (split) {
    wpb = kWaves;
    grid = (uint32_t)(nch < 256 ? nch : 256);
  } else {
    wpb = (uint32_t)((nch + 255) / 256);
    if (wpb > kWaves) wpb = kWaves;
    if (wpb < 1) wpb = 1;
    grid = (uint32_t)((nch + wpb - 1) / wpb);
    if (grid > 256) grid = 256;
  }
  hipLaunchKernelGGL(crc32c_chunks_kernel, dim3(grid), dim3(64 * wpb), kLdsWords * 4,
                     (hipStream_t)stream, (const uint8_t *)d_in, nbytes, chunk, (uint32_t)nch,
                     (int)split, d_out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int strom_crc32c_combine(const uint32_t *d_crcs, uint32_t nchunks, uint32_t chunk,
                                    uint64_t nbytes, uint32_t *d_out, void *stream) {
  if (!d_crcs || !d_out || chunk == 0 || nchunks == 0) return -22;
  if ((uint64_t)(nchunks - 1) * chunk >= nbytes || (uint64_t)nchunks * chunk < nbytes) return -22;
  hipLaunchKernelGGL(crc32c_combine_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_crcs,
                     nchunks, chunk, nbytes, d_out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
