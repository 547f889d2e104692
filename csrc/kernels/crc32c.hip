// crc32c.hip — CRC32C (Castagnoli) of HBM-resident data on CDNA4.
//
// Replaces the reference's verify path (nvme_test -c: DtoH readback +
// memcmp, utils/nvme_test.c:226-267) with an on-GPU checksum: the host
// computes the same CRC of the file with strom_crc32c_host and compares
// 4 bytes instead of reading the whole segment back over PCIe.
//
// Layout of the work (one wavefront per chunk, 64-wide, grid-stride):
//   the chunk is viewed as rows of 1 KiB = 64 lanes x 16 B (one
//   global_load_dwordx4 per lane per row, fully coalesced).  Lane l keeps a
//   running raw CRC A_l of its column: A_l <- shift1K(A_l) ^ R(piece), where
//   R() is zero-init CRC of a 16-byte piece by slicing-by-16 lookups and
//   shift1K() is the linear "append 1024 zero bytes" map, both as byte
//   tables staged in LDS (20 KiB).  Columns are then aligned with one GF(2)
//   multiply by x^(8*16*(63-l)) mod P and folded with a 6-step xor
//   butterfly — no cross-lane ordering, no serial dependency across lanes.
//   CRC linearity also turns the 0xFFFFFFFF initial value into an xor of
//   the first data word, so no pow(x, 8n) is needed for the init term.
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

struct Lds {
  uint32_t T[16][256];
  uint32_t X[4][256];
};

__device__ __forceinline__ uint32_t r16(const Lds &s, uint4 w) {
  uint32_t r = 0;
  const uint32_t v[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r ^= s.T[15 - 4 * i][v[i] & 0xff];
    r ^= s.T[14 - 4 * i][(v[i] >> 8) & 0xff];
    r ^= s.T[13 - 4 * i][(v[i] >> 16) & 0xff];
    r ^= s.T[12 - 4 * i][v[i] >> 24];
  }
  return r;
}

__device__ __forceinline__ uint32_t shift1k(const Lds &s, uint32_t a) {
  return s.X[0][a & 0xff] ^ s.X[1][(a >> 8) & 0xff] ^ s.X[2][(a >> 16) & 0xff] ^ s.X[3][a >> 24];
}

// append b (< 16) zero bytes
__device__ __forceinline__ uint32_t zshift(const Lds &s, uint32_t a, uint32_t b) {
  for (uint32_t j = 0; j < b; ++j) a = (a >> 8) ^ s.T[0][a & 0xff];
  return a;
}

__global__ __launch_bounds__(256) void crc32c_chunks_kernel(const uint8_t *__restrict__ in,
                                                            uint64_t n, uint32_t chunk,
                                                            uint32_t nchunks,
                                                            uint32_t *__restrict__ out) {
  __shared__ Lds s;
  {
    const uint32_t *srcT = &g_crc.T[0][0];
    uint32_t *dstT = &s.T[0][0];
    for (int i = threadIdx.x; i < 16 * 256; i += 256) dstT[i] = srcT[i];
    const uint32_t *srcX = &g_crc.X[0][0];
    uint32_t *dstX = &s.X[0][0];
    for (int i = threadIdx.x; i < 4 * 256; i += 256) dstX[i] = srcX[i];
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * 4;
  for (uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunks; c += nwaves) {
    const uint64_t base = (uint64_t)c * chunk;
    const uint32_t L = (uint32_t)min<uint64_t>(chunk, n - base);
    const uint8_t *p = in + base;
    uint32_t crc;
    if (L < 4) {
      uint32_t st = 0xffffffffu;
      for (uint32_t j = 0; j < L; ++j) st = (st >> 8) ^ s.T[0][(st ^ p[j]) & 0xff];
      crc = ~st;
    } else {
      const uint32_t nfull = L >> 10;
      uint32_t a = 0;
      uint32_t r = 0;
      // 4 rows in flight per lane
      for (; r + 4 <= nfull; r += 4) {
        uint4 w0 = *(const uint4 *)(p + (uint64_t)(r + 0) * 1024 + lane * 16);
        uint4 w1 = *(const uint4 *)(p + (uint64_t)(r + 1) * 1024 + lane * 16);
        uint4 w2 = *(const uint4 *)(p + (uint64_t)(r + 2) * 1024 + lane * 16);
        uint4 w3 = *(const uint4 *)(p + (uint64_t)(r + 3) * 1024 + lane * 16);
        if (r == 0 && lane == 0) w0.x ^= 0xffffffffu;
        a = shift1k(s, a) ^ r16(s, w0);
        a = shift1k(s, a) ^ r16(s, w1);
        a = shift1k(s, a) ^ r16(s, w2);
        a = shift1k(s, a) ^ r16(s, w3);
      }
      for (; r < nfull; ++r) {
        uint4 w = *(const uint4 *)(p + (uint64_t)r * 1024 + lane * 16);
        if (r == 0 && lane == 0) w.x ^= 0xffffffffu;
        a = shift1k(s, a) ^ r16(s, w);
      }
      uint32_t full = nfull ? wave_xor(multmodp(g_crc.sh16[63 - lane], a)) : 0u;
      const uint32_t rest = L - nfull * 1024;
      uint32_t res = full;
      if (rest) {
        const uint32_t q = rest >> 4, b = rest & 15;
        const uint8_t *rp = p + (uint64_t)nfull * 1024;
        const bool first = nfull == 0;
        uint32_t contrib = 0;
        if (lane < q) {
          uint4 w = *(const uint4 *)(rp + lane * 16);
          if (first && lane == 0) w.x ^= 0xffffffffu;
          contrib = zshift(s, multmodp(g_crc.sh16[q - 1 - lane], r16(s, w)), b);
        } else if (lane == q && b) {
          uint32_t st = 0;
          for (uint32_t j = 0; j < b; ++j) {
            uint32_t byte = rp[lane * 16 + j];
            if (first && q == 0 && j < 4) byte ^= 0xffu;
            st = (st >> 8) ^ s.T[0][(st ^ byte) & 0xff];
          }
          contrib = st;
        }
        contrib = wave_xor(contrib);
        res = zshift(s, multmodp(g_crc.sh16[q], full), b) ^ contrib;
      }
      crc = ~res;
    }
    if (lane == 0) out[c] = crc;
  }
}

// Fold per-chunk CRCs: one workgroup of 1024 threads; each thread folds a
// contiguous run (Horner with a fixed shift), then a log-depth tree with
// length-dependent shifts.
__global__ __launch_bounds__(1024) void crc32c_combine_kernel(const uint32_t *__restrict__ crcs,
                                                              uint32_t nchunks, uint32_t chunk,
                                                              uint64_t nbytes,
                                                              uint32_t *__restrict__ out) {
  __shared__ uint32_t sc[1024];
  __shared__ uint64_t sl[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (nchunks + 1023) / 1024;
  const uint32_t lo = min(nchunks, t * per), hi = min(nchunks, lo + per);
  const uint32_t kchunk = xpow8n(chunk);
  uint32_t acc = 0;
  uint64_t len = 0;
  for (uint32_t i = lo; i < hi; ++i) {
    uint64_t li = min<uint64_t>(chunk, nbytes - (uint64_t)i * chunk);
    uint32_t k = li == chunk ? kchunk : xpow8n(li);
    acc = (len ? multmodp(k, acc) : 0u) ^ crcs[i];
    len += li;
  }
  sc[t] = acc;
  sl[t] = len;
  __syncthreads();
  for (uint32_t stride = 1; stride < 1024; stride <<= 1) {
    uint32_t c2 = 0;
    uint64_t l2 = 0;
    bool active = (t % (2 * stride)) == 0 && t + stride < 1024;
    if (active) {
      uint64_t lr = sl[t + stride];
      c2 = (lr ? multmodp(xpow8n(lr), sc[t]) : sc[t]) ^ sc[t + stride];
      l2 = sl[t] + lr;
    }
    __syncthreads();
    if (active) {
      sc[t] = c2;
      sl[t] = l2;
    }
    __syncthreads();
  }
  if (t == 0) out[0] = sc[0];
}

}  // namespace

extern "C" int strom_crc32c_chunks(const void *d_in, uint64_t nbytes, uint32_t chunk,
                                   uint32_t *d_out, void *stream) {
  if (!d_in || !d_out || chunk == 0 || (chunk & 15) || ((uintptr_t)d_in & 15)) return -22;
  if (nbytes == 0) return 0;
  uint64_t nch = (nbytes + chunk - 1) / chunk;
  if (nch > 0xffffffffull) return -22;
  uint32_t waves_needed = (uint32_t)nch;
  uint32_t grid = (waves_needed + 3) / 4;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(crc32c_chunks_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t *)d_in, nbytes, chunk, (uint32_t)nch, d_out);
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
