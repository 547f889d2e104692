// decompress.hip — LZ4 / snappy decode of HBM-resident buffers on CDNA4.
//
// North-star config 5 (BASELINE.json): compressed columnar files land in HBM
// through the engine and are decompressed on the GPU before the filter.  The
// reference has no decompressor; this is new MI355X-side work.
//
// One 64-lane workgroup (= one wavefront) decodes one stream at a time
// (grid-stride over descriptors).  Parsing is wave-uniform; byte moves are
// spread over the 64 lanes, one byte per lane per pass:
//   * an 8 KiB LDS input window: tokens/lengths/offsets/literals are read from
//     LDS; the window is refilled (one coalesced sweep) ahead of the parser;
//   * a 64 KiB LDS history ring (LZ4 distances are < 64 KiB) serves every
//     match source; each output byte is stored to HBM and to the ring in the
//     same pass, so there is no flush pass and no HBM re-read;
//   * overlapping matches (distance < length) never use a modulo in the
//     copy loop: distance >= 64 copies pass by pass (each pass reads bytes a
//     previous pass wrote); distance < 64 seeds one 64-byte pass from the
//     pattern (k mod d, computed once per match) and continues with a period
//     Q = d * ceil(64 / d) in [64, 127].
// All positions are 32-bit (streams < 4 GiB).  Snappy copies farther than
// 64 KiB (legal, never produced by 64 KiB-fragment compressors) read the
// already-stored HBM output with L1-bypassing loads.
//
// Codecs: raw LZ4 block, LZ4 frame block sequence (linked or independent
// blocks, optional per-block checksums skipped), raw snappy, stored copy.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "strom/strom.h"

#ifndef STROM_DECOMP_RING
#define STROM_DECOMP_RING (8u << 10)
#endif
#ifndef STROM_DECOMP_INW
#define STROM_DECOMP_INW (2u << 10)
#endif

namespace {

// 16 KiB history + 4 KiB input = 20 KiB of LDS per wave -> 8 waves per CU.
// (A full 64 KiB LZ4 window fits only 2 per CU, and a wave-serial decoder
// is issue-bound: throughput scales with resident waves.)  Matches that
// reach past the ring read the HBM output this wave already stored.
constexpr uint32_t kRing = STROM_DECOMP_RING;
constexpr uint32_t kMask = kRing - 1;
constexpr uint32_t kInW = STROM_DECOMP_INW;
constexpr uint32_t kAhead = 512;  // keep this much input in the window

enum : int32_t { kErrFormat = -1, kErrOverflow = -2 };

// The workgroup is ONE wavefront, so lanes only need their LDS writes
// ordered before later LDS reads.  __syncthreads() would also wait for every
// outstanding HBM byte store (vmcnt(0)): ~1 us per call, twice per LZ4
// sequence, which capped v1 at ~6 GB/s.  The asm also fences the compiler.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t ld_bypass_byte(const uint8_t *p) {
  // dword-aligned agent-scope relaxed load: global_load ... sc1 (skips L1)
  const uint32_t *w = (const uint32_t *)((uintptr_t)p & ~(uintptr_t)3);
  uint32_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (v >> (8 * ((uintptr_t)p & 3))) & 0xff;
}

struct Decoder {
  const uint8_t *in;
  uint8_t *out;
  uint32_t ilen, ocap;
  uint32_t op = 0, win = 0xffffffffu;
  int32_t err = 0;
  uint8_t *ring;
  uint8_t *inw;
  uint32_t lane;

  // Register window: 256 input bytes, one dword per lane; the wave-uniform
  // parser reads them with v_readlane (scalar, a few cycles) instead of a
  // dependent LDS round trip per token/length/offset byte.
  uint32_t rwin = 0, rbase = 0xffffffffu;

  __device__ void load_reg(uint32_t q) {  // q: 4-aligned, win covers q
    const uint32_t o = q - win + 4 * lane;
    rwin = o + 4 <= kInW ? *(const uint32_t *)(inw + o) : 0u;
    rbase = q;
  }
  __device__ void load_window(uint32_t at) {
    at &= ~3u;  // dword-aligned window base (register window loads)
    lds_sync();
    rbase = 0xffffffffu;
    const uint32_t n = ilen - at < kInW ? ilen - at : kInW;
    // dword sweep when aligned, bytes otherwise
    const uint8_t *src = in + at;
    if (((uintptr_t)src & 3) == 0) {
      for (uint32_t k = lane * 4; k + 4 <= n; k += 256) *(uint32_t *)(inw + k) = *(const uint32_t *)(src + k);
      for (uint32_t k = (n & ~3u) + lane; k < n; k += 64) inw[k] = src[k];
    } else {
      for (uint32_t k = lane; k < n; k += 64) inw[k] = src[k];
    }
    win = at;
    lds_sync();
  }
  // keep [p, p + kAhead) inside the window when the input has it
  __device__ void ensure(uint32_t p) {
    const uint32_t end = p + kAhead < ilen ? p + kAhead : ilen;
    if (p < win || end > win + kInW) load_window(p);
  }
  __device__ uint32_t byte(uint32_t p) {
    if (p < rbase || p - rbase >= 256) {  // rbase = ~0 means empty
      const uint32_t q = p & ~3u;
      const uint32_t need = q + 256 < ilen ? q + 256 : ilen;
      if (q < win || need > win + kInW) load_window(q);
      load_reg(q);
    }
    const uint32_t rel = p - rbase;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)rwin, (int)(rel >> 2));
    return (w >> (8 * (rel & 3))) & 0xffu;
  }
  // literal bytes src[ip, ip+len) -> output
  __device__ void literal(uint32_t ip, uint32_t len) {
    for (uint32_t done = 0; done < len; done += 64) {
      const uint32_t k = done + lane;
      if (k < len) {
        const uint32_t p = ip + k;
        const uint8_t v = (p - win < kInW) ? inw[p - win] : in[p];
        ring[(op + k) & kMask] = v;
        out[op + k] = v;
      }
    }
    op += len;
    lds_sync();
  }
  __device__ void match(uint32_t off, uint32_t len) {
    if (off == 0 || off > op) {
      err = kErrFormat;
      return;
    }
    const uint32_t s = op;
    // near: every source byte stays in the ring for the whole match
    const bool near = off < 64 || off + len <= kRing;
    if (!near) {
      // far copy: sources are in HBM already, written by this wave; make
      // them visible to L1-bypassing loads
      __threadfence();
      for (uint32_t done = 0; done < len; done += 64) {
        const uint32_t k = done + lane;
        if (k < len) {
          const uint8_t v = (uint8_t)ld_bypass_byte(out + s - off + k);
          ring[(s + k) & kMask] = v;
          out[s + k] = v;
        }
        if (off < len) {
          __threadfence();
          lds_sync();
        }
      }
      op += len;
      lds_sync();
      return;
    }
    if (off >= 64 || off >= len) {
      const bool overlap = off < len;
      for (uint32_t done = 0; done < len; done += 64) {
        const uint32_t k = done + lane;
        if (k < len) {
          const uint8_t v = ring[(s - off + k) & kMask];
          ring[(s + k) & kMask] = v;
          out[s + k] = v;
        }
        if (overlap) lds_sync();  // next pass may read this one
      }
    } else {
      // short period: seed 64 bytes from the pattern, then period Q >= 64
      const uint32_t q = off * ((64 + off - 1) / off);
      const uint32_t r = lane % off;
      if (lane < len) {
        const uint8_t v = ring[(s - off + r) & kMask];
        ring[(s + lane) & kMask] = v;
        out[s + lane] = v;
      }
      lds_sync();
      for (uint32_t done = 64; done < len; done += 64) {
        const uint32_t k = done + lane;
        if (k < len) {
          const uint8_t v = ring[(s + k - q) & kMask];
          ring[(s + k) & kMask] = v;
          out[s + k] = v;
        }
        lds_sync();
      }
    }
    op += len;
    lds_sync();
  }
  // one raw LZ4 block occupying src[ip, end); returns new ip
  __device__ uint32_t lz4_block(uint32_t ip, uint32_t end) {
    while (ip < end && !err) {
      ensure(ip);
      const uint32_t token = byte(ip++);
      uint32_t lit = token >> 4;
      if (lit == 15) {
        uint32_t b;
        do {
          if (ip >= end) { err = kErrFormat; return ip; }
          b = byte(ip++);
          lit += b;
        } while (b == 255);
      }
      if (lit > end - ip) { err = kErrFormat; return ip; }
      if (lit > ocap - op) { err = kErrOverflow; return ip; }
      if (lit) literal(ip, lit);
      ip += lit;
      if (ip >= end) break;  // last sequence carries literals only
      if (end - ip < 2) { err = kErrFormat; return ip; }
      const uint32_t off = byte(ip) | (byte(ip + 1) << 8);
      ip += 2;
      uint32_t ml = token & 15;
      if (ml == 15) {
        uint32_t b;
        do {
          if (ip >= end) { err = kErrFormat; return ip; }
          b = byte(ip++);
          ml += b;
        } while (b == 255);
      }
      ml += 4;
      if (ml > ocap - op) { err = kErrOverflow; return ip; }
      match(off, ml);
    }
    return ip;
  }
  __device__ void snappy() {
    uint32_t ip = 0;
    uint64_t ulen = 0;
    ensure(0);
    for (int shift = 0;; shift += 7) {
      if (ip >= ilen || shift > 35) { err = kErrFormat; return; }
      const uint32_t b = byte(ip++);
      ulen |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) break;
    }
    if (ulen > ocap) { err = kErrOverflow; return; }
    const uint32_t olen = (uint32_t)ulen;
    while (ip < ilen && !err) {
      ensure(ip);
      const uint32_t tag = byte(ip++);
      uint32_t len, off;
      const uint32_t kind = tag & 3;
      if (kind == 0) {
        len = (tag >> 2) + 1;
        if (len > 60) {
          const uint32_t nb = len - 60;
          if (ilen - ip < nb) { err = kErrFormat; return; }
          len = 0;
          for (uint32_t i = 0; i < nb; ++i) len |= byte(ip + i) << (8 * i);
          len += 1;
          ip += nb;
        }
        if (len > ilen - ip || len > olen - op) { err = kErrFormat; return; }
        literal(ip, len);
        ip += len;
        continue;
      }
      if (kind == 1) {
        if (ip >= ilen) { err = kErrFormat; return; }
        len = 4 + ((tag >> 2) & 7);
        off = ((tag >> 5) << 8) | byte(ip++);
      } else if (kind == 2) {
        if (ilen - ip < 2) { err = kErrFormat; return; }
        len = (tag >> 2) + 1;
        off = byte(ip) | (byte(ip + 1) << 8);
        ip += 2;
      } else {
        if (ilen - ip < 4) { err = kErrFormat; return; }
        len = (tag >> 2) + 1;
        off = byte(ip) | (byte(ip + 1) << 8) | (byte(ip + 2) << 16) | (byte(ip + 3) << 24);
        ip += 4;
      }
      if (len > olen - op) { err = kErrFormat; return; }
      match(off, len);
    }
    if (!err && op != olen) err = kErrFormat;
  }
  // LZ4 frame data blocks (after the frame header): [u32 size|flag][data][u32 bcs?]...
  __device__ void lz4_frame_blocks(bool block_checksum) {
    uint32_t ip = 0;
    while (!err) {
      if (ilen - ip < 4) { err = kErrFormat; return; }
      ensure(ip);
      uint32_t bs = byte(ip) | (byte(ip + 1) << 8) | (byte(ip + 2) << 16) | (byte(ip + 3) << 24);
      ip += 4;
      if (bs == 0) return;  // end mark
      const bool stored = bs & 0x80000000u;
      bs &= 0x7fffffffu;
      if (bs > ilen - ip) { err = kErrFormat; return; }
      if (stored) {
        if (bs > ocap - op) { err = kErrOverflow; return; }
        for (uint32_t done = 0; done < bs; done += kInW / 2) {
          const uint32_t n = bs - done < kInW / 2 ? bs - done : kInW / 2;
          ensure(ip + done);
          literal(ip + done, n);
        }
        ip += bs;
      } else {
        const uint32_t end = ip + bs;
        lz4_block(ip, end);
        ip = end;
      }
      if (block_checksum) ip += 4;
    }
  }
};

__global__ __launch_bounds__(64) void decompress_kernel(int codec, const uint8_t *__restrict__ src,
                                                        uint8_t *__restrict__ dst,
                                                        const strom_decomp_desc *__restrict__ desc,
                                                        uint32_t nblocks, int32_t *status) {
  __shared__ uint8_t ring[kRing];
  __shared__ __attribute__((aligned(16))) uint8_t inw[kInW];
  for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const strom_decomp_desc d = desc[b];
    Decoder dec;
    dec.in = src + d.src_off;
    dec.out = dst + d.dst_off;
    dec.ilen = d.src_len;
    dec.ocap = d.dst_len;
    dec.ring = ring;
    dec.inw = inw;
    dec.lane = threadIdx.x;
    switch (codec) {
      case STROM_CODEC_LZ4:
        dec.lz4_block(0, dec.ilen);
        break;
      case STROM_CODEC_SNAPPY:
        dec.snappy();
        break;
      case STROM_CODEC_COPY:
        if (dec.ilen > dec.ocap) {
          dec.err = kErrOverflow;
        } else {
          for (uint32_t done = 0; done < dec.ilen; done += kInW / 2) {
            const uint32_t n = dec.ilen - done < kInW / 2 ? dec.ilen - done : kInW / 2;
            dec.ensure(done);
            dec.literal(done, n);
          }
        }
        break;
      default:  // LZ4 frame blocks, with (5) or without (4) block checksums
        dec.lz4_frame_blocks(codec == STROM_CODEC_LZ4_FRAME_BCS);
        break;
    }
    if (threadIdx.x == 0) status[b] = dec.err ? dec.err : (int32_t)dec.op;
    lds_sync();
  }
}

}  // namespace

extern "C" int strom_decompress(int codec, const void *d_src, void *d_dst,
                                const strom_decomp_desc *d_desc, uint32_t nblocks,
                                int32_t *d_status, void *stream) {
  if (codec < STROM_CODEC_LZ4 || codec > STROM_CODEC_LZ4_FRAME_BCS) return -22;
  if (!nblocks) return 0;
  uint32_t grid = nblocks < 4096 ? nblocks : 4096;
  hipLaunchKernelGGL(decompress_kernel, dim3(grid), dim3(64), 0, (hipStream_t)stream, codec,
                     (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nblocks, d_status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
