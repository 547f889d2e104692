// decompress.hip — LZ4 / snappy decode of HBM-resident buffers on CDNA4.
//
// North-star config 5 (BASELINE.json): compressed columnar files land in HBM
// through the engine and are decompressed on the GPU before the filter.  The
// reference has no decompressor; this is new MI355X-side work.
//
// One 64-lane workgroup (= one wavefront) decodes one stream at a time
// (grid-stride over descriptors).  Parsing is wave-uniform; byte moves are
// spread over the 64 lanes.  Two LDS structures keep latency off the serial
// parse path:
//   * a 16 KiB input window: tokens/lengths/offsets are read from LDS, the
//     window is refilled with one coalesced sweep when the parser leaves it;
//   * a 64 KiB history ring: LZ4 match distances are < 64 KiB, so every
//     match source is in LDS.  Output is flushed ring -> HBM in >= 4 KiB
//     sweeps (coalesced byte stores), never re-read from HBM.
// Overlapping matches use the periodic form out[s+k] = out[s-off+(k mod off)]
// so a piece never reads bytes it writes; pieces are <= 4 KiB and fenced by
// a barrier.  Snappy copies farther than 64 KiB (legal in the format, never
// produced by 64 KiB-fragment compressors) read the already-flushed HBM.
//
// Codecs: raw LZ4 block, LZ4 frame block sequence (linked or independent
// blocks, optional per-block checksums skipped), raw snappy, stored copy.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "strom/strom.h"

namespace {

constexpr uint32_t kRing = 1u << 16;
constexpr uint32_t kMask = kRing - 1;
constexpr uint32_t kInW = 16u << 10;
constexpr uint32_t kPiece = 4096;

enum : int32_t { kErrFormat = -1, kErrOverflow = -2, kErrDistance = -3 };

struct Decoder {
  const uint8_t *in;
  uint8_t *out;
  uint64_t ilen, ocap;
  uint64_t op = 0, flushed = 0, win = ~0ull;
  int32_t err = 0;
  uint8_t *ring;
  uint8_t *inw;
  uint32_t lane;

  __device__ void load_window(uint64_t at) {
    __syncthreads();
    for (uint32_t k = lane; k < kInW && at + k < ilen; k += 64) inw[k] = in[at + k];
    win = at;
    __syncthreads();
  }
  __device__ uint32_t byte(uint64_t p) {
    if (p < win || p >= win + kInW) load_window(p);
    return inw[p - win];
  }
  __device__ void flush(uint64_t upto) {
    for (uint64_t k = flushed + lane; k < upto; k += 64) out[k] = ring[k & kMask];
    flushed = upto;
  }
  __device__ void after_piece() {
    __syncthreads();
    if (op - flushed >= kPiece) flush(op);
  }
  // literal bytes src[ip, ip+len) -> output
  __device__ void literal(uint64_t ip, uint64_t len) {
    for (uint64_t done = 0; done < len;) {
      uint64_t n = len - done < kPiece ? len - done : kPiece;
      for (uint64_t k = lane; k < n; k += 64) {
        uint64_t p = ip + done + k;
        uint8_t v = (p >= win && p < win + kInW) ? inw[p - win] : in[p];
        ring[(op + k) & kMask] = v;
      }
      op += n;
      done += n;
      after_piece();
    }
  }
  __device__ void match(uint64_t off, uint64_t len) {
    if (off == 0 || off > op) {
      err = kErrFormat;
      return;
    }
    if (off > kRing - 1) {
      // far copy (snappy only): sources were flushed long ago
      flush(op);
      __threadfence();
      __syncthreads();
      for (uint64_t done = 0; done < len;) {
        uint64_t n = len - done < kPiece ? len - done : kPiece;
        for (uint64_t k = lane; k < n; k += 64) ring[(op + k) & kMask] = out[op - off + k];
        op += n;
        done += n;
        after_piece();
      }
      return;
    }
    for (uint64_t done = 0; done < len;) {
      uint64_t n = len - done < kPiece ? len - done : kPiece;
      if (off > kRing - kPiece && n > kRing - off) n = kRing - off;  // keep sources intact
      const uint64_t s = op;
      if (off >= n) {
        for (uint64_t k = lane; k < n; k += 64) ring[(s + k) & kMask] = ring[(s - off + k) & kMask];
      } else {
        for (uint64_t k = lane; k < n; k += 64)
          ring[(s + k) & kMask] = ring[(s - off + (k % off)) & kMask];
      }
      op += n;
      done += n;
      after_piece();
    }
  }
  // one raw LZ4 block occupying src[ip, end); returns new ip
  __device__ uint64_t lz4_block(uint64_t ip, uint64_t end) {
    while (ip < end && !err) {
      uint32_t token = byte(ip++);
      uint64_t lit = token >> 4;
      if (lit == 15) {
        uint32_t b;
        do {
          if (ip >= end) { err = kErrFormat; return ip; }
          b = byte(ip++);
          lit += b;
        } while (b == 255);
      }
      if (ip + lit > end) { err = kErrFormat; return ip; }
      if (op + lit > ocap) { err = kErrOverflow; return ip; }
      literal(ip, lit);
      ip += lit;
      if (ip >= end) break;  // last sequence carries literals only
      if (ip + 2 > end) { err = kErrFormat; return ip; }
      uint64_t off = byte(ip) | (byte(ip + 1) << 8);
      ip += 2;
      uint64_t ml = token & 15;
      if (ml == 15) {
        uint32_t b;
        do {
          if (ip >= end) { err = kErrFormat; return ip; }
          b = byte(ip++);
          ml += b;
        } while (b == 255);
      }
      ml += 4;
      if (op + ml > ocap) { err = kErrOverflow; return ip; }
      match(off, ml);
    }
    return ip;
  }
  __device__ void snappy() {
    uint64_t ip = 0, ulen = 0;
    for (int shift = 0;; shift += 7) {
      if (ip >= ilen || shift > 35) { err = kErrFormat; return; }
      uint32_t b = byte(ip++);
      ulen |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) break;
    }
    if (ulen > ocap) { err = kErrOverflow; return; }
    while (ip < ilen && !err) {
      uint32_t tag = byte(ip++);
      uint64_t len, off;
      uint32_t kind = tag & 3;
      if (kind == 0) {
        len = (tag >> 2) + 1;
        if (len > 60) {
          uint32_t nb = (uint32_t)len - 60;
          if (ip + nb > ilen) { err = kErrFormat; return; }
          len = 0;
          for (uint32_t i = 0; i < nb; ++i) len |= (uint64_t)byte(ip + i) << (8 * i);
          len += 1;
          ip += nb;
        }
        if (ip + len > ilen || op + len > ulen) { err = kErrFormat; return; }
        literal(ip, len);
        ip += len;
        continue;
      }
      if (kind == 1) {
        if (ip >= ilen) { err = kErrFormat; return; }
        len = 4 + ((tag >> 2) & 7);
        off = ((uint64_t)(tag >> 5) << 8) | byte(ip++);
      } else if (kind == 2) {
        if (ip + 2 > ilen) { err = kErrFormat; return; }
        len = (tag >> 2) + 1;
        off = byte(ip) | (byte(ip + 1) << 8);
        ip += 2;
      } else {
        if (ip + 4 > ilen) { err = kErrFormat; return; }
        len = (tag >> 2) + 1;
        off = byte(ip) | (byte(ip + 1) << 8) | (byte(ip + 2) << 16) | ((uint64_t)byte(ip + 3) << 24);
        ip += 4;
      }
      if (op + len > ulen) { err = kErrFormat; return; }
      match(off, len);
    }
    if (!err && op != ulen) err = kErrFormat;
  }
  // LZ4 frame data blocks (after the frame header): [u32 size|flag][data][u32 bcs?]...
  __device__ void lz4_frame_blocks(bool block_checksum) {
    uint64_t ip = 0;
    while (!err) {
      if (ip + 4 > ilen) { err = kErrFormat; return; }
      uint32_t bs = byte(ip) | (byte(ip + 1) << 8) | (byte(ip + 2) << 16) | (byte(ip + 3) << 24);
      ip += 4;
      if (bs == 0) return;  // end mark
      bool stored = bs & 0x80000000u;
      bs &= 0x7fffffffu;
      if (ip + bs > ilen) { err = kErrFormat; return; }
      if (stored) {
        if (op + bs > ocap) { err = kErrOverflow; return; }
        literal(ip, bs);
        ip += bs;
      } else {
        uint64_t end = ip + bs;
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
  __shared__ uint8_t inw[kInW];
  for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    strom_decomp_desc d = desc[b];
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
        if (dec.ilen > dec.ocap) dec.err = kErrOverflow;
        else dec.literal(0, dec.ilen);
        break;
      default:  // LZ4 frame blocks, with (5) or without (4) block checksums
        dec.lz4_frame_blocks(codec == 5);
        break;
    }
    __syncthreads();
    dec.flush(dec.op);
    if (threadIdx.x == 0) status[b] = dec.err ? dec.err : (int32_t)dec.op;
    __syncthreads();
  }
}

}  // namespace

extern "C" int strom_decompress(int codec, const void *d_src, void *d_dst,
                                const strom_decomp_desc *d_desc, uint32_t nblocks,
                                int32_t *d_status, void *stream) {
  if (codec < STROM_CODEC_LZ4 || codec > 5) return -22;
  if (!nblocks) return 0;
  uint32_t grid = nblocks < 2048 ? nblocks : 2048;
  hipLaunchKernelGGL(decompress_kernel, dim3(grid), dim3(64), 0, (hipStream_t)stream, codec,
                     (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nblocks, d_status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
