// decompress_wave.hip — wave-per-stream LZ4 / snappy decoder for few, long
// streams (config 5: an Arrow LZ4 column is ~2k frames of linked 64 KiB
// blocks, i.e. ~2k serial streams of 512 KiB).
//
// The lane-group decoder (decompress.hip) advances 16 streams per wave and
// wins when there are tens of thousands of streams; with a few thousand it
// leaves most SIMDs idle and each stream moves at ~10 MB/s.  Here one wave
// owns one stream and splits the work so the serial part is as short as
// possible:
//   1. parse: up to 64 sequences are parsed on the scalar path (one 16-byte
//      LDS broadcast read per sequence, uniform branches) into a lane table
//      (lane j = sequence j: literal source, output offset, match offset
//      and length);
//   2. literals: every lane copies its own sequence's literal run (they never
//      overlap), 4 bytes per lane per step;
//   3. matches whose source lies wholly before the batch (and far matches,
//      read back from HBM) are copied lane-parallel as well; the rest — a
//      match reading bytes this batch produced — are copied in order, each
//      by the whole wave (LDS executes a wave's accesses in order, so a
//      pass only waits for its own reads);
//   4. the batch's output leaves the LDS history ring as 16-byte stores.
// LDS per wave: 16 KiB ring + 2 KiB input window, so 8 waves (streams) per
// CU are resident: 2,048 streams fill the chip.
//
// Codecs and error semantics are those of decompress.hip (raw LZ4 block,
// LZ4 frame blocks, Arrow IPC compressed buffer, raw snappy, stored copy);
// the dispatcher in decompress.hip picks this kernel by stream count.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "strom/strom.h"

namespace {

constexpr uint32_t kRing = 16384, kRMask = kRing - 1;   // history ring (LDS)
constexpr uint32_t kInW = 2048;                          // input window (LDS)
constexpr uint32_t kNB = 64;                             // sequences per batch
constexpr uint32_t kBOut = 4096;                         // output bytes per batch
constexpr uint32_t kNear = kRing - kBOut - 256;          // batch: offsets served by the ring
constexpr uint32_t kPass = 256;                          // wave-wide copy pass
constexpr uint32_t kSNear = kRing - 2 * kPass;           // streaming: offsets served by the ring
constexpr uint32_t kPace = kRing / 2;                    // streaming: unflushed bytes bound
constexpr uint32_t kShort = 64;                          // lane-parallel copy limit
static_assert(kPace + 2 * kPass <= kRing && kBOut + kShort < kNear, "ring budget");

enum : int32_t { kErrFormat = -1, kErrOverflow = -2 };
enum : uint32_t { kHdr = 0, kLz4 = 1, kSnappy = 2, kDone = 3 };

// Optional cycle profile (-DSTROM_WAVE_PROF, tools/wave_prof.py): s_memtime
// spans per phase and event counts, summed over waves (lane 0).
enum : int { kTParse, kTLit, kTPar, kTSerial, kTFlush, kTSingle, kTRefill, kTTotal,
             kNBatch, kNUnits, kNSingle, kNSerial, kNPar, kNRefill, kNFence, kNFlush, kWN };
#ifdef STROM_WAVE_PROF
__device__ unsigned long long g_wprof[kWN];
#define WP_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define WP_ADD(k, v) (prof[k] += __builtin_amdgcn_s_memtime() - (v))
#define WP_CNT(k, n) (prof[k] += (n))
#else
#define WP_T0(v) (void)0
#define WP_ADD(k, v) (void)0
#define WP_CNT(k, n) (void)0
#endif

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t j) {
  return __builtin_amdgcn_readlane((int)v, (int)j);
}
// lane j of old := v (v, j wave-uniform)
__device__ __forceinline__ uint32_t wrl(uint32_t v, uint32_t j, uint32_t old, uint32_t lane) {
  return lane == j ? v : old;
}

// One decoded unit: literal run [lsrc, lsrc + lit) of the input, then a
// match of m bytes at distance off (m == 0: none); next = following unit.
struct Seq {
  uint32_t lsrc, lit, off, m, next;
};

struct WaveStream {
  const uint8_t *ina;  // 16-aligned input base (P space = offsets from here)
  uint8_t *out;
  uint8_t *ring;
  uint8_t *inw;
  uint8_t *sink;       // per-lane target of masked-off byte stores
  uint32_t *pv;        // resolve batches: per output byte a value or a source
  uint32_t lane;
  uint32_t iend, ocap, ip, op, bend, win, flushed, fenced, omis, olen, bcs, fhdr, mode;
  int32_t err;
#ifdef STROM_WAVE_PROF
  uint64_t prof[kWN];
#endif

  // ---------------------------------------------------------------- input
  // window = P-space [win, win + kInW), win 16-aligned; chunks past the
  // stream end read as zeros (a 16-B chunk holding a stream byte is mapped)
  __device__ void refill(uint32_t p) {
    WP_T0(t0);
    WP_CNT(kNRefill, 1);
    win = p & ~15u;
#pragma unroll
    for (uint32_t u = 0; u < kInW / (16 * 64); ++u) {
      const uint32_t c = 16 * (lane + 64 * u);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (win + c < iend) v = *(const uint4 *)(ina + win + c);
      *(uint4 *)(inw + c) = v;
    }
    WP_ADD(kTRefill, t0);
  }
  __device__ __forceinline__ bool in_window(uint32_t p, uint32_t need) const {
    return p - win <= kInW - need;   // unsigned: p < win wraps high
  }
  // byte p with the window moved to it when needed (header / slow paths)
  __device__ uint32_t rb(uint32_t p) {
    if (!in_window(p, 8)) refill(p);
    const uint32_t o = p - win;
    return rfl(*(const uint32_t *)(inw + (o & ~3u))) >> (8 * (o & 3)) & 0xff;
  }
  __device__ uint32_t rb4(uint32_t p) {
    return rb(p) | rb(p + 1) << 8 | rb(p + 2) << 16 | rb(p + 3) << 24;
  }
  // 16 bytes at p (window must hold [p, p + 20)), as four words
  __device__ __forceinline__ void rd16(uint32_t p, uint32_t w[4]) const {
    const uint32_t o = p - win;
    const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
    const uint32_t sh = o & 3;
    uint32_t x[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) x[i] = rfl(d[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = __builtin_amdgcn_alignbyte(x[i + 1], x[i], sh);
  }
  static __device__ __forceinline__ uint32_t byte_of(const uint32_t w[4], uint32_t i) {
    const uint32_t q = i >> 2;
    const uint32_t v = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
    return v >> (8 * (i & 3)) & 0xff;
  }

  // --------------------------------------------------------------- output
  __device__ __forceinline__ void put4(uint32_t pos, uint32_t v, uint32_t n) {
    const uint32_t a = pos + omis;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      uint8_t *d = j < n ? ring + ((a + j) & kRMask) : sink + 4 * lane + j;
      *d = (uint8_t)(v >> (8 * j));
    }
  }
  // 4 ring bytes from output position x (any alignment)
  __device__ __forceinline__ uint32_t ring4(uint32_t x) const {
    const uint32_t r = x + omis;
    const uint32_t a = r & kRMask & ~3u;
    const uint32_t d0 = *(const uint32_t *)(ring + a);
    const uint32_t d1 = *(const uint32_t *)(ring + ((a + 4) & kRMask));
    return __builtin_amdgcn_alignbyte(d1, d0, r & 3);
  }
  // 4 bytes of stored output at x (L1-bypassing: written by this wave)
  __device__ __forceinline__ uint32_t hbm4(uint32_t x) const {
    const uintptr_t q = (uintptr_t)(out + x);
    const uint32_t *w = (const uint32_t *)(q & ~(uintptr_t)3);
    const uint32_t d0 = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t d1 = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)(q & 3));
  }

  // ring bytes [flushed, upto) -> HBM: whole 16-B chunks as dwordx4 stores
  // (out + 16c - omis is 16-aligned), partial chunks byte by byte; exact =
  // false leaves a partial last chunk for later
  __device__ void flush(uint32_t upto, bool exact) {
    const uint32_t rb0 = flushed + omis, re = upto + omis;
    const uint32_t cb = rb0 >> 4, ce = exact ? (re + 15) >> 4 : re >> 4;
    if (ce <= cb) return;
    WP_T0(t0);
    WP_CNT(kNFlush, 1);
    for (uint32_t c = cb + lane; c < ce; c += 64) {
      const uint32_t r0 = c << 4;
      const uint4 v = *(const uint4 *)(ring + (r0 & kRMask));
      if (r0 >= rb0 && r0 + 16 <= re) {
        *(uint4 *)(out + (r0 - omis)) = v;
      } else {
        const uint32_t lo = r0 < rb0 ? rb0 : r0, hi = r0 + 16 > re ? re : r0 + 16;
        for (uint32_t x = lo; x < hi; ++x) {
          const uint32_t i = x - r0;
          const uint32_t w = i < 8 ? (i < 4 ? v.x : v.y) : (i < 12 ? v.z : v.w);
          out[x - omis] = (uint8_t)(w >> (8 * (i & 3)));
        }
      }
    }
    const uint32_t nf = exact ? upto : (ce << 4) - omis;
    if (nf > flushed) flushed = nf;
    WP_ADD(kTFlush, t0);
  }
  // far sources [.., end) must be stored and visible to L1-bypassing loads
  __device__ __forceinline__ void far_ready(uint32_t end) {
    if (end > flushed) flush(end, true);
    if (end > fenced) {
      WP_CNT(kNFence, 1);
      // this wave's stores done at its XCD's L2 (s_waitcnt vmcnt(0)); the
      // readers are this wave's own L1-bypassing loads, so no L2 write-back
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      fenced = flushed;
    }
  }
  __device__ __forceinline__ void pace(uint32_t cur) {
    if (cur - flushed >= kPace) flush(cur, false);
  }

  // literal [p, p + len) -> output at op, window moved as needed (long runs)
  __device__ void literal_stream(uint32_t p, uint32_t len) {
    const uint32_t k = 4 * lane;
    for (uint32_t done = 0; done < len; done += kPass) {
      const uint32_t n = len - done < kPass ? len - done : kPass;
      if (!in_window(p + done, kPass + 8)) refill(p + done);
      if (k < n) {
        const uint32_t o = p + done + k - win;
        const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
        put4(op + done + k, __builtin_amdgcn_alignbyte(d[1], d[0], o & 3), n - k);
      }
      pace(op + done + n);
    }
    op += len;
  }

  // match of m bytes at distance off written at output position d, by the
  // whole wave in passes of 256 B.  Byte i = out[d - off + (i mod off)]; for
  // off < 256 each pass uses the same residues relative to its own start
  // (the output from d - off on is periodic), and every source byte lies
  // before the pass.  stream: pace the ring (long matches).
  __device__ void match_wave(uint32_t d, uint32_t off, uint32_t m, bool stream) {
    const uint32_t k = 4 * lane;
    if (off > (stream ? kSNear : kNear)) {
      for (uint32_t done = 0; done < m; done += kPass) {
        const uint32_t n = m - done < kPass ? m - done : kPass;
        const uint32_t s = d + done - off;     // off > n: sources end before the pass
        far_ready(s + n);
        if (k < n) put4(d + done + k, hbm4(s + k), n - k);
        if (stream) pace(d + done + n);
      }
    } else if (off >= kPass) {
      for (uint32_t done = 0; done < m; done += kPass) {
        const uint32_t n = m - done < kPass ? m - done : kPass;
        if (k < n) put4(d + done + k, ring4(d + done - off + k), n - k);
        if (stream) pace(d + done + n);
      }
    } else {
      // k mod off for k < 256 by a float reciprocal (error far below 1/256,
      // corrected by one compare)
      uint32_t q = (uint32_t)((float)k * __builtin_amdgcn_rcpf((float)off));
      uint32_t r = k - q * off;
      if ((int32_t)r < 0) r += off;
      else if (r >= off) r -= off;
      uint32_t rr[4];
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        rr[j] = r;
        r = r + 1 == off ? 0 : r + 1;
      }
      for (uint32_t done = 0; done < m; done += kPass) {
        const uint32_t n = m - done < kPass ? m - done : kPass;
        const uint32_t base = d + done - off + omis;
        uint32_t v = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) v |= (uint32_t)ring[(base + rr[j]) & kRMask] << (8 * j);
        if (k < n) put4(d + done + k, v, n > k ? n - k : 0);
        if (stream) pace(d + done + n);
      }
    }
  }

  // ------------------------------------------------------------ parsing
  // Generic unit parse at p through rb() (window moves as needed).
  // Returns 0 or an error.
  template <bool kSnap>
  __device__ int32_t parse_slow(uint32_t p, Seq &q) {
    if (!kSnap) {
      const uint32_t t = rb(p++);
      uint32_t lit = t >> 4, ml = t & 15;
      if (lit == 15) {
        uint32_t b;
        do {
          if (p >= bend) return kErrFormat;
          b = rb(p++);
          lit += b;
        } while (b == 255);
      }
      if (lit > bend - p) return kErrFormat;
      q.lsrc = p;
      q.lit = lit;
      p += lit;
      q.off = 0;
      q.m = 0;
      if (p >= bend) { q.next = p; return 0; }      // last sequence: literals only
      if (bend - p < 2) return kErrFormat;
      q.off = rb(p) | rb(p + 1) << 8;
      p += 2;
      if (ml == 15) {
        uint32_t b;
        do {
          if (p >= bend) return kErrFormat;
          b = rb(p++);
          ml += b;
        } while (b == 255);
      }
      q.m = ml + 4;
      q.next = p;
      return 0;
    }
    const uint32_t tag = rb(p++), kind = tag & 3;
    q.lit = 0;
    q.m = 0;
    q.off = 0;
    q.lsrc = p;
    if (kind == 0) {
      uint32_t len = (tag >> 2) + 1;
      if (len > 60) {
        const uint32_t nb = len - 60;
        if (iend - p < nb) return kErrFormat;
        uint32_t x = 0;
        for (uint32_t i = 0; i < nb; ++i) x |= rb(p + i) << (8 * i);
        len = x + 1;
        if (len == 0) return kErrFormat;
        p += nb;
      }
      if (len > iend - p) return kErrFormat;
      q.lsrc = p;
      q.lit = len;
      q.next = p + len;
      return 0;
    }
    const uint32_t nb = kind == 1 ? 1 : kind == 2 ? 2 : 4;
    if (iend - p < nb) return kErrFormat;
    if (kind == 1) {
      q.m = 4 + ((tag >> 2) & 7);
      q.off = ((tag >> 5) << 8) | rb(p);
    } else {
      q.m = (tag >> 2) + 1;
      q.off = kind == 2 ? (rb(p) | rb(p + 1) << 8) : rb4(p);
    }
    q.next = p + nb;
    return 0;
  }

  // The common unit from one 16-byte read; false: take parse_slow (the
  // window must hold [p, p + 20))
  template <bool kSnap>
  __device__ __forceinline__ bool parse_fast(uint32_t p, Seq &q) const {
    uint32_t w[4];
    rd16(p, w);
    if (!kSnap) {
      const uint32_t t = w[0] & 0xff, lit = t >> 4, ml = t & 15;
      if (lit > 12) return false;
      const uint32_t po = 1 + lit;               // offset bytes po, po + 1; extension po + 2
      const uint32_t lsrc = p + 1, e = p + po;   // e = end of literals
      if (lit > bend - lsrc) return false;
      q.lsrc = lsrc;
      q.lit = lit;
      if (e >= bend) {
        q.m = 0;
        q.off = 0;
        q.next = e;
        return true;
      }
      if (bend - e < 3) return false;
      q.off = byte_of(w, po) | byte_of(w, po + 1) << 8;
      if (ml == 15) {
        const uint32_t x = byte_of(w, po + 2);
        if (x == 255) return false;
        q.m = 19 + x;
        q.next = e + 3;
      } else {
        q.m = ml + 4;
        q.next = e + 2;
      }
      return true;
    }
    const uint32_t tag = w[0] & 0xff, kind = tag & 3;
    if (iend - p < 6) return false;
    q.lit = 0;
    q.m = 0;
    q.off = 0;
    q.lsrc = p + 1;
    if (kind == 0) {
      uint32_t len = (tag >> 2) + 1, h = 1;
      if (len > 60) {
        const uint32_t nb = len - 60;
        const uint32_t x = nb == 4 ? (w[0] >> 8 | w[1] << 24) : (w[0] >> 8) & ((1u << (8 * nb)) - 1);
        if (x == 0xffffffffu) return false;
        len = x + 1;
        h += nb;
      }
      q.lsrc = p + h;
      q.lit = len;
      q.next = p + h + len;   // overflow / range checked by the caller
      return len <= iend - (p + h);
    }
    if (kind == 1) {
      q.m = 4 + ((tag >> 2) & 7);
      q.off = ((tag >> 5) << 8) | (w[0] >> 8 & 0xff);
      q.next = p + 2;
    } else if (kind == 2) {
      q.m = (tag >> 2) + 1;
      q.off = w[0] >> 8 & 0xffff;
      q.next = p + 3;
    } else {
      q.m = (tag >> 2) + 1;
      q.off = w[0] >> 8 | w[1] << 24;
      q.next = p + 5;
    }
    return true;
  }

  __device__ __forceinline__ uint32_t cap() const { return mode == kSnappy ? olen : ocap; }

  // validity of a unit producing output at o (checks shared by both paths)
  __device__ __forceinline__ int32_t check(const Seq &q, uint32_t o) const {
    const uint32_t c = cap();
    if (q.lit > c - o) return mode == kSnappy ? kErrFormat : kErrOverflow;
    if (q.m) {
      if (q.m > c - o - q.lit) return mode == kSnappy ? kErrFormat : kErrOverflow;
      if (q.off == 0 || q.off > o + q.lit) return kErrFormat;
    }
    return 0;
  }

  // --------------------------------------------------------------- batch
  // Parse and copy up to 64 units.  false: the unit at ip does not fit a
  // batch (long run, window edge, error) — the caller streams it alone.
  template <bool kSnap>
  __device__ bool batch() {
    if (!in_window(ip, kInW / 2)) refill(ip);
    WP_T0(tp);
    const uint32_t lim = kSnap ? iend : bend;
    uint32_t A = 0, B = 0, C = 0, D = 0;     // lane j: unit j (lsrc | rel,lit | off | m)
    uint32_t nb = 0, bout = 0, maxlit = 0, maxm = 0;
    uint64_t longlit = 0, serial = 0, par = 0;
    bool any_far = false;
    uint32_t far_end = 0;
    uint32_t p = ip;
    while (nb < kNB && p < lim && in_window(p, 24)) {
      Seq q;
      if (!parse_fast<kSnap>(p, q)) break;
      const uint32_t o = op + bout;
      if (check(q, o)) break;
      if (q.lit + q.m > kBOut - bout) break;
      if (!in_window(q.lsrc, 8) || q.lit > kInW - 8 - (q.lsrc - win)) break;
      A = wrl(q.lsrc, nb, A, lane);
      B = wrl(bout | q.lit << 16, nb, B, lane);
      C = wrl(q.off, nb, C, lane);
      D = wrl(q.m, nb, D, lane);
      const uint64_t bit = 1ull << nb;
      if (q.lit > kShort) longlit |= bit;
      else if (q.lit > maxlit) maxlit = q.lit;
      if (q.m) {
        // independent: the source lies wholly before this batch's output
        if (q.m <= kShort && bout + q.lit + q.m <= q.off) {
          par |= bit;
          if (q.m > maxm) maxm = q.m;
          if (q.off > kNear) {
            any_far = true;
            const uint32_t e = o + q.lit + q.m - q.off + 8;
            if (e > far_end) far_end = e;
          }
        } else {
          serial |= bit;
        }
      }
      bout += q.lit + q.m;
      ++nb;
      p = q.next;
      if (!kSnap && q.m == 0) break;    // last sequence of the block
    }
    if (nb == 0) return false;
    WP_ADD(kTParse, tp);
    WP_CNT(kNBatch, 1);
    WP_CNT(kNUnits, nb);
    WP_CNT(kNSerial, __builtin_popcountll(serial));
    WP_CNT(kNPar, __builtin_popcountll(par));
    WP_T0(tl);
    const bool act = lane < nb;
    const uint32_t rel = B & 0xffff, lit = B >> 16;
    const uint32_t dlit = op + rel, dm = dlit + lit;
    // (1) literals: lane j copies unit j's run
    {
      const uint32_t my = act && lit <= kShort ? lit : 0;
      for (uint32_t k = 0; k < maxlit; k += 4) {
        const uint32_t o = k < my ? A + k - win : 0;
        const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
        const uint32_t v = __builtin_amdgcn_alignbyte(d[1], d[0], o & 3);
        put4(dlit + k, v, k < my ? my - k : 0);
      }
      for (uint64_t mk = longlit; mk; mk &= mk - 1) {
        const uint32_t j = __builtin_ctzll(mk);
        const uint32_t src = rdl(A, j), n = rdl(B, j) >> 16, dst = op + (rdl(B, j) & 0xffff);
        for (uint32_t done = 0; done < n; done += kPass) {
          const uint32_t k = 4 * lane, c = n - done < kPass ? n - done : kPass;
          if (k < c) {
            const uint32_t o = src + done + k - win;
            const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
            put4(dst + done + k, __builtin_amdgcn_alignbyte(d[1], d[0], o & 3), c - k);
          }
        }
      }
    }
    WP_ADD(kTLit, tl);
    WP_T0(tq);
    // (2) independent matches, lane-parallel (far ones from HBM)
    if (par) {
      if (any_far) far_ready(far_end);
      const bool mine = (par >> lane) & 1;
      const uint32_t my = mine ? D : 0, off = C;
      const bool far = mine && off > kNear;
      for (uint32_t k = 0; k < maxm; k += 4) {
        const uint32_t x = dm - off + k;
        uint32_t v;
        if (far) v = k < my ? hbm4(x) : 0;
        else v = ring4(k < my ? x : 0);
        put4(dm + k, v, k < my ? my - k : 0);
      }
    }
    WP_ADD(kTPar, tq);
    WP_T0(ts);
    // (3) matches reading this batch's output, in order
    for (uint64_t mk = serial; mk; mk &= mk - 1) {
      const uint32_t j = __builtin_ctzll(mk);
      const uint32_t b = rdl(B, j);
      match_wave(op + (b & 0xffff) + (b >> 16), rdl(C, j), rdl(D, j), false);
    }
    WP_ADD(kTSerial, ts);
    op += bout;
    ip = p;
    return true;
  }

  // ---- resolve batch (LZ4, STROM_DECOMP_G=65): a lean scalar parse of up
  // to 64 sequences, then every output byte of the batch is resolved at once
  // — literal bytes carry their value, match byte x points at x - off — by
  // pointer doubling (pv[x] = pv[pv[x]], lane-parallel) until each entry is
  // a value or history before the batch (ring, or HBM past the ring).  No
  // match is copied sequence by sequence.
  static constexpr uint32_t kRB = 1024;         // output bytes per resolve batch
  // pv entry: bits 31:30 = 01 a byte value, 00 a source inside the batch,
  // 11 a (negative) source before it; sources stay within +-2^29
  static constexpr uint32_t kVal = 0x40000000u;
  __device__ bool batch_res() {
    if (!in_window(ip, kInW / 2)) refill(ip);
    uint32_t A = 0, B = 0, C = 0;
    uint32_t nb = 0, bout = 0, maxshort = 0;
    uint64_t longmask = 0;
    uint32_t p = ip;
    while (nb < kNB && p < bend && in_window(p, 24)) {
      const uint32_t o = p - win;
      const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
      const uint32_t x0 = rfl(d[0]), x1 = rfl(d[1]), x2 = rfl(d[2]), x3 = rfl(d[3]), x4 = rfl(d[4]);
      const uint32_t sh = 8 * (o & 3);
      const uint32_t w0 = (uint32_t)((((uint64_t)x1 << 32) | x0) >> sh);
      const uint32_t w1 = (uint32_t)((((uint64_t)x2 << 32) | x1) >> sh);
      const uint32_t w2 = (uint32_t)((((uint64_t)x3 << 32) | x2) >> sh);
      const uint32_t w3 = (uint32_t)((((uint64_t)x4 << 32) | x3) >> sh);
      const uint32_t lit = (w0 >> 4) & 15, ml = w0 & 15;
      const uint32_t e = p + 1 + lit;
      const uint32_t r = 1 + lit, sel = r >> 2;
      const uint32_t lo = sel == 0 ? w0 : sel == 1 ? w1 : sel == 2 ? w2 : w3;
      const uint32_t hi = sel == 0 ? w1 : sel == 1 ? w2 : w3;
      const uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (r & 3)));
      const uint32_t off = v & 0xffff, xb = (v >> 16) & 0xff;
      const bool last = e == bend;
      const uint32_t m = last ? 0u : (ml == 15 ? 19 + xb : ml + 4);
      const uint32_t oa = op + bout;
      const bool ok = (lit <= 12) & (e <= bend) & (last | (bend - e >= 3)) &
                      (last | (ml != 15) | (xb != 255)) &
                      (last | ((off != 0) & (off <= oa + lit))) & (lit + m <= ocap - oa) &
                      (lit + m <= kRB - bout);
      if (!ok) break;
      A = wrl(p + 1, nb, A, lane);
      B = wrl(bout | lit << 16, nb, B, lane);
      C = wrl(off | m << 16, nb, C, lane);
      const uint32_t n = lit + m;
      if (n > 32) longmask |= 1ull << nb;
      else if (n > maxshort) maxshort = n;
      bout += n;
      ++nb;
      p = last ? e : e + 2 + (ml == 15);
      if (last) break;
    }
    if (nb == 0) return false;
    const uint32_t rel = B & 0xffff, lit = B >> 16, off = C & 0xffff, m = C >> 16;
    const uint32_t n = lane < nb ? lit + m : 0u;
    // (1) fill: lane j writes record j (<= 32 bytes); longer records by the wave
    {
      const uint32_t my = n <= 32 ? n : 0u;
      for (uint32_t k = 0; k < maxshort; ++k) {
        if (k < my) {
          uint32_t val;
          if (k < lit) val = kVal | inw[A + k - win];
          else val = (uint32_t)((int32_t)(rel + k) - (int32_t)off);
          pv[rel + k] = val;
        }
      }
      for (uint64_t mk = longmask; mk; mk &= mk - 1) {
        const uint32_t j = __builtin_ctzll(mk);
        const uint32_t ja = rdl(A, j), jb = rdl(B, j), jc = rdl(C, j);
        const uint32_t jr = jb & 0xffff, jl = jb >> 16, jo = jc & 0xffff, jn = jl + (jc >> 16);
        for (uint32_t k = lane; k < jn; k += 64)
          pv[jr + k] = k < jl ? kVal | inw[ja + k - win] : (uint32_t)((int32_t)(jr + k) - (int32_t)jo);
      }
    }
    // (2) pointer doubling until every entry is a value or history (< 0)
    for (;;) {
      bool ch = false;
      for (uint32_t x = lane; x < bout; x += 64) {
        const uint32_t q = pv[x];
        if ((q >> 30) == 0) {
          pv[x] = pv[q];
          ch = true;
        }
      }
      if (!__any(ch)) break;
    }
    // (3) bytes into the ring; history from the ring, or HBM past it (a
    // resolved chain can end farther back than any single offset)
    bool need = false;
    for (uint32_t x = lane; x < bout; x += 64) {
      const uint32_t q = pv[x];
      need |= (q >> 30) == 3 && (uint32_t)(-(int32_t)q) > kNear;
    }
    if (__any(need)) far_ready(op);
    for (uint32_t x = lane; x < bout; x += 64) {
      const uint32_t q = pv[x];
      uint32_t byte;
      if ((q >> 30) == 1) {
        byte = q & 0xff;
      } else {
        const uint32_t h = op + (int32_t)q;     // absolute output position < op
        if (op - h <= kNear) {
          byte = ring[(h + omis) & kRMask];
        } else {
          const uintptr_t a = (uintptr_t)(out + h);
          const uint32_t w = __hip_atomic_load((const uint32_t *)(a & ~(uintptr_t)3), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
          byte = (w >> (8 * (a & 3))) & 0xff;
        }
      }
      ring[(op + x + omis) & kRMask] = (uint8_t)byte;
    }
    op += bout;
    ip = p;
    return true;
  }

  // one unit alone, window and ring paced (long runs, window edges, errors)
  template <bool kSnap>
  __device__ void single() {
    WP_T0(t0);
    WP_CNT(kNSingle, 1);
    Seq q;
    int32_t e = parse_slow<kSnap>(ip, q);
    if (!e) e = check(q, op);
    if (e) {
      err = e;
      return;
    }
    if (q.lit) literal_stream(q.lsrc, q.lit);
    if (q.m) {
      match_wave(op, q.off, q.m, true);
      op += q.m;
    }
    ip = q.next;
    WP_ADD(kTSingle, t0);
  }

  // ---------------------------------------------- stream-level headers
  template <bool kSnap>
  __device__ void header(int codec) {
    if (kSnap) codec = STROM_CODEC_SNAPPY;
    if (codec == STROM_CODEC_LZ4) {
      bend = iend;
      mode = kLz4;
    } else if (codec == STROM_CODEC_SNAPPY) {
      uint32_t p = ip, ulen = 0;
      for (uint32_t shift = 0;; shift += 7) {
        if (p >= iend || shift > 28) { err = kErrFormat; return; }
        const uint32_t b = rb(p++);
        if (shift == 28 && (b & 0x70)) { err = kErrOverflow; return; }
        ulen |= (b & 0x7f) << shift;
        if (!(b & 0x80)) break;
      }
      if (ulen > ocap) { err = kErrOverflow; return; }
      olen = ulen;
      ip = p;
      mode = kSnappy;
    } else if (codec == STROM_CODEC_COPY) {
      const uint32_t n = iend - ip;
      if (n > ocap) { err = kErrOverflow; return; }
      literal_stream(ip, n);
      ip = iend;
      mode = kDone;
    } else if (fhdr) {
      // Arrow IPC compressed buffer: int64 length (-1: raw), then a frame
      fhdr = 0;
      if (iend - ip < 8) { err = kErrFormat; return; }
      const uint32_t lo = rb4(ip), hi = rb4(ip + 4);
      ip += 8;
      if (lo == 0xffffffffu && hi == 0xffffffffu) {
        const uint32_t n = iend - ip;
        if (n > ocap) { err = kErrOverflow; return; }
        literal_stream(ip, n);
        ip = iend;
        mode = kDone;
        return;
      }
      if (hi != 0 || lo > ocap) { err = kErrOverflow; return; }
      if (iend - ip < 7 || rb4(ip) != 0x184D2204u) { err = kErrFormat; return; }
      const uint32_t flg = rb(ip + 4);
      if ((flg >> 6) != 1) { err = kErrFormat; return; }
      const uint32_t hl = 7 + ((flg & 0x08) ? 8 : 0) + ((flg & 0x01) ? 4 : 0);
      if (iend - ip < hl) { err = kErrFormat; return; }
      bcs = (flg & 0x10) ? 1 : 0;
      ip += hl;
    } else {
      // LZ4 frame data blocks: [u32 size | stored flag][data][u32 bcs?] ... [u32 0]
      if (iend - ip < 4) { err = kErrFormat; return; }
      uint32_t bs = rb4(ip);
      ip += 4;
      if (bs == 0) { mode = kDone; return; }
      const bool stored = bs & 0x80000000u;
      bs &= 0x7fffffffu;
      if (bs > iend - ip) { err = kErrFormat; return; }
      if (stored) {
        if (bs > ocap - op) { err = kErrOverflow; return; }
        literal_stream(ip, bs);
        ip += bs;
        if (bcs) ip += 4;
      } else {
        bend = ip + bs;
        mode = kLz4;
      }
    }
  }

  template <bool kSnap, bool kRes>
  __device__ void run(int codec) {
    while (!err && mode != kDone) {
      if (mode == kHdr) {
        header<kSnap>(codec);
      } else if (!kSnap && ip >= bend) {
        if (codec == STROM_CODEC_LZ4) {
          mode = kDone;
        } else {
          ip = bend + (bcs ? 4 : 0);
          mode = kHdr;
        }
      } else if (kSnap && ip >= iend) {
        if (op != olen) err = kErrFormat;
        mode = kDone;
      } else {
        if (!((kRes && !kSnap) ? batch_res() : batch<kSnap>())) single<kSnap>();
        flush(op, false);
      }
    }
    if (!err) flush(op, true);
  }
};

// one wave per workgroup; LDS (18.3 KiB) keeps 8 waves per CU
template <bool kSnap, bool kRes>
__global__ __launch_bounds__(64) void decompress_wave_kernel(int codec, const uint8_t *__restrict__ src,
                                                             uint8_t *__restrict__ dst,
                                                             const strom_decomp_desc *__restrict__ desc,
                                                             uint32_t nblocks, int32_t *status) {
  __shared__ __attribute__((aligned(16)))
  uint8_t lds[kRing + kInW + 16 + 256 + (kRes ? 4 * WaveStream::kRB : 0)];
  WaveStream s;
  s.lane = threadIdx.x;
  s.ring = lds;
  s.inw = lds + kRing;
  s.sink = lds + kRing + kInW + 16;
  s.pv = (uint32_t *)(lds + kRing + kInW + 16 + 256);
#ifdef STROM_WAVE_PROF
  for (int i = 0; i < kWN; ++i) s.prof[i] = 0;
  const uint64_t t_all = __builtin_amdgcn_s_memtime();
#endif
  for (uint32_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const strom_decomp_desc d = desc[b];
    const uint8_t *in = src + d.src_off;
    const uint32_t mis = (uint32_t)((uintptr_t)in & 15);
    s.ina = in - mis;
    s.out = dst + d.dst_off;
    s.iend = d.src_len + mis;
    s.ocap = d.dst_len;
    s.ip = mis;
    s.op = 0;
    s.bend = 0;
    s.win = 0xfffff000u;     // no window: in_window() fails for every p < 2^31
    s.flushed = 0;
    s.fenced = 0;
    s.omis = (uint32_t)((uintptr_t)s.out & 15);
    s.olen = 0;
    s.bcs = codec == STROM_CODEC_LZ4_FRAME_BCS;
    s.fhdr = codec == STROM_CODEC_ARROW_LZ4;
    s.mode = kHdr;
    s.err = 0;
    s.run<kSnap, kRes>(codec);
    if (s.lane == 0) status[b] = s.err ? s.err : (int32_t)s.op;
  }
#ifdef STROM_WAVE_PROF
  s.prof[kTTotal] = __builtin_amdgcn_s_memtime() - t_all;
  if (s.lane == 0)
    for (int i = 0; i < kWN; ++i) atomicAdd(&g_wprof[i], (unsigned long long)s.prof[i]);
#endif
}

}  // namespace

// Wave-per-stream decode (called by strom_decompress for few streams, or
// with STROM_DECOMP_G=64).
extern "C" int strom_decompress_wave(int codec, const void *d_src, void *d_dst,
                                     const strom_decomp_desc *d_desc, uint32_t nblocks,
                                     int32_t *d_status, void *stream) {
  if (codec < STROM_CODEC_LZ4 || codec > STROM_CODEC_ARROW_LZ4) return -22;
  if (!nblocks) return 0;
  const uint32_t grid = nblocks < 65535 ? nblocks : 65535;
  hipStream_t st = (hipStream_t)stream;
  const char *e = getenv("STROM_DECOMP_G");
  const bool res = e && atoi(e) == 65;     // resolve batches (LZ4 family)
  if (codec == STROM_CODEC_SNAPPY)
    hipLaunchKernelGGL((decompress_wave_kernel<true, false>), dim3(grid), dim3(64), 0, st, codec,
                       (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nblocks, d_status);
  else if (res)
    hipLaunchKernelGGL((decompress_wave_kernel<false, true>), dim3(grid), dim3(64), 0, st, codec,
                       (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nblocks, d_status);
  else
    hipLaunchKernelGGL((decompress_wave_kernel<false, false>), dim3(grid), dim3(64), 0, st, codec,
                       (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nblocks, d_status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

#ifdef STROM_WAVE_PROF
// read (and zero) the profile counters: out[kWN]
extern "C" int strom_wave_prof(uint64_t *out) {
  unsigned long long h[kWN] = {0};
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_wprof), sizeof h) != hipSuccess) return -5;
  unsigned long long z[kWN] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wprof), z, sizeof z);
  for (int i = 0; i < kWN; ++i) out[i] = h[i];
  return kWN;
}
#endif
