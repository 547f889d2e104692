// decompress.hip — LZ4 / snappy decode of HBM-resident buffers on CDNA4.
//
// North-star config 5 (BASELINE.json): compressed columnar files land in HBM
// through the engine and are decompressed on the GPU before the filter.  The
// reference has no decompressor; this is new MI355X-side work.
//
// Why lane groups.  LZ4/snappy parsing is serial within a stream.  A
// wave-per-stream decoder runs that parse on the scalar unit, and a CU has
// ONE scalar unit shared by all its waves: the previous version of this file
// measured ~130-160 CU-cycles per sequence (25-33 GB/s chip-wide) however
// many waves were resident.  Here a wave decodes G = 64/GL streams at once,
// one per group of GL lanes.  Every lane of a group runs the same parse on
// the same bytes (group-uniform values in VGPRs), so each VALU instruction
// advances G streams, and the copy work of a sequence is spread over the
// group's lanes, BPL consecutive bytes per lane per pass.
//
// Per stream (LDS, per group):
//   * an input window of kInW bytes ("P space": positions offset by the
//     stream's misalignment to 16 bytes).  The next window is prefetched
//     into VGPRs as soon as one is installed, so a sequential refill is LDS
//     stores only (VGPRs are free: LDS already limits residency to one wave
//     per SIMD);
//     token / length / offset bytes come from two dword reads + alignbyte;
//   * a history ring of kRing bytes.  Match bytes are read from the ring
//     with the period recurrence out[s+k] = out[s-off+(k mod off)], s = the
//     pass start, so a pass only reads bytes written before it began
//     (earlier passes' ds_writes precede its ds_reads in the wave's in-order
//     LDS stream).  Matches farther than kRing - W read the wave's own HBM
//     output instead (L1-bypassing loads after a fence; one fence covers all
//     output before it).
// The hot path waits on vmcnt only when it installs a prefetched window
// (on CDNA vmcnt also counts the wave's in-flight output stores).
//
// Codecs: raw LZ4 block, LZ4 frame block sequence (linked or independent
// blocks, optional per-block checksums skipped, stored blocks), a whole
// Arrow IPC compressed buffer (length prefix + frame header parsed on the
// device, so the host never reads the file), raw snappy, stored copy.  All positions are 32-bit (streams < 4 GiB).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "strom/strom.h"

namespace {

// Geometry, chosen per launch from the number of streams (strom_decompress):
//   GL  lanes per stream (G = 64 / GL streams per wave),
//   RING history ring and INW input window bytes per stream in LDS.
// Many streams: small groups, many streams per wave; few streams: whole
// waves per stream (wider copy passes, more waves resident per CU).
constexpr uint32_t BPL = 4;                  // bytes per lane per pass

// Optional cycle profile (-DSTROM_DECOMP_PROF, the libstrom_decprof.so
// build used by tools/decomp_prof.py): s_memtime spans per code path,
// summed by lane 0 of each group, plus event counts.
enum : int { kPSeq, kPLit, kPNear, kPShort, kPFar, kPRefill, kPFlush, kPHdr, kPFarFence,
             kPNSeq, kPNFar, kPNRefill, kPNFlush, kPNLitPass, kPNMatchPass, kPSteps,
             // wave-level (lane 0 only): loop iterations, cycles in the fast
             // step, cycles in the general step, cycles of whole iterations,
             // iterations in which some group took the general step
             kPWIter, kPWFast, kPWSlow, kPWLoop, kPWSlowIter, kPN };
#ifdef STROM_DECOMP_PROF
__device__ unsigned long long g_prof[kPN];
#define PROF_T0() const uint64_t _t0 = __builtin_amdgcn_s_memtime()
#define PROF_ADD(k) (prof[k] += __builtin_amdgcn_s_memtime() - _t0)
#define PROF_CNT(k, n) (prof[k] += (n))
#else
#define PROF_T0() (void)0
#define PROF_ADD(k) (void)0
#define PROF_CNT(k, n) (void)0
#endif

enum : int32_t { kErrFormat = -1, kErrOverflow = -2 };
enum : uint32_t { kHdr = 0, kLz4 = 1, kSnappy = 2, kDone = 3 };


// Group-uniform stream state (every lane of a group holds the same values).
template <uint32_t GL_, uint32_t RING_, uint32_t INW_>
struct Stream {
  static constexpr uint32_t GL = GL_;
  static constexpr uint32_t G = 64 / GL;     // streams per wave
  static constexpr uint32_t W = GL * BPL;    // bytes per pass per stream
  static constexpr uint32_t kRing = RING_;
  static constexpr uint32_t kMask = kRing - 1;
  static constexpr uint32_t kInW = INW_;
  static constexpr uint32_t kDummy = 16;     // sink for masked-off fast-path stores
  // far matches in the fast step: on for the few-stream geometries (config-5
  // frames 2x); with 16 streams per wave the extra predicate cost text -5 %
  static constexpr bool kFarFast = G <= 4;
  static constexpr uint32_t kSlot = kRing + kInW + kDummy;   // LDS bytes per stream
  // input prefetch: the next window, kPfN 16-byte loads per lane, starts
  // kSlide bytes past the current one (the overlap covers reads that
  // straddle the old window's end)
  static constexpr uint32_t kPfN = kInW / (16 * GL);
  static constexpr uint32_t kSlide = kInW - 64;
  // waves per SIMD the LDS footprint allows (160 KiB per CU, 4 SIMDs)
  static constexpr uint32_t kMinWaves = (160u * 1024 / (G * kSlot)) / 4 >= 4 ? 4 : 1;
  static_assert(64 % GL == 0 && (kRing & kMask) == 0, "geometry");
  static_assert(kRing >= 4 * W && kInW >= 4 * W && kInW % 4 == 0, "window sizes");
  static_assert(G * kSlot <= 64 * 1024, "LDS per wave");
  static_assert(kInW % (16 * GL) == 0 && kSlot % 16 == 0, "prefetch tiles");
  static_assert(kRing / 2 + 3 * W + 16 <= kRing, "flush pacing vs ring / far matches");

  const uint8_t *ina;  // 16-aligned input base (= stream start - mis)
  uint8_t *out;
  uint8_t *ring;       // this group's LDS history ring
  uint8_t *inw;        // this group's LDS input window
  uint32_t t;          // lane within the group
  uint32_t iend;       // input end (P space)
  uint32_t ocap;       // output capacity
  uint32_t ip;         // input position (P space)
  uint32_t op;         // output position
  uint32_t bend;       // end of the current LZ4 block (P space)
  uint32_t win;        // window base (P space, 4-aligned); ~0 = empty
  uint32_t vis;        // output below this is known complete in L2
  uint32_t flushed;    // output below this has been stored to HBM
  uint32_t omis;       // out & 15: ring index = (pos + omis) & kMask, so
                       // 16-B ring chunks are 16-B aligned in HBM too
  uint32_t olen;       // snappy: declared length
  uint32_t bcs;        // LZ4 frame blocks carry 4-byte checksums
  uint32_t fhdr;       // Arrow buffer: length prefix + frame header pending
  uint32_t mode;
  int32_t err;
  uint32_t pf_at;      // P-space start of the prefetched window; ~0 = none
  uint4 pf[kPfN];      // lane t: 16 bytes at pf_at + 16 (u GL + t)
#ifdef STROM_DECOMP_PROF
  uint64_t prof[kPN];
#endif

  // Window for [p, p + need).  Takes the prefetched next window when it
  // covers the range (the sequential case: its loads were issued one window
  // earlier, so no HBM latency here), else loads synchronously; then issues
  // the prefetch of the window after.  With the streams of a wave out of
  // step, each group's synchronous refill stalled all 16 (round 2 profile,
  // 61 distinct blocks: ~4.5k cycles per refill, ~30 % of the wave).
  __device__ void refill(uint32_t p, uint32_t need) {
    PROF_T0();
    PROF_CNT(kPNRefill, 1);
    if (pf_at != 0xffffffffu && p >= pf_at && p + need <= pf_at + kInW) {
#pragma unroll
      for (uint32_t u = 0; u < kPfN; ++u) *(uint4 *)(inw + 16 * (u * GL + t)) = pf[u];
      win = pf_at;
    } else {
      load_window(p);
    }
    const uint32_t nx = (win + kSlide) & ~15u;
    if (nx + kInW <= iend) {
#pragma unroll
      for (uint32_t u = 0; u < kPfN; ++u) pf[u] = *(const uint4 *)(ina + nx + 16 * (u * GL + t));
      pf_at = nx;
    } else {
      pf_at = 0xffffffffu;
    }
    PROF_ADD(kPRefill);
  }
  __device__ void load_window(uint32_t p) {
    const uint32_t at = p & ~3u;
    const uint32_t n = iend - at < kInW ? iend - at : kInW;
    const uint8_t *src = ina + at;
    uint32_t k = t * 4;
    // 8 independent dword loads in flight per lane, then their LDS writes
    for (; k + 7 * GL * 4 + 4 <= n; k += 8 * GL * 4) {
      uint32_t v[8];
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) v[u] = *(const uint32_t *)(src + k + u * GL * 4);
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) *(uint32_t *)(inw + k + u * GL * 4) = v[u];
    }
    for (; k + 4 <= n; k += GL * 4) *(uint32_t *)(inw + k) = *(const uint32_t *)(src + k);
    for (uint32_t kb = (n & ~3u) + t; kb < n; kb += GL) inw[kb] = src[kb];  // <= 3 tail bytes
    win = at;
  }
  // window holds [p, p + need) (bytes past iend are never used)
  __device__ __forceinline__ void ensure(uint32_t p, uint32_t need) {
    if (p < win || p + need > win + kInW) refill(p, need);
  }
  // bytes p..p+3 (little endian) and, in *b4, byte p+4
  __device__ __forceinline__ uint32_t rd4(uint32_t p, uint32_t *b4) {
    ensure(p, 8);
    const uint32_t o = p - win;
    const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
    const uint32_t d0 = d[0], d1 = d[1];
    const uint32_t sh = o & 3;
    if (b4) *b4 = (d1 >> (8 * sh)) & 0xff;
    return __builtin_amdgcn_alignbyte(d1, d0, sh);
  }
  __device__ __forceinline__ uint32_t rd1(uint32_t p) { return rd4(p, nullptr) & 0xff; }

  __device__ __forceinline__ void put(uint32_t pos, uint8_t v) { ring[(pos + omis) & kMask] = v; }
  // the first min(m, 4) bytes of v at pos..pos+3: one uniform test, then
  // unguarded byte stores for a full 4-byte span (no per-byte branch)
  __device__ __forceinline__ void put4(uint32_t pos, uint32_t v, uint32_t m) {
    const uint32_t a = pos + omis;
    if (m >= 4) {
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) ring[(a + j) & kMask] = (uint8_t)(v >> (8 * j));
    } else {
      for (uint32_t j = 0; j < m; ++j) ring[(a + j) & kMask] = (uint8_t)(v >> (8 * j));
    }
  }

  // Store ring bytes [flushed, upto) to HBM: whole 16-B chunks as one
  // dwordx4 store each (GL chunks per group instruction); partial chunks
  // (stream head/tail) byte by byte.  exact=false leaves a partial last
  // chunk for later.
  __device__ void flush(uint32_t upto, bool exact) {
    PROF_T0();
    PROF_CNT(kPNFlush, 1);
    const uint32_t rb = flushed + omis, re = upto + omis;
    const uint32_t cb = rb >> 4, ce = exact ? (re + 15) >> 4 : re >> 4;
    uint32_t c = cb + t;
    // whole chunks four at a time: the four LDS reads in flight together
    // instead of one read-then-store round trip per chunk
    const uint32_t cfull = re >> 4;
    for (; c + 3 * GL < cfull && (c << 4) >= rb; c += 4 * GL) {
      uint4 v[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) v[u] = *(const uint4 *)(ring + (((c + u * GL) << 4) & kMask));
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) *(uint4 *)(out + (((c + u * GL) << 4) - omis)) = v[u];
    }
    for (; c < ce; c += GL) {
      const uint32_t r0 = c << 4;
      const uint32_t lo = r0 < rb ? rb : r0, hi = r0 + 16 > re ? re : r0 + 16;
      const uint4 v = *(const uint4 *)(ring + (r0 & kMask));
      if (lo == r0 && hi == r0 + 16) {
        *(uint4 *)(out + (r0 - omis)) = v;
      } else {
        for (uint32_t x = lo; x < hi; ++x) {
          const uint32_t i = x - r0;
          const uint32_t w = i < 8 ? (i < 4 ? v.x : v.y) : (i < 12 ? v.z : v.w);
          out[x - omis] = (uint8_t)(w >> (8 * (i & 3)));
        }
      }
    }
    const uint32_t nf = exact ? upto : (ce << 4) - omis;
    if (ce > cb && nf > flushed) flushed = nf;
    PROF_ADD(kPFlush);
  }
  // bound the unflushed span so the ring never overwrites it (and far
  // matches only read flushed output): called after every pass
  __device__ __forceinline__ void pace(uint32_t cur) {
    if (cur - flushed >= kRing / 2) flush(cur, false);
  }

  // literal bytes [p, p+len) of the input -> output
  __device__ void literal(uint32_t p, uint32_t len) {
    PROF_T0();
    PROF_CNT(kPNLitPass, (len + W - 1) / W);
    const uint32_t k = t * BPL;
    for (uint32_t done = 0; done < len; done += W) {
      const uint32_t n = len - done < W ? len - done : W;
      ensure(p + done, W + 8);
      if (k < n) {
        const uint32_t o = p + done + k - win;
        const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
        const uint32_t v = __builtin_amdgcn_alignbyte(d[1], d[0], o & 3);
        put4(op + done + k, v, n - k);
      }
      pace(op + done + n);
    }
    op += len;
    PROF_ADD(kPLit);
  }

  __device__ void match(uint32_t off, uint32_t len) {
    PROF_T0();
    PROF_CNT(kPNMatchPass, (len + W - 1) / W);
    if (off == 0 || off > op) {
      err = kErrFormat;
      return;
    }
    const uint32_t k = t * BPL;
    if (off <= kRing - W) {
      if (off >= W) {
        // sources [s-off, s-off+W) lie before the pass: one unaligned
        // 4-byte read per lane (two dwords, ring-wrapped separately)
        for (uint32_t done = 0; done < len; done += W) {
          const uint32_t n = len - done < W ? len - done : W;
          if (k < n) {
            const uint32_t s = op + done + k;
            const uint32_t q = s - off + omis;
            const uint32_t a0 = q & kMask & ~3u;
            const uint32_t d0 = *(const uint32_t *)(ring + a0);
            const uint32_t d1 = *(const uint32_t *)(ring + ((a0 + 4) & kMask));
            const uint32_t v = __builtin_amdgcn_alignbyte(d1, d0, q & 3);
            put4(s, v, n - k);
          }
          pace(op + done + n);
        }
        PROF_ADD(kPNear);
      } else {
        // short period: byte k of a pass starting at s repeats s-off+(k mod off)
        uint32_t r[BPL];
        // k % off for k < 256, off < W: one float reciprocal instead of the
        // ~30-instruction integer remainder (exact: the quotient error of
        // the rcp is far below 1/256, corrected by one compare)
        {
          uint32_t q = (uint32_t)((float)k * __builtin_amdgcn_rcpf((float)off));
          uint32_t rem = k - q * off;
          if ((int32_t)rem < 0) rem += off;
          else if (rem >= off) rem -= off;
          r[0] = rem;
        }
#pragma unroll
        for (uint32_t j = 1; j < BPL; ++j) {
          r[j] = r[j - 1] + 1;
          if (r[j] >= off) r[j] = 0;
        }
        for (uint32_t done = 0; done < len; done += W) {
          const uint32_t n = len - done < W ? len - done : W;
          const uint32_t s = op + done;
          uint8_t v[BPL];
#pragma unroll
          for (uint32_t j = 0; j < BPL; ++j) v[j] = ring[(s - off + r[j] + omis) & kMask];
#pragma unroll
          for (uint32_t j = 0; j < BPL; ++j)
            if (k + j < n) put(s + k + j, v[j]);
          pace(s + n);
        }
        PROF_ADD(kPShort);
      }
    } else {
      PROF_CNT(kPNFar, 1);
      // far (off > kRing - W >= 3W): sources are this wave's stored output
      for (uint32_t done = 0; done < len; done += W) {
        const uint32_t n = len - done < W ? len - done : W;
        const uint32_t s = op + done;
        if (s - off + n > vis) {
          // pace() keeps these sources flushed already; stay safe anyway
          PROF_T0();
          if (s - off + n > flushed) flush(s, true);
          // our stores complete at L2 before the L1-bypassing loads below.
          // Workgroup scope = s_waitcnt vmcnt(0): the reader is this wave,
          // whose traffic all goes to its own XCD's L2, so no L2 write-back
          // (the agent-scope form adds buffer_wbl2: ~4.9k cycles per far
          // match on the config-5 column, where 24 % of matches are far)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          vis = flushed;
          PROF_ADD(kPFarFence);
        }
        if (k < n) {
          // two L1-bypassing dword loads + alignbyte per lane (the second
          // dword ends below s: off > 3W)
          const uintptr_t q = (uintptr_t)(out + s + k - off);
          const uint32_t *w = (const uint32_t *)(q & ~(uintptr_t)3);
          const uint32_t d0 = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint32_t d1 = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint32_t v = __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)(q & 3));
#pragma unroll
          for (uint32_t j = 0; j < BPL; ++j)
            if (k + j < n) put(s + k + j, (uint8_t)(v >> (8 * j)));
        }
        pace(s + n);
      }
      PROF_ADD(kPFar);
    }
    op += len;
  }

  // window bytes p..p+3 without the window check (caller guarantees it)
  __device__ __forceinline__ uint32_t rd4u(uint32_t p) const {
    const uint32_t o = p - win;
    const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
    return __builtin_amdgcn_alignbyte(d[1], d[0], o & 3);
  }

  // ---- the common LZ4 sequence in one straight-line pass: short literal
  // run and short near match (lit < 15, match < 19 without a length
  // extension and <= W bytes, 1 <= off <=
  // kRing - W), input window and output ring already in place.  Every lane
  // stores its 4 literal and 4 match bytes unconditionally — bytes past the
  // run go to a per-stream sink — so the step has no per-byte branches and
  // no loops; the round 2 cycle profile put ~2k cycles per sequence in the
  // general path, most of it control flow.  false: take the general path
  // (nothing was changed).
  // lane t stores literal bytes k..k+3 of [src, src + lit) at op (bytes
  // past the run go to the sink)
  __device__ __forceinline__ void fast_lit(uint32_t src, uint32_t lit) {
    uint8_t *sink = inw + kInW;
    const uint32_t k = t * BPL;
    const uint32_t v = rd4u(src + k);
#pragma unroll
    for (uint32_t j = 0; j < BPL; ++j) {
      uint8_t *d = k + j < lit ? ring + ((op + k + j + omis) & kMask) : sink + j;
      *d = (uint8_t)(v >> (8 * j));
    }
  }

  // match at s, mlen <= 2W: byte i of the copy is out[s - off + (i mod off)].
  // Relative to any pass start sp the same holds with sp for s (the output
  // from s - off on is periodic), so both passes use the same residues;
  // the second runs only for groups whose match needs it.
  // far (off > kRing - W, sources below vis: stored and fenced) reads the
  // wave's HBM output instead of the ring: off > 2W >= mlen, so the 4 bytes
  // of a lane are consecutive (two L1-bypassing dword loads + alignbyte)
  __device__ __forceinline__ void fast_copy(uint32_t s, uint32_t off, uint32_t mlen, bool far) {
    uint8_t *sink = inw + kInW;
    const uint32_t k = t * BPL;
    if (far) {
#pragma unroll
      for (uint32_t c = 0; c < 2 * W; c += W) {
        if (c && mlen <= W) break;
        const uintptr_t q = (uintptr_t)(out + s - off + c + k);
        const uint32_t *w = (const uint32_t *)(q & ~(uintptr_t)3);
        const uint32_t d0 = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t d1 = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t v = __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)(q & 3));
#pragma unroll
        for (uint32_t j = 0; j < BPL; ++j) {
          uint8_t *d = c + k + j < mlen ? ring + ((s + c + k + j + omis) & kMask) : sink + 4 + j;
          *d = (uint8_t)(v >> (8 * j));
        }
      }
      return;
    }
    const uint32_t base = s - off + omis;
    uint32_t q = (uint32_t)((float)k * __builtin_amdgcn_rcpf((float)off));
    uint32_t r = k - q * off;
    if ((int32_t)r < 0) r += off;
    else if (r >= off) r -= off;
    uint32_t rr[BPL];
#pragma unroll
    for (uint32_t j = 0; j < BPL; ++j) {
      rr[j] = r;
      r = r + 1 == off ? 0 : r + 1;
    }
#pragma unroll
    for (uint32_t c = 0; c < 2 * W; c += W) {
      if (c && mlen <= W) break;
      uint8_t v[BPL];
#pragma unroll
      for (uint32_t j = 0; j < BPL; ++j) v[j] = ring[(base + c + rr[j]) & kMask];
#pragma unroll
      for (uint32_t j = 0; j < BPL; ++j) {
        uint8_t *d = c + k + j < mlen ? ring + ((s + c + k + j + omis) & kMask) : sink + 4 + j;
        *d = v[j];
      }
    }
  }

  // the fast step's only obstacle is the end of the loaded input window
  __device__ __forceinline__ bool window_short(bool snap) const {
    const uint32_t end = snap ? iend : bend;
    return mode == (snap ? kSnappy : kLz4) && win != 0xffffffffu && ip >= win &&
           ip + 24 > win + kInW && ip + 24 <= end;
  }

  __device__ __forceinline__ bool fast_window(uint32_t end) const {
    return win != 0xffffffffu && ip >= win && ip + 24 <= win + kInW && ip + 24 <= end;
  }

  // en: the group is live in LZ4 mode.  Every test is folded into one
  // predicate (bitwise, no short circuit) behind one branch: each early
  // return used to be a v_cmp -> s_and_saveexec -> s_cbranch chain waiting
  // on the compare (round 2 stamps: ~1,150 cycles per step for ~150
  // instructions).  Reads before the test use a clamped window offset, so
  // they stay inside this stream's LDS slot whatever the state.
  __device__ __forceinline__ bool lz4_fast(bool en) {
    bool ok = en & (win != 0xffffffffu) & (ip >= win) & (ip + 24 <= win + kInW) & (ip + 24 <= bend);
    const uint32_t o = ok ? ip - win : 0u;
    const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
    const uint32_t w = __builtin_amdgcn_alignbyte(d[1], d[0], o & 3);
    const uint32_t lit = (w >> 4) & 15, ml = w & 15;
    const uint32_t oo = o + 1 + lit;
    const uint32_t *e = (const uint32_t *)(inw + (oo & ~3u));
    const uint32_t ox = __builtin_amdgcn_alignbyte(e[1], e[0], oo & 3);
    const uint32_t off = ox & 0xffff, xb = (ox >> 16) & 0xff;   // xb: length extension byte
    const uint32_t mlen = ml == 15 ? 19 + xb : ml + 4;
    // this lane's 4 literal bytes, read with the offset (same round trip)
    const uint32_t ol = o + 1 + t * BPL;
    const uint32_t *f = (const uint32_t *)(inw + (ol & ~3u));
    const uint32_t lv = __builtin_amdgcn_alignbyte(f[1], f[0], ol & 3);
    // a far match (past the ring) stays in the fast step when its source
    // lies below vis (already stored and fenced: read back from HBM)
    const bool far = off > kRing - W;
    ok = ok & (lit != 15) & ((ml != 15) | (xb != 255)) & (mlen <= 2 * W) & (off != 0) &
         (off <= op + lit) & (!far | (kFarFast & (op + lit + mlen <= vis + off))) &
         (lit + mlen <= ocap - op);
    if (!ok) return false;
    {
      uint8_t *sink = inw + kInW;
      const uint32_t k = t * BPL;
#pragma unroll
      for (uint32_t j = 0; j < BPL; ++j) {
        uint8_t *dd = k + j < lit ? ring + ((op + k + j + omis) & kMask) : sink + j;
        *dd = (uint8_t)(lv >> (8 * j));
      }
    }
    fast_copy(op + lit, off, mlen, kFarFast && far);
    ip += 3 + lit + (ml == 15);
    op += lit + mlen;
    return true;                 // flush pacing: the kernel loop's exception test
  }

  // the same for one snappy element: a literal with its length in the tag
  // or a copy with a 1- or 2-byte offset, <= W bytes either way.  Both
  // halves always run (a literal is a copy of length 0 and a copy a
  // literal of length 0, their stores going to the sink), so groups on
  // different element kinds do not diverge.
  __device__ __forceinline__ bool snappy_fast(bool en) {
    bool ok = en & (win != 0xffffffffu) & (ip >= win) & (ip + 24 <= win + kInW) & (ip + 24 <= iend);
    const uint32_t o = ok ? ip - win : 0u;
    const uint32_t *d = (const uint32_t *)(inw + (o & ~3u));
    const uint32_t w = __builtin_amdgcn_alignbyte(d[1], d[0], o & 3);
    const uint32_t ol = o + 1 + t * BPL;
    const uint32_t *f = (const uint32_t *)(inw + (ol & ~3u));
    const uint32_t lv = __builtin_amdgcn_alignbyte(f[1], f[0], ol & 3);
    const uint32_t tag = w & 0xff, kind = tag & 3;
    const bool islit = kind == 0;
    const uint32_t len = kind == 1 ? 4 + ((tag >> 2) & 7) : (tag >> 2) + 1;
    const uint32_t coff = kind == 1 ? ((tag >> 5) << 8) | ((w >> 8) & 0xff) : (w >> 8) & 0xffff;
    const uint32_t lit = islit ? len : 0u, mlen = islit ? 0u : len, off = islit ? 1u : coff;
    // literal tag lengths 61..64 announce length bytes; a literal longer
    // than the 24 guaranteed bytes (wide groups) must lie in the window
    ok = ok & (kind != 3) & (len <= W) & (len <= olen - op) &
         (islit ? (len <= 60) & (ip + 1 + len <= win + kInW) & (ip + 1 + len <= iend)
                : (off != 0) & (off <= op) & (off <= kRing - W));
    if (!ok) return false;
    {
      uint8_t *sink = inw + kInW;
      const uint32_t k = t * BPL;
#pragma unroll
      for (uint32_t j = 0; j < BPL; ++j) {
        uint8_t *dd = k + j < lit ? ring + ((op + k + j + omis) & kMask) : sink + j;
        *dd = (uint8_t)(lv >> (8 * j));
      }
    }
    fast_copy(op, off, mlen, false);
    ip += islit ? 1 + len : 1 + kind;
    op += len;
    return true;
  }

  // ---- one LZ4 sequence of the block ending at bend
  __device__ void lz4_seq() {
    PROF_T0();
    PROF_CNT(kPNSeq, 1);
    const uint32_t w = rd4(ip, nullptr);
    uint32_t lit = (w >> 4) & 15, ml = w & 15;
    uint32_t p = ip + 1;
    if (lit == 15) {
      uint32_t b;
      do {
        if (p >= bend) { err = kErrFormat; return; }
        b = rd1(p++);
        lit += b;
      } while (b == 255);
    }
    if (lit > bend - p) { err = kErrFormat; return; }
    if (lit > ocap - op) { err = kErrOverflow; return; }
    if (lit) literal(p, lit);
    p += lit;
    if (p >= bend) { ip = p; return; }  // last sequence: literals only
    if (bend - p < 2) { err = kErrFormat; return; }
    // with no literals the offset bytes came with the token
    const uint32_t off = (lit == 0 ? (w >> 8) : rd4(p, nullptr)) & 0xffff;
    p += 2;
    if (ml == 15) {
      uint32_t b;
      do {
        if (p >= bend) { err = kErrFormat; return; }
        b = rd1(p++);
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (ml > ocap - op) { err = kErrOverflow; return; }
    match(off, ml);
    ip = p;
    PROF_ADD(kPSeq);
  }

  // ---- one snappy element (literal run or copy)
  __device__ void snappy_tag() {
    uint32_t b4;
    const uint32_t w = rd4(ip, &b4);
    const uint32_t tag = w & 0xff, kind = tag & 3;
    uint32_t p = ip + 1, len, off;
    if (kind == 0) {
      len = (tag >> 2) + 1;
      if (len > 60) {
        const uint32_t nb = len - 60;  // 1..4 length bytes
        if (iend - p < nb) { err = kErrFormat; return; }
        const uint32_t x = nb == 4 ? ((w >> 8) | (b4 << 24)) : (w >> 8) & ((1u << (8 * nb)) - 1);
        len = x + 1;
        if (len == 0) { err = kErrFormat; return; }
        p += nb;
      }
      if (len > iend - p || len > olen - op) { err = kErrFormat; return; }
      literal(p, len);
      ip = p + len;
      return;
    }
    if (kind == 1) {
      if (iend - p < 1) { err = kErrFormat; return; }
      len = 4 + ((tag >> 2) & 7);
      off = ((tag >> 5) << 8) | ((w >> 8) & 0xff);
      p += 1;
    } else if (kind == 2) {
      if (iend - p < 2) { err = kErrFormat; return; }
      len = (tag >> 2) + 1;
      off = (w >> 8) & 0xffff;
      p += 2;
    } else {
      if (iend - p < 4) { err = kErrFormat; return; }
      len = (tag >> 2) + 1;
      off = (w >> 8) | (b4 << 24);
      p += 4;
    }
    if (len > olen - op) { err = kErrFormat; return; }
    match(off, len);
    ip = p;
  }

  // ---- stream-level headers: frame block header, snappy preamble, copy
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
        const uint32_t b = rd1(p++);
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
      literal(ip, n);
      ip = iend;
      mode = kDone;
    } else if (fhdr) {
      // Arrow IPC compressed buffer (BodyCompression LZ4_FRAME): int64
      // uncompressed length (-1: the rest is stored raw), then one LZ4 frame
      fhdr = 0;
      if (iend - ip < 8) { err = kErrFormat; return; }
      const uint32_t lo = rd4(ip, nullptr), hi = rd4(ip + 4, nullptr);
      ip += 8;
      if (lo == 0xffffffffu && hi == 0xffffffffu) {
        const uint32_t n = iend - ip;
        if (n > ocap) { err = kErrOverflow; return; }
        literal(ip, n);
        ip = iend;
        mode = kDone;
        return;
      }
      if (hi != 0 || lo > ocap) { err = kErrOverflow; return; }
      if (iend - ip < 7 || rd4(ip, nullptr) != 0x184D2204u) { err = kErrFormat; return; }
      const uint32_t flg = rd1(ip + 4);
      if ((flg >> 6) != 1) { err = kErrFormat; return; }
      const uint32_t hl = 7 + ((flg & 0x08) ? 8 : 0) + ((flg & 0x01) ? 4 : 0);
      if (iend - ip < hl) { err = kErrFormat; return; }
      bcs = (flg & 0x10) ? 1 : 0;
      ip += hl;
    } else {
      // LZ4 frame data blocks: [u32 size|stored flag][data][u32 bcs?]... [u32 0]
      if (iend - ip < 4) { err = kErrFormat; return; }
      uint32_t bs = rd4(ip, nullptr);
      ip += 4;
      if (bs == 0) { mode = kDone; return; }
      const bool stored = bs & 0x80000000u;
      bs &= 0x7fffffffu;
      if (bs > iend - ip) { err = kErrFormat; return; }
      if (stored) {
        if (bs > ocap - op) { err = kErrOverflow; return; }
        literal(ip, bs);
        ip += bs;
        if (bcs) ip += 4;
      } else {
        bend = ip + bs;
        mode = kLz4;
      }
    }
  }

  // one unit of work; false once the stream is finished (or failed)
  template <bool kSnap>
  __device__ bool step(int codec) {
    if (mode == kHdr) {
      header<kSnap>(codec);
    } else if (!kSnap && mode == kLz4) {
      if (ip >= bend) {
        if (codec == STROM_CODEC_LZ4) {
          mode = kDone;
        } else {
          ip = bend + (bcs ? 4 : 0);
          mode = kHdr;
        }
      } else {
        lz4_seq();
      }
    } else if (kSnap && mode == kSnappy) {
      if (ip >= iend) {
        if (op != olen) err = kErrFormat;
        mode = kDone;
      } else {
        snappy_tag();
      }
    }
    return !err && mode != kDone;
  }
};

// 64 threads, >= 4 waves per SIMD (<= 128 VGPRs): the decoder is latency
// bound per wave (round 2 trace: 256 or 1024 waves took the same ~9 ms),
// so throughput comes from waves resident per CU
// kSnap: the snappy kernel, else the LZ4 family (raw, frame, Arrow) — one
// fast step per kernel keeps the register budget of the 4-wave launch bound
template <class S, bool kSnap>
__global__ __launch_bounds__(64, S::kMinWaves) void decompress_kernel(int codec, const uint8_t *__restrict__ src,
                                                        uint8_t *__restrict__ dst,
                                                        const strom_decomp_desc *__restrict__ desc,
                                                        uint32_t nblocks, int32_t *status) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[S::G * S::kSlot];
  const uint32_t lane = threadIdx.x, g = lane / S::GL;
  const uint32_t stride = gridDim.x * S::G;
  S st;
#ifdef STROM_DECOMP_PROF
  for (int i = 0; i < kPN; ++i) st.prof[i] = 0;
#endif
  st.t = lane % S::GL;
  st.ring = lds + g * S::kSlot;
  st.inw = st.ring + S::kRing;
  uint32_t b = blockIdx.x * S::G + g;
  bool live = false;
  for (;;) {
#ifdef STROM_DECOMP_PROF
    if (live) st.prof[kPSteps] += 1;
    const uint64_t _w0 = __builtin_amdgcn_s_memtime();
#endif
    // The common short sequence goes through the straight-line step.  One
    // rare, wave-uniform branch covers everything else: the general step
    // (long runs, far matches, block/frame edges, errors), flush pacing,
    // finishing a stream and taking the next one — every extra branch in
    // the common path cost a compare-to-branch round trip per step.
    bool fast;
    if constexpr (kSnap) fast = st.snappy_fast(live & (st.mode == kSnappy));
    else fast = st.lz4_fast(live & (st.mode == kLz4));
    const bool exc = !fast | (st.op - st.flushed >= S::kRing / 2);
#ifdef STROM_DECOMP_PROF
    const uint64_t _w1 = __builtin_amdgcn_s_memtime();
    const bool _slow = __any(live && !fast);
#endif
    if (__builtin_expect(__any(exc), 0)) {
      if (fast) {
        st.pace(st.op);
      } else if (live && st.window_short(kSnap)) {
        // only the input window ran short: slide it now rather than send
        // the next few sequences through the general step one by one
        st.refill(st.ip, 24);
      } else if (live && !st.template step<kSnap>(codec)) {
        if (!st.err) st.flush(st.op, true);
        if (st.t == 0) status[b] = st.err ? st.err : (int32_t)st.op;
        live = false;
        b += stride;
      }
      if (!live && b < nblocks) {
        const strom_decomp_desc d = desc[b];
        const uint8_t *in = src + d.src_off;
        const uint32_t mis = (uint32_t)((uintptr_t)in & 15);
        st.ina = in - mis;
        st.out = dst + d.dst_off;
        st.iend = d.src_len + mis;
        st.ocap = d.dst_len;
        st.ip = mis;
        st.op = 0;
        st.bend = 0;
        st.win = 0xffffffffu;
        st.pf_at = 0xffffffffu;
        st.vis = 0;
        st.flushed = 0;
        st.omis = (uint32_t)((uintptr_t)st.out & 15);
        st.olen = 0;
        st.bcs = codec == STROM_CODEC_LZ4_FRAME_BCS;
        st.fhdr = codec == STROM_CODEC_ARROW_LZ4;
        st.mode = kHdr;
        st.err = 0;
        live = true;
      }
      if (!__any(live)) break;
    }
#ifdef STROM_DECOMP_PROF
    const uint64_t _w2 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
      st.prof[kPWIter] += 1;
      st.prof[kPWFast] += _w1 - _w0;
      st.prof[kPWSlow] += _w2 - _w1;
      st.prof[kPWLoop] += _w2 - _w0;
      st.prof[kPWSlowIter] += _slow ? 1 : 0;
    }
#endif
  }
#ifdef STROM_DECOMP_PROF
  if (st.t == 0)
    for (int i = 0; i < kPN; ++i) atomicAdd(&g_prof[i], (unsigned long long)st.prof[i]);
#endif
}

// 16 x 2496 B = 39 KiB (+ the runtime's 512 B) lets 4 waves share a CU's
// 160 KiB: at 40.5 KiB only 3 fit (round 2 trace: LDS_Block_Size 41472)
using S16 = Stream<4, 2048, 448>;     // 16 streams per wave
// A/B variant: half the LDS (2 waves per SIMD), a 1 KiB history ring
using S16s = Stream<4, 1024, 256>;    // 16 streams per wave, 19.5 KiB
using S8 = Stream<8, 2048, 512>;      // 8 streams per wave, 19.5 KiB (2 waves per SIMD)
using S4 = Stream<16, 2048, 512>;     // 4 streams per wave, 10 KiB
using S1 = Stream<64, 2048, 1024>;    // 1 stream per wave, 3 KiB
// few streams (<= 2,048: a launch leaves most SIMDs idle anyway): large
// history rings, so far matches (sources past the ring, read back from HBM)
// stay rare — on the config-5 column 24 % of LZ4 matches reach past 2 KiB,
// 5 % past 16 KiB
using S2L = Stream<32, 16384, 512>;   // 2 streams per wave, 33 KiB
using S4L = Stream<16, 8192, 512>;    // 4 streams per wave, 35 KiB
using S1L = Stream<64, 16384, 1024>;  // 1 stream per wave, 17 KiB (2 waves per SIMD)

template <class S>
int launch(int codec, const void *d_src, void *d_dst, const strom_decomp_desc *d_desc,
           uint32_t nblocks, int32_t *d_status, hipStream_t st) {
  const uint32_t waves = (nblocks + S::G - 1) / S::G;
  const uint32_t grid = waves < 16384 ? waves : 16384;
  if (codec == STROM_CODEC_SNAPPY)
    hipLaunchKernelGGL((decompress_kernel<S, true>), dim3(grid), dim3(64), 0, st, codec,
                       (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nblocks, d_status);
  else
    hipLaunchKernelGGL((decompress_kernel<S, false>), dim3(grid), dim3(64), 0, st, codec,
                       (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nblocks, d_status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace

// lz4par.hip: one workgroup per stream, parallel parse + pointer doubling
extern "C" int strom_decompress_par(int codec, const void *d_src, void *d_dst,
                                    const strom_decomp_desc *d_desc, uint32_t nstreams,
                                    int32_t *d_status, void *stream);

extern "C" int strom_decompress_par512(int codec, const void *d_src, void *d_dst,
                                       const strom_decomp_desc *d_desc, uint32_t nstreams,
                                       int32_t *d_status, void *stream);

extern "C" int strom_decompress_par512b(int codec, const void *d_src, void *d_dst,
                                        const strom_decomp_desc *d_desc, uint32_t nstreams,
                                        int32_t *d_status, void *stream);

extern "C" int strom_decompress_lanes(int codec, const void *d_src, void *d_dst,
                                      const strom_decomp_desc *d_desc, uint32_t nblocks,
                                      int32_t *d_status, void *stream);

// CUs of the current device (resident-workgroup arithmetic of the dispatch)
static uint32_t device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    return 256;
  return (uint32_t)n;
}

// Streams per wave by stream count: keep >= ~8 waves per CU (256 CUs)
// when there are enough streams, else give each stream more lanes.
// STROM_DECOMP_G (1, 4, 8, 16; 32 = 16 with the small ring; 3 / 2 / 6 = 1 /
// 2 / 4 streams per wave with 16 / 16 / 8 KiB rings)
// forces a geometry (A/B runs).
extern "C" int strom_decompress(int codec, const void *d_src, void *d_dst,
                                const strom_decomp_desc *d_desc, uint32_t nblocks,
                                int32_t *d_status, void *stream) {
  if (codec == STROM_CODEC_ZSTD || codec == STROM_CODEC_ARROW_ZSTD)
    return strom_decompress_zstd(codec, d_src, d_dst, d_desc, nblocks, d_status, nullptr, 0,
                                 stream);
  if (codec < STROM_CODEC_LZ4 || codec > STROM_CODEC_ARROW_LZ4) return -22;
  if (!nblocks) return 0;
  // Up to 8,192 LZ4 streams: the block-parallel decoder (lz4par.hip) — a
  // stream is decoded by a whole workgroup, so a launch no longer takes one
  // serial stream's time (profiles/r3/dec/lz4par_threshold.json, 512 KiB
  // frames, par vs lanes GB/s: 4,096 val 115/48, ids 104/58, text 56/54;
  // 8,192 val 116/66, ids 106/83, text 56/78).  From 16k streams the lane
  // groups win on near-match data (ids 194/108, text 170/57; val, a quarter
  // of its matches past 2 KiB, stays 118/52).  Streams that fit in one
  // round of the 512-thread build's resident workgroups (3 per CU) take it:
  // shorter per-stream chains (lz4par_nt512.hip; config-5 frames 512: 61 ->
  // 85 GB/s, 768: 86 -> 115; profiles/r3/dec/lz4par_nt_occupancy_ab.json).
  // STROM_DECOMP_PAR=0 forces the lane groups, 1 the block-parallel choice,
  // 256 / 512 / 8192 a build (8192: 512 threads, 8 KiB batches).
  const char *pe = getenv("STROM_DECOMP_PAR");
  const int pv = pe ? atoi(pe) : -1;
  // snappy takes the same block-parallel decoder (its element grammar, round 4)
  const bool par_codec = codec != STROM_CODEC_COPY;
  if (par_codec && (pe ? pv != 0 : nblocks <= 8192)) {
    // up to two streams per CU: the 8 KiB-batch build (lz4par_nt512_ob8k.hip)
    const uint32_t cus = device_cus();
    const bool pick = pv != 256 && pv != 512 && pv != 8192;   // the library's choice
    if (pv == 8192 || (pick && nblocks <= 2 * cus))
      return strom_decompress_par512b(codec, d_src, d_dst, d_desc, nblocks, d_status, stream);
    // snappy takes the 512-thread build at every larger count (its walkers,
    // r4: 2,048 / 8,192 streams text 85 -> 94 / 88 -> 101, val 76 -> 84 /
    // 79 -> 91, ids 78 -> 85 / 81 -> 91 GB/s, profiles/r4/dec/snappy_final.json)
    // LZ4 from 12 streams per CU too: text / ids / val at 3,072 streams 116 /
    // 111 / 110 against 99 / 102 / 110 GB/s (8,192: 120 / 115 / 113 against
    // 102 / 105 / 112; profiles/r4/dec/lz4par_many_streams.json); between
    // 3 and 12 per CU the 256-thread build keeps val (2,048: 110 vs 104).
    // Literal-heavy streams (utf8 characters) lose on it (8,192: 74 vs 110)
    // and go to the lane decoder from decompress() and the Arrow scan.
    if (pv == 512 ||
        (pick && (codec == STROM_CODEC_SNAPPY || nblocks <= 3 * cus || nblocks >= 12 * cus)))
      return strom_decompress_par512(codec, d_src, d_dst, d_desc, nblocks, d_status, stream);
    return strom_decompress_par(codec, d_src, d_dst, d_desc, nblocks, d_status, stream);
  }
  return strom_decompress_lanes(codec, d_src, d_dst, d_desc, nblocks, d_status, stream);
}

// the lane-group decoders only (A/B runs: tools/lz4par_bench.py)
extern "C" int strom_decompress_lanes(int codec, const void *d_src, void *d_dst,
                                      const strom_decomp_desc *d_desc, uint32_t nblocks,
                                      int32_t *d_status, void *stream) {
  if (codec < STROM_CODEC_LZ4 || codec > STROM_CODEC_ARROW_LZ4) return -22;
  if (!nblocks) return 0;
  const char *e = getenv("STROM_DECOMP_G");
  uint32_t g = e ? (uint32_t)atoi(e) : 0u;
  // Default geometry by stream count (round 2 same-box A/B over 61 distinct
  // blocks + config-5 frames, profiles/r2/dec/geometry_ab.json): few
  // streams leave SIMDs idle whatever the geometry, so they get fewer
  // streams per wave and larger history rings (far matches — HBM reads —
  // stay rare); from ~16k streams 16 per wave wins (VALU per stream).
  //   <= 1,024: 1 per wave, 16 KiB ring (every SIMD busy: +7-12 % over 2/wave)
  //   <= 2,048: 2 per wave, 16 KiB rings (config-5 frames 14.6 -> 27.5 GB/s)
  //   <= 4,096: 4 per wave, 8 KiB rings;  <= 8,192: 4 per wave, 2 KiB rings
  if (!e)
    g = nblocks <= 1024 ? 3 : nblocks <= 2048 ? 2 : nblocks <= 4096 ? 6 : nblocks <= 8192 ? 4 : 16;
  if (g != 1 && g != 2 && g != 3 && g != 4 && g != 6 && g != 8 && g != 16 && g != 32) g = 16;
  hipStream_t st = (hipStream_t)stream;
  if (g == 2) return launch<S2L>(codec, d_src, d_dst, d_desc, nblocks, d_status, st);
  if (g == 6) return launch<S4L>(codec, d_src, d_dst, d_desc, nblocks, d_status, st);
  if (g == 3) return launch<S1L>(codec, d_src, d_dst, d_desc, nblocks, d_status, st);
  if (g == 16) return launch<S16>(codec, d_src, d_dst, d_desc, nblocks, d_status, st);
  if (g == 32) return launch<S16s>(codec, d_src, d_dst, d_desc, nblocks, d_status, st);
  if (g == 8) return launch<S8>(codec, d_src, d_dst, d_desc, nblocks, d_status, st);
  if (g == 4) return launch<S4>(codec, d_src, d_dst, d_desc, nblocks, d_status, st);
  return launch<S1>(codec, d_src, d_dst, d_desc, nblocks, d_status, st);
}

#ifdef STROM_DECOMP_PROF
// read (and zero) the profile counters: out[kPN]
extern "C" int strom_decomp_prof(uint64_t *out) {
  unsigned long long h[kPN] = {0};
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_prof), sizeof h) != hipSuccess) return -5;
  unsigned long long z[kPN] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z);
  for (int i = 0; i < kPN; ++i) out[i] = h[i];
  return kPN;
}
#endif
