// lz4par.hip — LZ4 decode with parallelism INSIDE a stream, for few long
// streams (BASELINE config 5: pyarrow writes each 512 KiB column buffer as
// one LZ4 frame of linked 64 KiB blocks, so a 134M-row column is only 2,048
// streams and decompress.hip — one stream per lane group, parse serial —
// leaves most of the chip idle: 27.5 GB/s, profiles/r2/dec/SUMMARY.md).
//
// One workgroup of NT threads per stream.  The compressed input is taken in
// windows of PW bytes that start on a known token:
//
//  1. speculative parse: thread t follows the token chain from the start of
//     its SL-byte slice, marking token starts in an LDS bitmap, up to its
//     exit (first token at or past the slice end).  Chains from wrong
//     starts merge into the true chain within a few tokens.
//  2. validation: slice t is right when its true entry (slice t-1's exit)
//     is one of its marked tokens; the few that are not re-parse from the
//     true entry, in rounds, until nothing changes (correct for any input,
//     fast when chains merge — the usual case).
//  3. every thread walks its true sequences: output bytes -> block scan ->
//     each slice's output start.
//  4. output in batches of OB bytes: a source pointer per output byte
//     (literal byte: its input position; match byte: the byte `off` back —
//     "history" when that lies before the batch, already stored), then
//     pointer doubling p = ptr[p] until every pointer is a literal or
//     history root (chain depth d resolves in log2 d rounds; the r2 replay,
//     tools/lz4_pointer_jump_sim.py, measured <= 7 rounds for 4 KiB), then
//     one gather per byte, dword stores.
//
// Matches reaching into earlier batches, windows or linked blocks read the
// stream's own stored output back with L1-bypassing loads after a
// workgroup release fence (the stores are this workgroup's, on this XCD).
//
// The phases are plain functions of (shared state, thread id); the kernel
// runs them with barriers between, strom_lz4par_host() runs the SAME
// functions thread by thread on the CPU (tests/test_codecs_cpu.py pins it
// against the host LZ4 codec and pyarrow's frames).
//
// Snappy (raw format: varint length preamble, then elements) takes the same
// path with its own element grammar (template SN): an element is a literal
// run (tag 00, lengths in the tag or 1-4 bytes after it) or a copy (tags
// 01 / 10 / 11: 1-, 2- or 4-byte offsets) — a sequence with either no
// match or no literals — so speculation, validation, counting, the pointer
// fill and doubling are shared; the preamble's length is checked at the end.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "strom/strom.h"

#define HD __host__ __device__ inline

// lz4par_nt512.hip builds this file again with 512 threads per stream under
// its own namespace and entry point (LZ4P_NS / LZ4PAR_ENTRY, no host copy)
#ifndef LZ4P_NS
#define LZ4P_NS lz4p
#endif
#ifndef LZ4PAR_ENTRY
#define LZ4PAR_ENTRY strom_decompress_par
#endif

namespace LZ4P_NS {

#ifndef LZ4PAR_NT
#define LZ4PAR_NT 256
#endif
constexpr uint32_t NT = LZ4PAR_NT;       // threads per stream (4 waves)
#ifndef LZ4PAR_PW
#define LZ4PAR_PW 16384
#endif
constexpr uint32_t PW = LZ4PAR_PW;       // compressed bytes per parse window
constexpr uint32_t SL = PW / NT;         // slice per thread (64 B = 2 bitmap words)
constexpr uint32_t SW = SL / 32;         // bitmap words per slice
constexpr uint32_t PAD = 64;             // window overhang (reads past the window end)
#ifndef LZ4PAR_OB
#define LZ4PAR_OB 4096
#endif
#ifndef LZ4PAR_HR
#define LZ4PAR_HR 0
#endif
constexpr uint32_t OB = LZ4PAR_OB;       // output bytes per resolve batch
constexpr uint32_t HR = LZ4PAR_HR;       // LDS ring of the latest output (history), 0: none
constexpr uint32_t KW = OB / 4 / NT + 1; // output dwords a thread holds per batch
constexpr uint32_t EPT = OB / NT;        // batch entries a thread expands (contiguous)
constexpr uint32_t HW = OB / 32;         // run-head bitmap words
constexpr uint32_t HS = (HW + 31) / 32;  // summary words (bit w: head word w not empty)
// The pointer fill's unit of work: UB compressed bytes of a slice (CP per
// slice).  The count records where each unit's first sequence starts and
// its output offset; a batch's fill then runs on every thread whose unit
// meets it, not only on the ~OB / (output per slice) threads whose slices
// do (round 4: the fill was 0.27-0.48 of thread 0's cycles).
#ifndef LZ4PAR_UB
#define LZ4PAR_UB 16
#endif
constexpr uint32_t UB = LZ4PAR_UB < SL ? LZ4PAR_UB : SL;
constexpr uint32_t CP = SL / UB;
constexpr uint32_t kCkNone = 0xffu;      // checkpoint: no sequence starts in the unit
// Chain steps per entry per doubling round: 3 cut the host twin's rounds
// per stream from 662 to ~350 (text) and took 2,048 streams from 119 / 124
// / 114 GB/s (text / val / ids, one hop) to 133 / 136 / 125, snappy 111 /
// 105 / 97 to 126 / 115 / 107; 4 hops lose again on text / ids (LDS
// latency per round), profiles/r5/lz4par/lz4par_hops_ab_r5j.json
#ifndef LZ4PAR_HOPS
#define LZ4PAR_HOPS 3
#endif
constexpr uint32_t HOPS = LZ4PAR_HOPS;
// The count's prefix over the slices: a wave shuffle scan plus the waves'
// totals (2 barriers) instead of log2(NT) Hillis-Steele steps (2 each)
#ifndef LZ4PAR_WSCAN
#define LZ4PAR_WSCAN 1
#endif
constexpr bool WSCAN = LZ4PAR_WSCAN;
// Pointer doubling with no barrier per round (ph_double_async): off — the
// waves advance on stale values of each other's entries and need more
// passes than the round-synchronous loop saves in barriers (ids 118.7 vs
// 126.3 GB/s at 2,048 streams, text 128.0 vs 132.9, val level, snappy
// −1 to −6 %: profiles/r6/lz4par/async_doubling_ab_r6ad.json)
#ifndef LZ4PAR_ASYNC_DOUBLE
#define LZ4PAR_ASYNC_DOUBLE 0
#endif
constexpr bool ASYNC_DOUBLE = LZ4PAR_ASYNC_DOUBLE;
static_assert(LZ4PAR_NT % 64 == 0, "whole waves");
static_assert(SL % UB == 0 && SL < kCkNone, "fill units");
static_assert(OB % NT == 0 && 32 % EPT == 0 && HW <= NT && 4 * KW <= 32, "expansion tiling");
static_assert((HR & (HR - 1)) == 0, "ring: a power of two");
#ifndef LZ4PAR_LOOKBACK
#define LZ4PAR_LOOKBACK (LZ4PAR_NT == 512 ? 512 : 448)
#endif
// a speculative chain starts this many bytes before its slice (its bits
// are recorded from the slice start on): a chain from a wrong start needs
// ~100 bytes to fall onto the true token grid on int columns, and a slice
// whose chain has not merged by its true entry costs a serial fix-up round.
// 256-thread build, 2,048 / 8,192 streams (profiles/r6/lz4par/lookback_ab_r6y.json):
// 448 beats 512 on every column (val 137.9 / 141.1 vs 136.7 / 140.0, ids
// 126.6 / 130.7 vs 124.5 / 128.9, text level); 384 and 320 fall off the val
// cliff (~100 GB/s) for ids 128-135.  The 512-thread build keeps 512 (not
// measured at 448)
constexpr uint32_t LB = LZ4PAR_LOOKBACK;
// snappy's chains (with restarts) meet the true one within ~100 bytes:
// 512 -> 128 bytes of run-in took 512 streams from 55 / 44 / 39 GB/s
// (text / val / ids) to 72 / 59 / 40, 2048 streams text 71 -> 84, val
// 60 -> 71 (profiles/r4/dec/snappy_lookback_ab.json); 64 or 96 no better
#ifndef LZ4PAR_SN_LOOKBACK
#define LZ4PAR_SN_LOOKBACK 128
#endif
constexpr uint32_t SLB = LZ4PAR_SN_LOOKBACK;
// LZ4: NW speculative walkers per slice instead of one, started WLB,
// WLB - 1, ... bytes before it (NW = 1: the single chain from LB).  WLB
// 16: the walkers are there for the phases, not for a long run-in (text
// windows validate in one scan from 8 bytes back; 128 -> 16 took text from
// 85 to 97 GB/s, profiles/r4/dec/lz4par_walkers_wlb.json).  One
// chain phase-locks on dense LZ4 (text: 3-byte sequences whose offset high
// byte is 0 read as a token with no literals and a short match, so a chain
// entering 2 bytes late stays 2 bytes late): 30 % of text slices' chains
// never met the true one (16 windows x 36 validation rounds, 51 % of the
// decode's cycles).  Walkers from consecutive bytes start on every phase;
// they advance lowest position first and merge where they meet, so the
// steps are those of the distinct positions.  Replay of pyarrow's frames
// (tools/lz4par_bench.py kinds): text 30 % -> 0 % slices unmatched at
// 124 steps per slice instead of 189, val 0.35 % -> 0.35 % at 53 instead
// of 115 (r4 host simulation, profiles/r4/dec/lz4par_walkers.json).
#ifndef LZ4PAR_WALKERS
#define LZ4PAR_WALKERS 4
#endif
#ifndef LZ4PAR_WLOOKBACK
#define LZ4PAR_WLOOKBACK 16
#endif
constexpr uint32_t NW = LZ4PAR_WALKERS;
constexpr uint32_t WLB = LZ4PAR_WLOOKBACK;
static_assert(NW >= 1 && NW <= 8 && WLB >= NW, "walkers");
// A stream starts with the single chain (int columns merge: ~1.5 rounds a
// window, and the walkers cost their lockstep: val 110 -> 98 GB/s when
// always on) and switches to the walkers — that window again, and the
// stream's later ones — once a window needs WALK_AFTER rounds without the
// serial walk taking over (text: 36 rounds; a literal-heavy column goes
// serial at SERIAL_AFTER and stays).  The thresholds keep every window of
// the bench's 32 val frames single-chain (its worst needs 9 rounds at 64-
// byte slices, 23 at 32): one switched stream in 16 cost val 7 % of its
// GB/s, the launch waiting for its slowest workgroups.
#ifndef LZ4PAR_WALK_AFTER
#define LZ4PAR_WALK_AFTER (LZ4PAR_NT == 512 ? 24 : 10)
#endif
constexpr uint32_t WALK_AFTER = LZ4PAR_WALK_AFTER;
// ... or already after WALK_EARLY rounds when an eighth of the slices
// re-parsed in the last one and the serial walk would not take over (a
// phase-locked text window; an int column re-parses a slice or two)
#ifndef LZ4PAR_WALK_EARLY
#define LZ4PAR_WALK_EARLY 2
#endif
constexpr uint32_t WALK_EARLY = LZ4PAR_WALK_EARLY;
// Snappy walks from its first window: its single chains meet the true one
// (restarting at a failed parse) but the settled-prefix rounds still
// re-walked 1-3 slices a window on int columns; four walkers from
// SWLB..SWLB-3 bytes back validate every text / val / ids window of the
// bench frames in one scan with no re-parse (host twin, 8 frames each:
// ids 488 rounds + 4,584 re-walks -> 136 scans + 0).
#ifndef LZ4PAR_SN_WALK
#define LZ4PAR_SN_WALK 1
#endif
// GPU A/B (profiles/r4/dec/snappy_walkers_ab.json), 2,048 streams: text /
// val / ids / chars 84 / 71 / 56 / 315 GB/s with the settled prefix, 85 /
// 77 / 78 / 314 with walkers from 16 bytes back (32: 84 / 75 / 76; 128:
// 76 / 66 / 65); the 512-thread build takes 32 (512 streams 71 / 64 / 65).
#ifndef LZ4PAR_SN_WLOOKBACK
#define LZ4PAR_SN_WLOOKBACK 16
#endif
constexpr bool SN_WALK = LZ4PAR_SN_WALK && NW > 1;
constexpr uint32_t SWLB = LZ4PAR_SN_WLOOKBACK;
#ifndef LZ4PAR_RESTART
#define LZ4PAR_RESTART 1
#endif
constexpr bool RESTART = LZ4PAR_RESTART;   // restart a speculative chain at a failed parse
constexpr uint32_t kLit = 0x80000000u;   // pointer tag: literal, input position
constexpr uint32_t kHist = 0x40000000u;  // pointer tag: stored output position
constexpr uint32_t kTag = kLit | kHist;
constexpr uint32_t kPosMax = 1u << 30;   // streams and outputs below 1 GiB
static_assert(SL % 32 == 0, "slices cover whole bitmap words");

enum : int32_t { kErrFormat = -1, kErrOverflow = -2, kErrDistance = -3 };
enum : uint32_t { kModeBlock = 0, kModeDone = 1 };

// LDS bank spreading (32 banks of 4 bytes).  Thread t works at slice t of
// the window (SL = 64 bytes: the same bank every 2 lanes) and expands
// entries [16t, 16t + 16) of the pointer batch (again every 2 lanes): one
// pad dword per 128 window bytes / per 32 entries puts 32 lanes on 32
// distinct banks.
HD constexpr uint32_t WI(uint32_t r) { return r + ((r >> 7) << 2); }
HD constexpr uint32_t PI(uint32_t e) { return e + (e >> 5); }

// the walkers' marks and exits (LZ4, NW > 1), live from the speculation to
// the end of validation: they share LDS with the pointer batch, live after
struct WalkMem {
  uint32_t bits[NW * (PW / 32)];   // walker j, slice t: bits[j * PW / 32 + SW * t + i]
  uint32_t ex[NW * NT];            // walker j, slice t: ex[j * NT + t]
};

struct Smem {
  uint8_t win[WI(PW + PAD) + 4];
  union {
    struct {
      uint32_t bits[PW / 32];  // the chain slice t follows (a walker's, or a fix-up's)
      uint32_t en[NT];         // true entry of slice t
    };
    // from the count on: unit u's first sequence, (output offset in its
    // slice << 8) | (input offset in its slice), or kCkNone
    uint32_t ck[NT * CP];
  };
  uint32_t ex[NT];       // exit of slice t's chain
  uint32_t ost[NT];      // output bytes of slice t's true sequences, then their inclusive prefix
  union {
    uint32_t ptr[PI(OB)];
    WalkMem wk;
  };
  uint32_t hb[HW];       // run heads of the batch (entries whose pointer fill wrote)
  uint32_t hsum[HS];
  uint8_t ring[HR ? HR : 4];   // output byte at absolute position x: ring[x % HR]
  // stream scalars (thread 0 writes, everyone reads after a barrier)
  uint32_t ip;           // input position of the next block header
  uint32_t bstart, bend; // current block
  uint32_t braw;         // current block stored uncompressed
  uint32_t ws, wend, wload;   // window start (a true token), parse end, bytes in win
  uint32_t op;           // output bytes so far
  uint32_t total;        // output bytes of the current window
  int32_t err;
  uint32_t mode;
  uint32_t bcs;          // 4-byte checksum after each block
  uint32_t raw_block;    // codec LZ4: the whole input is one block
  uint32_t expect;       // snappy: the preamble's decoded length (else ~0)
  uint32_t minfix;       // snappy: first slice not yet settled
  uint32_t cov;          // snappy: last slice settled by the current round
  uint32_t walk;         // LZ4: this stream speculates with walkers (WALK_AFTER)
};

static_assert(sizeof(WalkMem) <= sizeof(uint32_t) * PI(OB), "walkers fit the pointer batch");

struct Ctx {
  const uint8_t *in;
  uint8_t *out;
  uint32_t len;          // input bytes
  uint32_t cap;          // output capacity
};

// ---------------------------------------------------------------- input
HD uint8_t inb(const Smem &s, const Ctx &c, uint32_t p) {
  const uint32_t r = p - s.ws;
#ifdef __HIP_DEVICE_COMPILE__
  // explicit address spaces: left generic, the two loads were merged into
  // one flat load of a selected pointer on the parse paths (round 4: 54
  // flat_load_ubyte in the LZ4 kernel, ~10 % slower than round 3's
  // ds_read / global_load split)
  typedef __attribute__((address_space(3))) const uint8_t lds_u8;
  typedef __attribute__((address_space(1))) const uint8_t glb_u8;
  if (r < s.wload) return ((lds_u8 *)s.win)[WI(r)];
  return p < c.len ? ((glb_u8 *)c.in)[p] : 0;
#else
  if (r < s.wload) return s.win[WI(r)];
  return p < c.len ? c.in[p] : 0;
#endif
}

HD uint32_t rd32(const Ctx &c, uint32_t p) {
  if (p + 4 > c.len) return 0xffffffffu;
  return (uint32_t)c.in[p] | ((uint32_t)c.in[p + 1] << 8) | ((uint32_t)c.in[p + 2] << 16) |
         ((uint32_t)c.in[p + 3] << 24);
}

struct Seq {
  uint32_t lit0, lit, off, mlen, next;
  bool last;
};

// One snappy element at p: a literal run (off = mlen = 0) or a copy (lit =
// 0).  false: malformed.
HD bool parse_snappy(const Smem &s, const Ctx &c, uint32_t p, uint32_t bend, Seq &q) {
  const uint32_t tag = inb(s, c, p);
  uint32_t x = p + 1;
  const uint32_t kind = tag & 3;
  if (kind == 0) {
    uint32_t n = tag >> 2;
    if (n >= 60) {                       // 1-4 length bytes follow
      const uint32_t nb = n - 59;
      const uint32_t v = (uint32_t)inb(s, c, x) | ((uint32_t)inb(s, c, x + 1) << 8) |
                         ((uint32_t)inb(s, c, x + 2) << 16) | ((uint32_t)inb(s, c, x + 3) << 24);
      n = nb == 4 ? v : v & ((1u << (8 * nb)) - 1u);
      x += nb;
    }
    const uint64_t le = (uint64_t)x + n + 1;
    q.lit0 = x;
    q.lit = n + 1;
    q.off = q.mlen = 0;
    q.last = le >= bend;
    q.next = le < bend ? (uint32_t)le : bend;
    return le <= bend && n < kPosMax;
  }
  q.lit0 = x;
  q.lit = 0;
  if (kind == 1) {
    q.mlen = 4 + ((tag >> 2) & 7);
    q.off = ((tag >> 5) << 8) | inb(s, c, x);
    x += 1;
  } else if (kind == 2) {
    q.mlen = (tag >> 2) + 1;
    q.off = (uint32_t)inb(s, c, x) | ((uint32_t)inb(s, c, x + 1) << 8);
    x += 2;
  } else {
    q.mlen = (tag >> 2) + 1;
    q.off = (uint32_t)inb(s, c, x) | ((uint32_t)inb(s, c, x + 1) << 8) |
            ((uint32_t)inb(s, c, x + 2) << 16) | ((uint32_t)inb(s, c, x + 3) << 24);
    x += 4;
  }
  q.last = x >= bend;
  q.next = x < bend ? x : bend;
  return x <= bend && q.off != 0;
}

// One LZ4 sequence at p (block ends at bend).  false: malformed (for a
// speculative chain that just means "wrong start").
template <bool SN>
HD bool parse(const Smem &s, const Ctx &c, uint32_t p, uint32_t bend, Seq &q) {
  if (SN) return parse_snappy(s, c, p, bend, q);
  const uint32_t tok = inb(s, c, p);
  uint32_t x = p + 1;
  uint32_t lit = tok >> 4;
  if (lit == 15) {
    uint32_t b;
    do {
      b = inb(s, c, x);
      ++x;
      lit += b;
    } while (b == 255 && x < bend);
  }
  q.lit0 = x;
  q.lit = lit;
  const uint64_t le = (uint64_t)x + lit;
  if (le >= bend) {                      // the last sequence: literals only
    q.last = true;
    q.off = 0;
    q.mlen = 0;
    q.next = bend;
    return le == bend;
  }
  x = (uint32_t)le;
  q.off = (uint32_t)inb(s, c, x) | ((uint32_t)inb(s, c, x + 1) << 8);
  x += 2;
  uint32_t m = tok & 15;
  if (m == 15) {
    uint32_t b;
    do {
      b = inb(s, c, x);
      ++x;
      m += b;
    } while (b == 255 && x < bend);
  }
  q.mlen = m + 4;
  q.last = false;
  q.next = x < bend ? x : bend;
  return x < bend && q.off != 0;         // a match is never the block's end
}

HD void setbit(Smem &s, uint32_t p) {
  const uint32_t r = p - s.ws;
  s.bits[r >> 5] |= 1u << (r & 31);
}

HD bool getbit(const Smem &s, uint32_t p) {
  const uint32_t r = p - s.ws;
  return (s.bits[r >> 5] >> (r & 31)) & 1u;
}

HD uint32_t slice_lo(const Smem &s, uint32_t t) { return s.ws + t * SL; }
HD uint32_t slice_hi(const Smem &s, uint32_t t) {
  const uint32_t e = s.ws + (t + 1) * SL;
  return e < s.wend ? e : s.wend;
}

// ---------------------------------------------------------------- phases
// window load: input bytes [ws, ws + wload) into LDS
#ifndef LZ4PAR_LOADU
#define LZ4PAR_LOADU 16
#endif
HD void ph_load(Smem &s, const Ctx &c, uint32_t t) {
  // all loads of a thread issued before the first LDS store (16 at a time):
  // a plain loop waited for each load in turn
  constexpr uint32_t U = LZ4PAR_LOADU;
  for (uint32_t j0 = 0; j0 * NT < s.wload; j0 += U) {
    uint8_t r[U];
#pragma unroll
    for (uint32_t j = 0; j < U; ++j) {
      const uint32_t i = t + (j0 + j) * NT;
      r[j] = i < s.wload ? c.in[s.ws + i] : 0;
    }
#pragma unroll
    for (uint32_t j = 0; j < U; ++j) {
      const uint32_t i = t + (j0 + j) * NT;
      if (i < s.wload) s.win[WI(i)] = r[j];
    }
  }
}

// (1') LZ4 speculative walkers of slice t.  Walker slots hold a position
// and the mask of walker ids that have merged into them; every id keeps its
// own marks (registers, fully unrolled: no scratch) and exit.  The slice
// starts on walker 0's chain.
template <bool SN>
HD void ph_spec_walk(Smem &s, const Ctx &c, uint32_t t) {
  const uint32_t lo = slice_lo(s, t), hi = slice_hi(s, t);
  uint32_t wp[NW], wm[NW];
  uint32_t *wb = s.wk.bits + SW * t;     // walker j's words: wb[j * PW / 32 + i]
#pragma unroll
  for (uint32_t w = 0; w < NW; ++w) {
    const uint32_t back = (SN ? SWLB : WLB) - w;
    wp[w] = lo - s.ws > back ? lo - back : s.ws;   // the window start is a true token
    wm[w] = lo < hi ? 1u << w : 0u;
#pragma unroll
    for (uint32_t i = 0; i < SW; ++i) wb[w * (PW / 32) + i] = 0;
  }
  for (;;) {
    uint32_t pm = 0xffffffffu;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w)
      if (wm[w] && wp[w] < pm) pm = wp[w];
    if (pm >= hi) break;
    // every walker at pm merges into the first of them
    uint32_t m = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w)
      if (wm[w] && wp[w] == pm) m |= wm[w];
    bool kept = false;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w)
      if (wm[w] && wp[w] == pm) {
        wm[w] = kept ? 0u : m;
        kept = true;
      }
    // marks straight to LDS (the slice's words are this thread's): held in
    // registers they cost 8 VGPRs and the 4th workgroup per CU
    if (pm >= lo) {
      const uint32_t r = pm - lo, bit = 1u << (r & 31);
#pragma unroll
      for (uint32_t w = 0; w < NW; ++w)
        if ((m >> w) & 1u) wb[w * (PW / 32) + (r >> 5)] |= bit;
    }
    Seq q;
    // a failed parse: an LZ4 chain goes on anyway; a snappy one restarts at
    // the next byte (a garbage literal tag may claim kilobytes)
    if (!parse<SN>(s, c, pm, s.bend, q) && SN) q.next = pm + 1;
    kept = false;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w)
      if (wm[w] && wp[w] == pm && !kept) {
        wp[w] = q.next;
        kept = true;
      }
  }
#pragma unroll
  for (uint32_t j = 0; j < NW; ++j) {
    uint32_t e = lo;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w)
      if ((wm[w] >> j) & 1u) e = wp[w];
    s.wk.ex[j * NT + t] = e;
    if (j == 0) s.ex[t] = e;
  }
#pragma unroll
  for (uint32_t i = 0; i < SW; ++i) s.bits[SW * t + i] = wb[i];
}

// The first walker of slice t whose chain holds position e (>= the slice
// start), or NW: a chain through e is the true one from e on whatever
// came before, and its earlier marks are never read (counting starts at
// the entry), so for e past the slice an exit equal to e suffices
HD uint32_t wv_holder(const Smem &s, uint32_t t, uint32_t e) {
  const uint32_t hi = slice_hi(s, t);
  for (uint32_t k = 0; k < NW; ++k) {
    if (e < hi) {
      const uint32_t r = e - s.ws;
      if ((s.wk.bits[k * (PW / 32) + (r >> 5)] >> (r & 31)) & 1u) return k;
    } else if (s.wk.ex[k * NT + t] == e) {
      return k;
    }
  }
  return NW;
}

// walker k's marks and exit become slice t's
HD void wv_adopt(Smem &s, uint32_t t, uint32_t k) {
  for (uint32_t i = 0; i < SW; ++i) s.bits[SW * t + i] = s.wk.bits[k * (PW / 32) + SW * t + i];
  s.ex[t] = s.wk.ex[k * NT + t];
}

// slice t's chain from `ent`, if one of its walkers holds it
HD bool adopt_walker(Smem &s, uint32_t t, uint32_t ent) {
  const uint32_t k = wv_holder(s, t, ent);
  if (k >= NW) return false;
  wv_adopt(s, t, k);
  return true;
}

// (1) speculative chain of slice t
template <bool SN>
HD void ph_spec(Smem &s, const Ctx &c, uint32_t t, bool walk) {
  if constexpr (NW > 1) {
    if (walk) {
      ph_spec_walk<SN>(s, c, t);
      return;
    }
  }
  const uint32_t lo = slice_lo(s, t), hi = slice_hi(s, t);
  for (uint32_t i = 0; i < SW; ++i) s.bits[SW * t + i] = 0;
  if (lo >= hi) {
    s.ex[t] = lo;
    return;
  }
  constexpr uint32_t lb = SN ? SLB : LB;
  uint32_t p = lo - s.ws > lb ? lo - lb : s.ws;   // the window start is a true token
  Seq q;
  while (p < hi) {
    if (p >= lo) setbit(s, p);
    // a token no valid stream can hold (a length running past the block, a
    // zero offset) proves the chain wrong: restart it at the next byte
    // instead of letting it die.  The true chain never fails a parse, so
    // from any marked token it reaches, the chain continues as the true one.
    // Snappy only: a garbage literal tag of kind 60-63 carries a 1-4 byte
    // length — one tag in 64 of random bytes — and killed most chains
    // (round 4, val columns 182 validation rounds per window, 12 after);
    // LZ4 chains merge anyway and the restarts only cost there
    // (profiles/r4/dec/lz4_variant_ab.json).
    if (!parse<SN>(s, c, p, s.bend, q) && SN && RESTART) {
      ++p;
      continue;
    }
    p = q.next;
  }
  s.ex[t] = p;
}

// (2) validation round, read half: the entry slice t sees now
HD uint32_t ph_entry(const Smem &s, uint32_t t) { return t == 0 ? s.ws : s.ex[t - 1]; }

// (2) validation round, fix half: true when slice t had to re-parse
template <bool SN>
HD bool ph_fix(Smem &s, const Ctx &c, uint32_t t, uint32_t ent) {
  const uint32_t lo = slice_lo(s, t), hi = slice_hi(s, t);
  if (lo >= hi) return false;
  s.en[t] = ent;
  bool valid;
  if (ent < hi) {
    valid = getbit(s, ent);
  } else {
    uint32_t any = 0;
    for (uint32_t i = 0; i < SW; ++i) any |= s.bits[SW * t + i];
    valid = any == 0 && s.ex[t] == ent;
  }
  if (valid) return false;
  for (uint32_t i = 0; i < SW; ++i) s.bits[SW * t + i] = 0;
  uint32_t p = ent;
  Seq q;
  while (p < hi) {
    setbit(s, p);
    parse<SN>(s, c, p, s.bend, q);
    p = q.next;
  }
  s.ex[t] = p;
  return true;
}

// (2'') LZ4 windows whose chains do not merge: thread 0 walks the rest of
// the window's true chain itself.  A slice inside a long literal run (an
// incompressible column: 96 % literals, one token per ~370 input bytes for
// pyarrow's LZ4 of random-letter strings) sees garbage tokens, and its
// wrong chain meets the true one only by landing on a true token — never,
// at that density — so the rounds fix one slice each (110 per 16 KiB
// window, ~4 us apiece: the whole decode time of such a column, r4
// strings trace).  A serial walk of the true chain costs one step per TRUE
// token, ~44 per such window.  Slices from `f` on get their final entry
// and exit; a slice whose own chain holds the entry keeps its marks.
template <bool SN>
HD uint32_t ph_serial(Smem &s, const Ctx &c, uint32_t f, uint32_t nsl, bool walk) {
  uint32_t p = s.ex[f - 1], steps = 0;
  for (uint32_t t = f; t < nsl; ++t) {
    const uint32_t lo = slice_lo(s, t), hi = slice_hi(s, t);
    if (lo >= hi) break;
    s.en[t] = p;
    if (p < hi && getbit(s, p)) {    // merged: the slice's chain from p is its own
      p = s.ex[t];
      continue;
    }
    if constexpr (!SN && NW > 1) {
      if (walk && p < hi && adopt_walker(s, t, p)) {   // (single chain: no walkers)
        p = s.ex[t];
        continue;
      }
    }
    for (uint32_t i = 0; i < SW; ++i) s.bits[SW * t + i] = 0;
    Seq q;
    while (p < hi) {
      setbit(s, p);
      parse<SN>(s, c, p, s.bend, q);
      p = q.next;
      ++steps;
    }
    s.ex[t] = p;
  }
  return steps;
}

// From round SERIAL_AFTER on, a window walks serially when its final
// prefix (slices up to the frontier f) predicts at most SERIAL_TOKENS true
// tokens in the rest: a serial step costs about what a round's slowest
// slice does, and the rounds advance the frontier a slice or two each (a
// dense column — text, 3 input bytes per token — keeps its rounds: its
// chains merge, and 5,000 serial steps would cost more).
#ifndef LZ4PAR_SERIAL_AFTER
#define LZ4PAR_SERIAL_AFTER 3
#endif
#ifndef LZ4PAR_SERIAL_TOKENS
#define LZ4PAR_SERIAL_TOKENS 256
#endif
constexpr uint32_t SERIAL_AFTER = LZ4PAR_SERIAL_AFTER;
constexpr uint32_t SERIAL_TOKENS = LZ4PAR_SERIAL_TOKENS;

HD bool serial_worth(const Smem &s, uint32_t f) {
  uint32_t tok = 0;
  for (uint32_t i = 0; i < SW * (f + 1); ++i) tok += (uint32_t)__builtin_popcount(s.bits[i]);
  const uint32_t done = s.ex[f] - s.ws, rest = s.wend > s.ex[f] ? s.wend - s.ex[f] : 0;
  return (uint64_t)tok * rest <= (uint64_t)SERIAL_TOKENS * (done ? done : 1);
}

// (2*) LZ4 walker validation (NW > 1): no re-parse rounds.  Slice t's
// transition map sends its walker j to the walker of slice t+1 that holds
// j's exit (NW: none holds it); slice 0's walkers all start at the window
// start, a true token, so the true chain of slice t is walker
// (M_{t-1} o ... o M_0)(0) — an inclusive scan of map compositions, log2 NT
// steps.  The first slice f whose walker comes out "none" re-parses from
// its (final) entry; its map becomes the constant "the walker of f+1
// holding my exit" (slices it passes whole, inside one literal run, too),
// and the scan runs again.  Iterations: misses + 1 (text ~1 per 6 windows,
// val ~1 per window), against ~36 re-parse rounds per text window before.
// Maps pack NW + 1 4-bit entries, entry NW being "none" in and out.
HD uint32_t wv_get(uint32_t m, uint32_t j) { return (m >> (4 * j)) & 15u; }

HD uint32_t wv_const(uint32_t h) {
  uint32_t m = 0;
  for (uint32_t j = 0; j <= NW; ++j) m |= h << (4 * j);
  return m;
}

// a after b
HD uint32_t wv_compose(uint32_t a, uint32_t b) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t j = 0; j <= NW; ++j) m |= wv_get(a, wv_get(b, j)) << (4 * j);
  return m;
}

// slice t's map (`fixed`: the slice's chain is final, from its re-parse)
HD uint32_t wv_map(const Smem &s, uint32_t t, uint32_t nsl, bool fixed) {
  if (t + 1 >= nsl) return wv_const(NW);
  if (fixed) return wv_const(wv_holder(s, t + 1, s.ex[t]));
  uint32_t m = NW << (4 * NW);
  for (uint32_t j = 0; j < NW; ++j) m |= wv_holder(s, t + 1, s.wk.ex[j * NT + t]) << (4 * j);
  return m;
}

// slice t re-parses from its final entry
template <bool SN>
HD void wv_fix(Smem &s, const Ctx &c, uint32_t t, uint32_t ent) {
  const uint32_t hi = slice_hi(s, t);
  for (uint32_t i = 0; i < SW; ++i) s.bits[SW * t + i] = 0;
  uint32_t p = ent;
  Seq q;
  while (p < hi) {
    setbit(s, p);
    parse<SN>(s, c, p, s.bend, q);
    p = q.next;
  }
  s.ex[t] = p;
}

// after slice f's re-parse: slice t lies wholly before f's exit (inside one
// element), so its chain is empty and its exit f's
HD bool wv_pass(Smem &s, uint32_t t, uint32_t f) {
  const uint32_t e = s.ex[f];
  if (t <= f || slice_lo(s, t) >= slice_hi(s, t) || slice_hi(s, t) > e) return false;
  for (uint32_t i = 0; i < SW; ++i) s.bits[SW * t + i] = 0;
  s.ex[t] = e;
  return true;
}

// (2') snappy validation: a SETTLED prefix instead of rounds in which every
// slice re-parses from its predecessor's current exit.  Snappy chains from
// wrong starts merge within ~100 bytes, but one that reads a garbage
// literal tag with a 1-4 byte length jumps kilobytes ahead; in the round
// scheme that wrong exit travelled forward one slice per round ahead of the
// correction (round 4: 220 rounds in one 16 KiB window of val data).  Here:
//   link(t)   slice t accepts its predecessor's speculative exit (a token
//             its own chain marked): then its speculative exit is right
//             whenever its predecessor's is;
//   a round   settles the FIRST slice S without a link (its entry, the
//             settled exit of S-1, is final): parse from it (or pass it
//             through when it lies past the slice), then every later slice
//             wholly before the new exit sits inside one element and takes
//             it too (a long literal of incompressible bytes spans hundreds
//             of slices); the next slice re-checks its link against it;
//   meanwhile every other broken slice re-walks from its predecessor's
//   current exit (the round-4 A/B: sorted-id columns break often and
//   resolve in parallel this way), unless that exit lies past the slice —
//   a far jump is never passed on before it is settled.
// Rounds <= breaks in the chain of links, not slices.
HD bool sn_link(const Smem &s, uint32_t t, uint32_t ent) {
  const uint32_t hi = slice_hi(s, t);
  return ent < hi && getbit(s, ent);
}

// slice t's chain from `ent`: its marks and exit replace the old ones (a
// slice's marks and exit always belong to one chain, so a link check stays
// sound whatever entry the chain came from)
HD void sn_walk(Smem &s, const Ctx &c, uint32_t t, uint32_t ent) {
  const uint32_t lo = slice_lo(s, t), hi = slice_hi(s, t);
  uint32_t p = ent;
  if (lo < hi && ent < hi) {
    for (uint32_t i = 0; i < SW; ++i) s.bits[SW * t + i] = 0;
    Seq q;
    while (p < hi) {
      setbit(s, p);
      parse<true>(s, c, p, s.bend, q);
      p = q.next;
    }
  }
  s.ex[t] = p;
}

// settle slice t from its final entry; returns the last slice it covers
HD uint32_t sn_settle(Smem &s, const Ctx &c, uint32_t t, uint32_t ent) {
  sn_walk(s, c, t, ent);
  const uint32_t p = s.ex[t];
  const uint32_t n = (s.wend - s.ws + SL - 1) / SL;
  uint32_t j = t + 1;
  for (; j < n && slice_hi(s, j) <= p; ++j) s.ex[j] = p;
  return j - 1;
}

// (3) output bytes of slice t's true sequences from its entry `ent` (read
// from s.en before a barrier: the checkpoints overwrite it) and the
// checkpoint of each of its fill units (errors set s.err)
template <bool SN>
HD void ph_count(Smem &s, const Ctx &c, uint32_t t, uint32_t ent) {
  const uint32_t lo = slice_lo(s, t), hi = slice_hi(s, t);
  uint32_t o = 0, j = 0;
  if (lo < hi) {
    uint32_t p = ent;
    Seq q;
    while (p < hi) {
      // p is the first sequence of every unit whose start it has reached
      // (an output offset past 24 bits merges the slice's later units)
      for (; j < CP && p >= lo + j * UB; ++j)
        s.ck[t * CP + j] = o < (1u << 24) ? (o << 8) | (p - lo) : kCkNone;
      if (!parse<SN>(s, c, p, s.bend, q)) {
        s.err = kErrFormat;
        break;
      }
      const uint64_t n = (uint64_t)o + q.lit + q.mlen;
      if (n >= kPosMax) {
        s.err = kErrOverflow;
        break;
      }
      o = (uint32_t)n;
      p = q.next;
    }
  }
  for (; j < CP; ++j) s.ck[t * CP + j] = kCkNone;
  s.ost[t] = o;
  if (t < HW) s.hb[t] = 0;
  if (t < HS) s.hsum[t] = 0;
}

// (3) inclusive scan step d (Hillis-Steele; read and write halves)
HD uint32_t ph_scan_read(const Smem &s, uint32_t t, uint32_t d) { return t >= d ? s.ost[t - d] : 0; }
HD void ph_scan_write(Smem &s, uint32_t t, uint32_t v) { s.ost[t] += v; }

// (4a) source pointers of the batch [b0, b0 + OB): slice t's sequences
// write the pointer of the FIRST byte of each run (literal run, match run;
// a match run whose source crosses the batch start is two runs) and mark
// it in the head bitmap; (4a') fills the rest.  Within a run the pointer
// grows by one per byte in all three kinds (input position, stored output
// position, batch index), so entry e = ptr[h] + (e - h) for the last head
// h <= e.  Only the ~OB/(output per slice) threads whose slices meet the
// batch have work in (4a); (4a') spreads the per-byte writes over all.
HD void head(Smem &s, uint32_t e, uint32_t v) {
  s.ptr[PI(e)] = v;
  const uint32_t w = e >> 5;
#ifdef __HIP_DEVICE_COMPILE__
  atomicOr(&s.hb[w], 1u << (e & 31));
  atomicOr(&s.hsum[w >> 5], 1u << (w & 31));
#else
  s.hb[w] |= 1u << (e & 31);
  s.hsum[w >> 5] |= 1u << (w & 31);
#endif
}

// (4a) thread t fills for units t, t + NT, ...: consecutive units (one
// slice's, then the next slice's) on consecutive threads, so the ~OB /
// (output per unit) units a batch meets spread over as many threads.  A
// unit longer than a batch is walked again from its start by the next one.
template <bool SN>
HD void ph_fill(Smem &s, const Ctx &c, uint32_t t, uint32_t b0) {
  const uint32_t b1 = b0 + OB;
  const uint32_t opw = s.op;             // output position of the window start
  for (uint32_t k = 0; k < CP; ++k) {
    const uint32_t u = t + k * NT, sl = u / CP, j = u % CP;
    const uint32_t v = s.ck[u];
    if ((v & 0xff) == kCkNone) continue;
    const uint32_t base = sl ? s.ost[sl - 1] : 0, lo = slice_lo(s, sl);
    uint32_t o = base + (v >> 8);
    if (o >= b1) continue;
    // the unit ends where the slice's next unit with a sequence starts
    uint32_t oend = s.ost[sl], pend = slice_hi(s, sl);
    for (uint32_t i = j + 1; i < CP; ++i) {
      const uint32_t w = s.ck[sl * CP + i];
      if ((w & 0xff) != kCkNone) {
        oend = base + (w >> 8);
        pend = lo + (w & 0xff);
        break;
      }
    }
    if (oend <= b0) continue;
    uint32_t p = lo + (v & 0xff);
    Seq q;
    while (p < pend && o < b1) {
      parse<SN>(s, c, p, s.bend, q);     // checked by ph_count
      const uint32_t le = o + q.lit;
      if (le > b0 && q.lit) {
        const uint32_t x0 = o > b0 ? o : b0;
        head(s, x0 - b0, kLit | (q.lit0 + (x0 - o)));
      }
      o = le;
      if (SN ? q.mlen != 0 : !q.last) {
        const uint32_t me = o + q.mlen;
        if (me > b0 && o < b1) {
          if ((uint64_t)q.off > (uint64_t)opw + o) {
            s.err = kErrDistance;
            return;
          }
          const uint32_t x0 = o > b0 ? o : b0, x1 = me < b1 ? me : b1;
          // source of byte x: absolute opw + x - off; inside the batch (index
          // x - off - b0) from x = b0 + off on, stored history before
          const uint32_t xs = b0 + q.off;
          if (x0 < xs) {
            head(s, x0 - b0, kHist | (opw + x0 - q.off));
            if (xs < x1) head(s, xs - b0, 0);
          } else {
            head(s, x0 - b0, x0 - q.off - b0);
          }
        }
        o = me;
      }
      p = q.next;
    }
  }
}

HD uint32_t clz32(uint32_t x) { return (uint32_t)__builtin_clz(x); }

// (4a') expansion: thread t fills entries [t * EPT, t * EPT + EPT)
HD void ph_expand(Smem &s, uint32_t t, uint32_t nb) {
  const uint32_t e0 = t * EPT;
  if (e0 >= nb) return;
  const uint32_t w = e0 >> 5, sh = e0 & 31;
  // the last head at or before e0 (entry 0 always is one)
  const uint32_t m = s.hb[w] & (0xffffffffu >> (31 - sh));
  uint32_t h = 0;
  if (m) {
    h = (w << 5) + 31 - clz32(m);
  } else if (w) {
    int32_t sw = (int32_t)((w - 1) >> 5);
    uint32_t sm = s.hsum[sw] & (0xffffffffu >> (31 - ((w - 1) & 31)));
    while (!sm && --sw >= 0) sm = s.hsum[sw];
    if (sm) {
      const uint32_t wl = ((uint32_t)sw << 5) + 31 - clz32(sm);
      h = (wl << 5) + 31 - clz32(s.hb[wl]);
    }
  }
  uint32_t cur = h, base = s.ptr[PI(h)];
  const uint32_t hm = s.hb[w] >> sh;
  for (uint32_t i = 0; i < EPT; ++i) {
    const uint32_t e = e0 + i;
    if ((hm >> i) & 1u) {
      cur = e;
      base = s.ptr[PI(e)];
    } else {
      // a match run whose source is inside the batch starts off = cur -
      // base bytes after it; past off bytes the run copies itself
      // (overlapping match: RLE-like runs), so byte e also equals the
      // source byte (e - cur) mod off — one step to a byte before the run
      // instead of a chain through the run that pointer doubling would
      // need log2(run / off) rounds for
      uint32_t d = e - cur;
      if (!(base & kTag) && base < cur) {
        const uint32_t off = cur - base;
        if (d >= off) d = off == 1 ? 0 : d % off;
      }
      s.ptr[PI(e)] = base + d;
    }
  }
}

// (4b) one pointer-doubling round over the batch; true while any pointer
// still points inside the batch
HD bool ph_double(Smem &s, uint32_t t, uint32_t nb) {
  // in order, each replacement visible to the thread's later entries (a
  // chain through this thread's entries collapses within the round;
  // reading all entries before writing any measured 30 % slower)
  bool more = false;
  for (uint32_t e = t; e < nb; e += NT) {
    const uint32_t v = s.ptr[PI(e)];
    if (!(v & kTag)) {
      // v < e always (a match reads backwards); the bound only keeps a
      // corrupt table inside the array.  HOPS > 1 follows the chain further
      // within the round (any value read is a valid pointer of the byte:
      // they only move towards the root), trading LDS latency for rounds.
      uint32_t w = v < e ? s.ptr[PI(v)] : kLit;
      for (uint32_t k = 1; k < HOPS && !(w & kTag); ++k) {
        const uint32_t x = w;
        w = x < e ? s.ptr[PI(x)] : kLit;
      }
      s.ptr[PI(e)] = w;
      more |= !(w & kTag);
    }
  }
  return more;
}

// (4b') the doubling without a barrier per round: each thread repeats
// passes over its own unresolved entries until all of them hold a tagged
// (final) pointer.  Correct without synchronization because every value an
// entry ever holds is a valid pointer of its byte and pointers only move
// towards the roots (v < e, roots are tagged and never change): a stale read
// of another wave's entry is an earlier point of the same chain, so a pass
// still moves each entry at least one step, and a thread ends in at most
// (chain length) passes even if no other wave progressed.  LDS accesses are
// volatile so each pass sees the other waves' latest replacements; the
// caller's barrier after it publishes the result.
__device__ __forceinline__ void ph_double_async(Smem &s, uint32_t t, uint32_t nb) {
  volatile uint32_t *p = s.ptr;
  bool more = true;
  while (more) {
    more = false;
    for (uint32_t e = t; e < nb; e += NT) {
      const uint32_t v = p[PI(e)];
      if (v & kTag) continue;
      uint32_t w = v < e ? p[PI(v)] : kLit;
      for (uint32_t k = 1; k < HOPS && !(w & kTag); ++k) {
        const uint32_t x = w;
        w = x < e ? p[PI(x)] : kLit;
      }
      p[PI(e)] = w;
      more |= !(w & kTag);
    }
  }
}

HD uint8_t hist_byte(const Ctx &c, uint32_t pos) {
#ifdef __HIP_DEVICE_COMPILE__
  // stored by this workgroup in an earlier batch, visible after the
  // release fence + barrier that ended it; bypass L1 (it may hold an older
  // copy of the line)
  const uint32_t *w = (const uint32_t *)(((uintptr_t)(c.out + pos)) & ~(uintptr_t)3);
  const uint32_t d = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint8_t)(d >> (8 * (((uintptr_t)(c.out + pos)) & 3)));
#else
  return c.out[pos];
#endif
}

HD uint8_t resolve(const Smem &s, const Ctx &c, uint32_t v) {
  if (v & kLit) return inb(s, c, v & ~kLit);
  return hist_byte(c, v & ~kHist);
}

// (4c) gather: thread t resolves the output dwords it owns (aligned in
// HBM) into registers; history within HR bytes comes from the LDS ring
// (read-only in this phase), older history from HBM
struct Held {
  uint32_t w[KW];
};

HD void ph_resolve(const Smem &s, const Ctx &c, uint32_t t, uint32_t b0, uint32_t nb, Held &h) {
  const uint8_t *base = c.out + s.op + b0;
  const uint32_t mis = (uint32_t)((uintptr_t)base & 3);
  const uint32_t nw = (nb + mis + 3) / 4;
  const uint32_t bs = s.op + b0;         // absolute output position of the batch
  for (uint32_t j = 0; j < KW; ++j) {
    const uint32_t k = t + j * NT;
    uint32_t w = 0;
    if (k < nw) {
      for (uint32_t b = 0; b < 4; ++b) {
        const int32_t e = (int32_t)(4 * k + b) - (int32_t)mis;
        if (e < 0 || (uint32_t)e >= nb) continue;
        const uint32_t v = s.ptr[PI(e)];
        uint8_t x;
        if (v & kLit) {
          x = inb(s, c, v & ~kLit);
        } else {
          const uint32_t hp = v & ~kHist;
          x = HR && bs - hp <= HR ? s.ring[hp & (HR - 1)] : hist_byte(c, hp);
        }
        w |= (uint32_t)x << (8 * b);
      }
    }
    h.w[j] = w;
  }
}

// (4d) store the held dwords to HBM and to the history ring
HD void ph_write(Smem &s, const Ctx &c, uint32_t t, uint32_t b0, uint32_t nb, const Held &h) {
  uint8_t *base = c.out + s.op + b0;
  const uint32_t mis = (uint32_t)((uintptr_t)base & 3);
  const uint32_t nw = (nb + mis + 3) / 4;
  const uint32_t bs = s.op + b0;
  if (t < HW) s.hb[t] = 0;               // heads of the next batch start empty
  if (t < HS) s.hsum[t] = 0;
  for (uint32_t j = 0; j < KW; ++j) {
    const uint32_t k = t + j * NT;
    if (k >= nw) break;
    const int32_t e0 = (int32_t)(4 * k) - (int32_t)mis;
    const uint32_t w = h.w[j];
    if (e0 >= 0 && (uint32_t)e0 + 4 <= nb) {
      *(uint32_t *)(base + e0) = w;
      if (HR)
        for (uint32_t b = 0; b < 4; ++b) s.ring[(bs + e0 + b) & (HR - 1)] = (uint8_t)(w >> (8 * b));
    } else {
      for (uint32_t b = 0; b < 4; ++b) {
        const int32_t e = e0 + (int32_t)b;
        if (e >= 0 && (uint32_t)e < nb) {
          base[e] = (uint8_t)(w >> (8 * b));
          if (HR) s.ring[(bs + e) & (HR - 1)] = (uint8_t)(w >> (8 * b));
        }
      }
    }
  }
}

// stored (uncompressed) block: [bstart, bend) -> out[op..]; its last HR
// bytes also go to the history ring
HD void ph_rawcopy(Smem &s, const Ctx &c, uint32_t t) {
  const uint32_t n = s.bend - s.bstart;
  const uint32_t keep = n > HR ? n - HR : 0;
  for (uint32_t i = t; i < n; i += NT) {
    const uint8_t x = c.in[s.bstart + i];
    c.out[s.op + i] = x;
    if (HR && i >= keep) s.ring[(s.op + i) & (HR - 1)] = x;
  }
}

// ---------------------------------------------------------------- scalar steps (thread 0)
// stream header: sets ip / bcs / raw_block, or mode done with op = bytes copied
HD void st_header(Smem &s, const Ctx &c, int codec) {
  s.op = 0;
  s.err = 0;
  s.walk = codec == STROM_CODEC_SNAPPY && SN_WALK;
  s.mode = kModeBlock;
  s.bcs = codec == STROM_CODEC_LZ4_FRAME_BCS;
  s.raw_block = codec == STROM_CODEC_LZ4;
  s.expect = 0xffffffffu;
  s.ip = 0;
  s.ws = 0;
  s.wload = 0;
  if (c.len >= kPosMax || c.cap >= kPosMax) {
    s.err = kErrOverflow;
    s.mode = kModeDone;
    return;
  }
  if (codec == STROM_CODEC_SNAPPY) {     // varint preamble: the decoded length
    uint32_t ul = 0, sh = 0, p = 0, b;
    do {
      if (p >= c.len || sh > 28) {
        s.err = kErrFormat;
        s.mode = kModeDone;
        return;
      }
      b = c.in[p++];
      ul |= (b & 0x7fu) << sh;
      sh += 7;
    } while (b & 0x80);
    if (ul > c.cap || ul >= kPosMax) {
      s.err = kErrOverflow;
      s.mode = kModeDone;
      return;
    }
    s.expect = ul;
    s.ip = p;
    s.raw_block = 4;                     // one element stream to the input end
    return;
  }
  if (codec != STROM_CODEC_ARROW_LZ4) return;
  if (c.len < 8) {
    s.err = kErrFormat;
    s.mode = kModeDone;
    return;
  }
  const uint32_t lo = rd32(c, 0), hi = rd32(c, 4);
  if (lo == 0xffffffffu && hi == 0xffffffffu) {   // -1: stored raw after the prefix
    s.bstart = 8;
    s.bend = c.len;
    s.braw = 1;
    s.raw_block = 2;                              // one stored block, then done
    return;
  }
  uint32_t p = 8;
  if (rd32(c, p) != 0x184D2204u || p + 7 > c.len) {
    s.err = kErrFormat;
    s.mode = kModeDone;
    return;
  }
  const uint32_t flg = c.in[p + 4];
  if ((flg >> 6) != 1) {
    s.err = kErrFormat;
    s.mode = kModeDone;
    return;
  }
  p += 6;                                         // magic, FLG, BD
  if (flg & 0x08) p += 8;                         // content size
  if (flg & 0x01) p += 4;                         // dictionary id
  p += 1;                                         // header checksum
  s.bcs = (flg >> 4) & 1;
  s.ip = p;
}

// next block: sets bstart/bend/braw, or mode done
HD void st_block(Smem &s, const Ctx &c) {
  if (s.raw_block == 4) {                         // snappy: the elements after the preamble
    s.raw_block = 3;
    s.bstart = s.ip;
    s.bend = c.len;
    s.braw = 0;
    if (s.bstart >= s.bend) s.mode = kModeDone;   // empty input
    return;
  }
  if (s.raw_block == 1) {                         // codec LZ4: one raw block
    s.raw_block = 3;
    s.bstart = 0;
    s.bend = c.len;
    s.braw = 0;
    return;
  }
  if (s.raw_block == 2) {                         // Arrow "-1": the stored copy
    s.raw_block = 3;
    return;
  }
  if (s.raw_block == 3) {
    s.mode = kModeDone;
    return;
  }
  const uint32_t h = rd32(c, s.ip);
  if (h == 0xffffffffu && s.ip + 4 > c.len) {     // ran off the input: no end mark
    s.mode = kModeDone;
    return;
  }
  if (h == 0) {                                   // end mark
    s.mode = kModeDone;
    return;
  }
  const uint32_t n = h & 0x7fffffffu;
  const uint64_t end = (uint64_t)s.ip + 4 + n;
  if (end > c.len) {
    s.err = kErrFormat;
    s.mode = kModeDone;
    return;
  }
  s.bstart = s.ip + 4;
  s.bend = (uint32_t)end;
  s.braw = h >> 31;
  s.ip = s.bend + (s.bcs ? 4 : 0);
}

HD void st_window(Smem &s, const Ctx &c, uint32_t ws) {
  s.ws = ws;
  const uint32_t we = ws + PW;
  s.wend = we < s.bend ? we : s.bend;
  const uint32_t ld = PW + PAD;
  s.wload = ws + ld <= c.len ? ld : c.len - ws;
}

}  // namespace LZ4P_NS

// ---------------------------------------------------------------- device
// -DSTROM_DECOMP_PROF (libstrom_decprof.so): thread 0 of every workgroup
// stamps s_memtime at each phase boundary; strom_lz4par_prof() returns the
// sums (tools/lz4par_bench.py --prof)
enum : int { kLpHdr, kLpLoad, kLpSpec, kLpValid, kLpScan, kLpFill, kLpDouble, kLpResolve,
             kLpWrite, kLpRaw, kLpExpand, kLpNWin, kLpNRound, kLpNBatch, kLpNDouble, kLpN };
#ifdef STROM_DECOMP_PROF
__device__ unsigned long long g_lz4par_prof[kLpN];
#define LP_INIT() uint64_t lp[kLpN] = {0}; uint64_t lp_t = __builtin_amdgcn_s_memtime()
#define LP_MARK(k)                                                    \
  do {                                                                \
    const uint64_t _n = __builtin_amdgcn_s_memtime();                 \
    lp[k] += _n - lp_t;                                               \
    lp_t = _n;                                                        \
  } while (0)
#define LP_CNT(k) (lp[k] += 1)
#define LP_FLUSH()                                                    \
  do {                                                                \
    if (t == 0)                                                       \
      for (int _i = 0; _i < kLpN; ++_i) atomicAdd(&g_lz4par_prof[_i], (unsigned long long)lp[_i]); \
  } while (0)
#else
#define LP_INIT() (void)0
#define LP_MARK(k) (void)0
#define LP_CNT(k) (void)0
#define LP_FLUSH() (void)0
#endif

namespace {
using namespace LZ4P_NS;

// Occupancy hints per grammar: the 512-thread build holds its LZ4 kernel at
// 80 VGPRs (6 waves per SIMD, 3 workgroups per CU — what round 3 measured
// 85 -> 115 GB/s with) without spilling; the snappy instantiation keeps the
// compiler's choice (it would spill there).
// The 256-thread LZ4 kernel is held at 128 VGPRs (4 waves per SIMD: its
// LDS allows 4 workgroups per CU); left alone the walkers' validation took
// it to 149 and one workgroup less.
#if !defined(LZ4PAR_WPE_LZ4) && LZ4PAR_NT == 256
#define LZ4PAR_WPE_LZ4 4
#endif
#if !defined(LZ4PAR_WPE) && LZ4PAR_NT == 256
#define LZ4PAR_WPE 4   // the snappy kernel likewise (140 with its walkers)
#endif
#ifdef LZ4PAR_WPE
#define LZ4PAR_OCC __attribute__((amdgpu_waves_per_eu(LZ4PAR_WPE)))
#else
#define LZ4PAR_OCC
#endif
#ifdef LZ4PAR_WPE_LZ4
#define LZ4PAR_OCC_LZ4 __attribute__((amdgpu_waves_per_eu(LZ4PAR_WPE_LZ4)))
#else
#define LZ4PAR_OCC_LZ4 LZ4PAR_OCC
#endif

template <bool SN>
__device__ __forceinline__ void lz4par_body(Smem &s, int codec, const uint8_t *__restrict__ src,
                                            uint8_t *__restrict__ dst,
                                            const strom_decomp_desc *__restrict__ desc,
                                            uint32_t nstreams, int32_t *status) {
  const uint32_t t = threadIdx.x;
  LP_INIT();
  for (uint32_t b = blockIdx.x; b < nstreams; b += gridDim.x) {
    const strom_decomp_desc d = desc[b];
    Ctx c{src + d.src_off, dst + d.dst_off, d.src_len, d.dst_len};
    if (t == 0) st_header(s, c, codec);
    __syncthreads();
    for (;;) {
      if (t == 0 && s.mode != kModeDone) st_block(s, c);
      __syncthreads();
      if (s.mode == kModeDone || s.err) break;
      LP_MARK(kLpHdr);
      if (s.braw) {
        const uint64_t n = s.bend - s.bstart;
        if ((uint64_t)s.op + n > c.cap) {
          if (t == 0) s.err = kErrOverflow;
          __syncthreads();
          break;
        }
        ph_rawcopy(s, c, t);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        if (t == 0) s.op += (uint32_t)n;
        __syncthreads();
        LP_MARK(kLpRaw);
        continue;
      }
      uint32_t ws = s.bstart;
      while (ws < s.bend && !s.err) {
        LP_CNT(kLpNWin);
        if (t == 0) st_window(s, c, ws);
        __syncthreads();
        ph_load(s, c, t);
        __syncthreads();
        LP_MARK(kLpLoad);
        bool walk = s.walk;
      respec:
        ph_spec<SN>(s, c, t, walk);
        __syncthreads();
        LP_MARK(kLpSpec);
        if (SN && !walk) {
          const uint32_t nsl = (s.wend - s.ws + SL - 1) / SL;
          if (t == 0) s.minfix = nsl;
          __syncthreads();
          bool link = t == 0 || t >= nsl || sn_link(s, t, s.ex[t - 1]);
          if (!link) atomicMin(&s.minfix, t);
          __syncthreads();
          for (;;) {
            const uint32_t S = s.minfix;
            if (S >= nsl) break;
            LP_CNT(kLpNRound);
            // entries of the other broken slices, read before anything moves
            const uint32_t e = t > S && !link ? s.ex[t - 1] : 0;
            __syncthreads();               // everyone has read minfix and e
            if (t == 0) s.minfix = nsl;
            if (t == S) s.cov = sn_settle(s, c, t, s.ex[t - 1]);
            __syncthreads();
            const uint32_t cov = s.cov;
            if (t > cov + 1 && !link && e < slice_hi(s, t)) sn_walk(s, c, t, e);
            __syncthreads();
            if (t > cov) {
              link = t >= nsl || sn_link(s, t, s.ex[t - 1]);
              if (!link) atomicMin(&s.minfix, t);
            }
            __syncthreads();
          }
          s.en[t] = t == 0 ? s.ws : s.ex[t - 1];
          __syncthreads();
        } else if (NW > 1 && walk) {
          const uint32_t nsl = (s.wend - s.ws + SL - 1) / SL;
          const uint32_t lane = t & 63, wave = t >> 6;
          bool fixed = false;
          uint32_t mine = wv_map(s, t, nsl, false);
          for (uint32_t r = 1;; ++r) {
            LP_CNT(kLpNRound);
            // inclusive scan of the maps: in the wave by shuffles, then
            // the earlier waves' totals (s.hb is free until the count)
            uint32_t x = mine;
#pragma unroll
            for (uint32_t d = 1; d < 64; d <<= 1) {
              const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
              if (lane >= d) x = wv_compose(x, y);
            }
            if (lane == 63) s.hb[wave] = x;
            if (t == 0) s.minfix = NT;
            __syncthreads();
            for (uint32_t v = wave; v-- > 0;) x = wv_compose(x, s.hb[v]);
            s.ost[t] = x;
            __syncthreads();
            const uint32_t w = t == 0 ? 0u : wv_get(s.ost[t - 1], 0);
            if (t < nsl && !fixed && w >= NW) atomicMin(&s.minfix, t);
            __syncthreads();
            const uint32_t f = s.minfix;
            if (t < nsl && t < f && !fixed) wv_adopt(s, t, w);
            __syncthreads();
            if (f >= nsl) break;
            if (t == f) {
              wv_fix<SN>(s, c, t, s.ex[t - 1]);
              fixed = true;
            }
            __syncthreads();
            if (wv_pass(s, t, f)) fixed = true;
            __syncthreads();
            if (r >= SERIAL_AFTER) {
              if (t == 0) s.cov = serial_worth(s, f) ? 1u : 0u;
              __syncthreads();
              if (s.cov) {
                if (t == 0) ph_serial<SN>(s, c, f + 1, nsl, true);
                __syncthreads();
                break;
              }
            }
            if (fixed) mine = wv_map(s, t, nsl, true);
          }
          s.en[t] = t == 0 ? s.ws : s.ex[t - 1];
          __syncthreads();
        } else {
          const uint32_t nsl = (s.wend - s.ws + SL - 1) / SL;
          for (uint32_t r = 1;; ++r) {
            LP_CNT(kLpNRound);
            const uint32_t ent = ph_entry(s, t);
            if (t == 0) s.minfix = NT;
            __syncthreads();
            const bool changed = ph_fix<SN>(s, c, t, ent);
            if (changed) atomicMin(&s.minfix, t);
            const uint32_t nchg = (uint32_t)__syncthreads_count(changed);
            if (!nchg) break;
            if (NW > 1 && (r == WALK_AFTER || (r == WALK_EARLY && nchg >= NT / 8))) {
              // this window and the stream's next ones go to the walkers
              // (every thread has passed its fix: the count's barrier);
              // early only when the serial walk would not take over
              bool go = r == WALK_AFTER;
              if (!go) {
                if (t == 0) s.cov = serial_worth(s, s.minfix) ? 1u : 0u;
                __syncthreads();
                go = !s.cov;
                __syncthreads();
              }
              if (go) {
                if (t == 0) s.walk = 1;
                walk = true;
                goto respec;
              }
            }
            if (r >= SERIAL_AFTER) {
              // the frontier slice was just re-parsed from a final entry
              if (t == 0) s.cov = serial_worth(s, s.minfix) ? 1u : 0u;
              __syncthreads();
              if (s.cov) {
                if (t == 0) ph_serial<SN>(s, c, s.minfix + 1, nsl, false);
                __syncthreads();
                break;
              }
            }
          }
        }
        LP_MARK(kLpValid);
        {
          const uint32_t ent = s.en[t];
          __syncthreads();
          ph_count<SN>(s, c, t, ent);
        }
        if (WSCAN) {
          // inclusive scan of the slices' output bytes: in the wave by
          // shuffles, then the earlier waves' totals through the pointer
          // batch (free from the end of validation to the fill) — two
          // barriers instead of two per Hillis-Steele step
          const uint32_t lane = t & 63, wave = t >> 6;
          uint32_t x = s.ost[t];
#pragma unroll
          for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
            if (lane >= d) x += y;
          }
          if (lane == 63) s.ptr[wave] = x;
          __syncthreads();                 // the totals and every count's s.err
          for (uint32_t v = 0; v < wave; ++v) x += s.ptr[v];
          s.ost[t] = x;
          if (t == NT - 1) {
            s.total = x;
            if (!s.err && (uint64_t)s.op + x > c.cap) s.err = kErrOverflow;
          }
        } else {
          for (uint32_t dd = 1; dd < NT; dd <<= 1) {
            __syncthreads();
            const uint32_t v = ph_scan_read(s, t, dd);
            __syncthreads();
            ph_scan_write(s, t, v);
          }
          __syncthreads();
          if (t == 0) {
            s.total = s.ost[NT - 1];
            if (!s.err && (uint64_t)s.op + s.total > c.cap) s.err = kErrOverflow;
          }
        }
        __syncthreads();
        LP_MARK(kLpScan);
        if (s.err) break;
        const uint32_t total = s.total;
        for (uint32_t b0 = 0; b0 < total; b0 += OB) {
          LP_CNT(kLpNBatch);
          const uint32_t nb = total - b0 < OB ? total - b0 : OB;
          ph_fill<SN>(s, c, t, b0);
          __syncthreads();
          LP_MARK(kLpFill);
          if (s.err) break;
          ph_expand(s, t, nb);
          __syncthreads();
          LP_MARK(kLpExpand);
          if (ASYNC_DOUBLE) {
            LP_CNT(kLpNDouble);
            ph_double_async(s, t, nb);
            __syncthreads();
          } else {
            bool more;
            do {
              LP_CNT(kLpNDouble);
              more = ph_double(s, t, nb);
            } while (__syncthreads_or(more));
          }
          LP_MARK(kLpDouble);
          Held h;
          ph_resolve(s, c, t, b0, nb, h);
          // the write changes only what the resolve does not read (HBM
          // past the batch start, the head bitmaps) unless there is a ring
          if (HR) __syncthreads();
          LP_MARK(kLpResolve);
          ph_write(s, c, t, b0, nb, h);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __syncthreads();
          LP_MARK(kLpWrite);
        }
        // the next window starts at the last slice's true exit
        const uint32_t last = (s.wend - s.ws + SL - 1) / SL - 1;
        ws = s.ex[last];
        __syncthreads();
        if (t == 0) s.op += total;
        __syncthreads();
      }
      __syncthreads();
      if (s.err) break;
    }
    if (SN) {
      if (t == 0 && !s.err && s.op != s.expect) s.err = kErrFormat;
      __syncthreads();
    }
    if (t == 0) status[b] = s.err ? s.err : (int32_t)s.op;
    __syncthreads();
  }
  LP_FLUSH();
}

__global__ __launch_bounds__(NT) LZ4PAR_OCC_LZ4 void lz4par_kernel_lz4(
    int codec, const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
    const strom_decomp_desc *__restrict__ desc, uint32_t nstreams, int32_t *status) {
  __shared__ __attribute__((aligned(16))) Smem s;
  lz4par_body<false>(s, codec, src, dst, desc, nstreams, status);
}

__global__ __launch_bounds__(NT) LZ4PAR_OCC void lz4par_kernel_snappy(
    int codec, const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
    const strom_decomp_desc *__restrict__ desc, uint32_t nstreams, int32_t *status) {
  __shared__ __attribute__((aligned(16))) Smem s;
  lz4par_body<true>(s, codec, src, dst, desc, nstreams, status);
}

}  // namespace

// Few long LZ4 streams (raw blocks, frames, Arrow IPC buffers): one
// workgroup per stream, parallel parse + pointer-doubling resolve.
extern "C" int LZ4PAR_ENTRY(int codec, const void *d_src, void *d_dst,
                            const strom_decomp_desc *d_desc, uint32_t nstreams,
                            int32_t *d_status, void *stream) {
  if (codec != STROM_CODEC_LZ4 && codec != STROM_CODEC_LZ4_FRAME &&
      codec != STROM_CODEC_LZ4_FRAME_BCS && codec != STROM_CODEC_ARROW_LZ4 &&
      codec != STROM_CODEC_SNAPPY)
    return -22;
  if (!nstreams) return 0;
  const uint32_t grid = nstreams < 65535 ? nstreams : 65535;
  if (codec == STROM_CODEC_SNAPPY)
    hipLaunchKernelGGL(lz4par_kernel_snappy, dim3(grid), dim3(NT), 0, (hipStream_t)stream, codec,
                       (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nstreams, d_status);
  else
    hipLaunchKernelGGL(lz4par_kernel_lz4, dim3(grid), dim3(NT), 0, (hipStream_t)stream, codec,
                       (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nstreams, d_status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

#ifndef LZ4PAR_NO_HOST
#ifdef STROM_DECOMP_PROF
// phase cycle sums of thread 0 of every workgroup (and event counts), zeroed
extern "C" int strom_lz4par_prof(uint64_t *out) {
  unsigned long long h[kLpN] = {0};
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_lz4par_prof), sizeof h) != hipSuccess) return -5;
  unsigned long long z[kLpN] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lz4par_prof), z, sizeof z);
  for (int i = 0; i < kLpN; ++i) out[i] = h[i];
  return kLpN;
}
#endif

// The same phases run thread by thread on the CPU: the algorithm's
// reference (tests/test_codecs_cpu.py), no GPU involved.  Returns decoded
// bytes or a negative error as the kernel's status.
namespace {
template <bool SN>
int lz4par_host(int codec, const uint8_t *src, uint32_t src_len, uint8_t *dst, uint32_t cap,
                uint32_t *stats) {
  using namespace LZ4P_NS;
  static_assert(NT != 256 || PW != 16384 || OB != 4096 || HR != 0 || UB != 16 ||
                    sizeof(Smem) <= 40 * 1024,
                "default geometry: four workgroups per CU (160 KiB LDS)");
  Smem *sp = new Smem;
  Smem &s = *sp;
  Ctx c{src, dst, src_len, cap};
  uint32_t ent[NT];
  bool flag[NT];
  Held *held = new Held[NT];
  uint32_t rounds = 0, fixes = 0, windows = 0, dbl = 0, serial = 0, serial_windows = 0;
  uint32_t walk_windows = 0;
  st_header(s, c, codec);
  for (;;) {
    if (s.mode != kModeDone) st_block(s, c);
    if (s.mode == kModeDone || s.err) break;
    if (s.braw) {
      if ((uint64_t)s.op + (s.bend - s.bstart) > c.cap) {
        s.err = kErrOverflow;
        break;
      }
      for (uint32_t t = 0; t < NT; ++t) ph_rawcopy(s, c, t);
      s.op += s.bend - s.bstart;
      continue;
    }
    uint32_t ws = s.bstart;
    while (ws < s.bend && !s.err) {
      ++windows;
      st_window(s, c, ws);
      for (uint32_t t = 0; t < NT; ++t) ph_load(s, c, t);
      bool walk = s.walk;
    respec:
      for (uint32_t t = 0; t < NT; ++t) ph_spec<SN>(s, c, t, walk);
      if (SN && !walk) {
        const uint32_t nsl = (s.wend - s.ws + SL - 1) / SL;
        for (uint32_t t = 0; t < NT; ++t)
          flag[t] = t == 0 || t >= nsl || sn_link(s, t, s.ex[t - 1]);   // link
        for (;;) {
          uint32_t S = 1;
          while (S < nsl && flag[S]) ++S;
          if (S >= nsl) break;
          ++rounds;
          for (uint32_t t = 0; t < NT; ++t) ent[t] = t > S && !flag[t] ? s.ex[t - 1] : 0;
          const uint32_t cov = sn_settle(s, c, S, s.ex[S - 1]);
          ++fixes;
          for (uint32_t t = cov + 2; t < nsl; ++t)
            if (!flag[t] && ent[t] < slice_hi(s, t)) {
              sn_walk(s, c, t, ent[t]);
              ++fixes;
            }
          for (uint32_t t = cov + 1; t < NT; ++t) flag[t] = t >= nsl || sn_link(s, t, s.ex[t - 1]);
          for (uint32_t t = S; t <= cov; ++t) flag[t] = true;
        }
        for (uint32_t t = 0; t < NT; ++t) s.en[t] = t == 0 ? s.ws : s.ex[t - 1];
      } else if (NW > 1 && walk) {
        ++walk_windows;
        const uint32_t nsl = (s.wend - s.ws + SL - 1) / SL;
        uint32_t mp[NT];
        for (uint32_t t = 0; t < NT; ++t) {
          flag[t] = false;                      // fixed
          mp[t] = wv_map(s, t, nsl, false);
        }
        for (uint32_t r = 1;; ++r) {
          ++rounds;
          uint32_t x = 0, f = NT;
          for (uint32_t t = 0; t < NT; ++t) {   // ent[t]: slice t's walker
            ent[t] = t == 0 ? 0u : wv_get(x, 0);
            x = t == 0 ? mp[0] : wv_compose(mp[t], x);
            if (t < nsl && !flag[t] && ent[t] >= NW && f == NT) f = t;
          }
          for (uint32_t t = 0; t < nsl && t < f; ++t)
            if (!flag[t]) wv_adopt(s, t, ent[t]);
          if (f >= nsl) break;
          ++fixes;
          wv_fix<SN>(s, c, f, s.ex[f - 1]);
          flag[f] = true;
          for (uint32_t t = f + 1; t < NT; ++t)
            if (wv_pass(s, t, f)) flag[t] = true;
          if (r >= SERIAL_AFTER && serial_worth(s, f)) {
            serial += ph_serial<SN>(s, c, f + 1, nsl, true);
            ++serial_windows;
            break;
          }
          for (uint32_t t = 0; t < NT; ++t)
            if (flag[t]) mp[t] = wv_map(s, t, nsl, true);
        }
        for (uint32_t t = 0; t < NT; ++t) s.en[t] = t == 0 ? s.ws : s.ex[t - 1];
      } else {
        const uint32_t nsl = (s.wend - s.ws + SL - 1) / SL;
        for (uint32_t r = 1;; ++r) {
          ++rounds;
          for (uint32_t t = 0; t < NT; ++t) ent[t] = ph_entry(s, t);
          uint32_t nchg = 0, first = NT;
          for (uint32_t t = 0; t < NT; ++t) {
            flag[t] = ph_fix<SN>(s, c, t, ent[t]);
            nchg += flag[t];
            if (flag[t] && t < first) first = t;
          }
          fixes += nchg;
          if (!nchg) break;
          if (NW > 1 && (r == WALK_AFTER || (r == WALK_EARLY && nchg >= NT / 8 &&
                                             !serial_worth(s, first)))) {
            s.walk = 1;
            walk = true;
            goto respec;
          }
          if (r >= SERIAL_AFTER && serial_worth(s, first)) {
            serial += ph_serial<SN>(s, c, first + 1, nsl, false);
            ++serial_windows;
            break;
          }
        }
      }
      for (uint32_t t = 0; t < NT; ++t) ent[t] = s.en[t];
      for (uint32_t t = 0; t < NT; ++t) ph_count<SN>(s, c, t, ent[t]);
      for (uint32_t dd = 1; dd < NT; dd <<= 1) {
        for (uint32_t t = 0; t < NT; ++t) ent[t] = ph_scan_read(s, t, dd);
        for (uint32_t t = 0; t < NT; ++t) ph_scan_write(s, t, ent[t]);
      }
      s.total = s.ost[NT - 1];
      if (!s.err && (uint64_t)s.op + s.total > c.cap) s.err = kErrOverflow;
      if (s.err) break;
      for (uint32_t b0 = 0; b0 < s.total; b0 += OB) {
        const uint32_t nb = s.total - b0 < OB ? s.total - b0 : OB;
        for (uint32_t t = 0; t < NT; ++t) ph_fill<SN>(s, c, t, b0);
        if (s.err) break;
        for (uint32_t t = 0; t < NT; ++t) ph_expand(s, t, nb);
        bool any;
        do {
          ++dbl;
          any = false;
          for (uint32_t t = 0; t < NT; ++t) any |= ph_double(s, t, nb);
        } while (any);
        for (uint32_t t = 0; t < NT; ++t) ph_resolve(s, c, t, b0, nb, held[t]);
        for (uint32_t t = 0; t < NT; ++t) ph_write(s, c, t, b0, nb, held[t]);
      }
      const uint32_t last = (s.wend - s.ws + SL - 1) / SL - 1;
      ws = s.ex[last];
      s.op += s.total;
    }
    if (s.err) break;
  }
  if (stats) {
    stats[0] = windows;
    stats[1] = rounds;
    stats[2] = fixes;
    stats[3] = dbl;
    stats[4] = serial_windows;
    stats[5] = serial;
    stats[6] = walk_windows;
  }
  if (!s.err && s.expect != 0xffffffffu && s.op != s.expect) s.err = kErrFormat;
  const int r = s.err ? s.err : (int)s.op;
  delete sp;
  delete[] held;
  return r;
}
}  // namespace

extern "C" int strom_lz4par_host(int codec, const uint8_t *src, uint32_t src_len, uint8_t *dst,
                                 uint32_t cap, uint32_t *stats) {
  return codec == STROM_CODEC_SNAPPY ? lz4par_host<true>(codec, src, src_len, dst, cap, stats)
                                     : lz4par_host<false>(codec, src, src_len, dst, cap, stats);
}
#endif  // LZ4PAR_NO_HOST
