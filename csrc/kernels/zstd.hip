// zstd.hip — Zstandard (RFC 8878) decode on CDNA4, for Arrow IPC buffers
// compressed with ZSTD (BodyCompression codec 1: i64 length prefix + one
// zstd frame per buffer — the other Arrow IPC codec next to LZ4_FRAME,
// lz4par.hip).  Not in the reference (the columnar decode path
// is north-star work); it widens BASELINE config 5 to ZSTD-written files.
//
// One wavefront (workgroup of 64) per stream, up to 9 streams per CU (the
// serial entropy stage is latency-bound, so throughput follows the streams
// in flight: the LDS is phase-shared to 16.5 KB per stream).  A compressed
// block is entropy-decoded serially and executed in parallel:
//
//  1. literals: the Huffman table (FSE-coded or direct weights) is built in
//     LDS; the 1 or 4 literal bitstreams are decoded by lanes 0..3 at once,
//     LSYM symbols per stream per round (four per container check), each
//     stream read from its own LDS window that the whole wave refills
//     between rounds; decoded literals are staged in LDS and copied to the
//     stream's scratch slot in HBM, coalesced.  Raw / RLE literals are read
//     in place.
//  2. sequences: LL / OF / ML FSE tables (predefined, RLE, compressed or
//     repeated) in LDS with the code baselines folded into the entries; the
//     wave decodes up to SEQN sequences of the backward bitstream from an
//     LDS window (refilled by the wave per chunk) in a branch-free loop —
//     every lane computes, lane i % 64 keeps entry i in registers — with
//     two bit extractions per sequence, select-based repeat offsets and
//     running output / literal positions, so no scan is needed.
//  3. execution, all 64 lanes: the chunk's output is produced in batches of
//     OB bytes — a source pointer per byte (literal index; stored output
//     before the batch; or an earlier byte of the batch), pointer doubling
//     until every pointer is a literal or stored byte (log2 of the longest
//     in-batch chain), one gather per byte, coalesced byte stores.  Stored
//     output and scratch literals are read back with plain loads after the
//     workgroup release fence + barrier that ended their writes (the
//     workgroup's waves share the CU's L1).
//
// The phases are plain functions of (shared state, lane); the kernel runs
// them with barriers between, strom_zstd_host() runs the SAME functions
// lane by lane on the CPU (tests/test_codecs_cpu.py pins it against
// pyarrow's zstd frames at several levels).  Raw / RLE blocks, skippable
// frames, several frames per stream, the frame content size and the Arrow
// length prefix are checked; dictionaries are refused (Arrow writes none);
// a frame's content checksum, when present, is verified (XXH64, -5).
#include <hip/hip_runtime.h>

#include <cstddef>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <type_traits>

#include "strom/strom.h"

// everything inlines into the kernel: an outlined phase would reach LDS
// through generic pointers
#define HD __host__ __device__ inline __attribute__((always_inline))

// host debug builds (-DZS_DEBUG): report the line of the first failed check
#if defined(ZS_DEBUG) && !defined(__HIP_DEVICE_COMPILE__)
#include <cstdio>
#define ZF(v) (fprintf(stderr, "zstd: check failed at line %d\n", __LINE__), (v))
#else
#define ZF(v) (v)
#endif

// internal linkage throughout: the profiled build (libstrom_zstdprof.so) is
// loaded next to libstrom.so, and exported kernel stubs / statics would
// interpose across the two
namespace zs {
namespace {

constexpr uint32_t NT = 64;              // one wave per stream
#ifndef ZS_SEQN
#define ZS_SEQN 128
#endif
#ifndef ZS_WPE       // the occupancy target given to the register allocator
#define ZS_WPE 2
#endif
#ifndef ZS_LITDIRECT  // 1: a literals-only block's literals decode straight into the output
#define ZS_LITDIRECT 1
#endif
#ifndef ZS_WZERO      // 1: a container fill zeroes the bits below the stream start
#define ZS_WZERO 0
#endif
#ifndef ZS_OB
#define ZS_OB 1024
#endif
constexpr uint32_t SEQN = ZS_SEQN;       // sequences per decode chunk
constexpr uint32_t OB = ZS_OB;           // output bytes per resolve batch
constexpr uint32_t EPT = OB / NT;        // batch entries per lane (strided)
constexpr uint32_t SWIN = (SEQN * 89 / 8 + 24 + 63) / 64 * 64;   // sequence bitstream window: SEQN x <= 89 bits
constexpr uint32_t LSYM = 256;           // literal symbols per stream per round
constexpr uint32_t LWIN = 384;           // literal stream window: LSYM x <= 11 bits
constexpr uint32_t MAXB = 128u << 10;    // Block_Maximum_Size
constexpr uint32_t SLOT = MAXB;          // literal scratch per resident workgroup
constexpr uint32_t kLit = 0x80000000u;   // pointer tag: literal index
constexpr uint32_t kHist = 0x40000000u;  // pointer tag: stored output position
constexpr uint32_t kTag = kLit | kHist;
constexpr uint32_t kPosMax = 1u << 30;   // outputs below 1 GiB
static_assert(SEQN * 89 / 8 + 24 <= SWIN && LSYM * 11 / 8 + 24 <= LWIN, "windows cover a chunk");

enum : int32_t { kErrFormat = -1, kErrOverflow = -2, kErrDistance = -3, kErrUnsupported = -4,
                 kErrChecksum = -5 };
enum : uint32_t { kFrame = 0, kBlock = 1, kDone = 2, kStored = 3 };
enum : uint32_t { kRaw = 0, kRle = 1, kComp = 2 };
enum : uint32_t { kLitScratch = 0, kLitInput = 1, kLitRle = 2 };
enum : uint32_t { kLL = 0, kOF = 1, kML = 2, kPlain = 3 };
// phase profile slots (-DZS_PROF builds, DevTeam::mark / count)
enum { kZpHdr, kZpCopy, kZpLitLoad, kZpLitDec, kZpSeqLoad, kZpSeqDec, kZpFill, kZpDouble,
       kZpWrite, kZpNChunk, kZpNBatch, kZpNDouble, kZpNLitRound, kZpN };

// Batch pointer index, skewed by one dword per EPT entries: the fill phase
// writes EPT contiguous entries per lane (lane t at t * EPT + k), which
// without the skew puts every 4th lane on one of 4 banks (PMC: 4.0G
// bank-conflict cycles against 4.9G active LDS cycles, profiles/r3/zstd/)
HD constexpr uint32_t PI(uint32_t e) { return e + e / EPT; }

// FSE decoding entry (8 bytes): the state's code folded into baseline +
// extra bits (for Huffman weights: base = the weight), its bit count and
// the next state's base — the wave-uniform sequence loop is bound by
// scalar issue, so per-sequence arithmetic is traded for LDS
struct alignas(8) SeqEnt {   // one ds_read_b64 per lookup
  uint32_t base;
  uint16_t next;
  uint8_t nb;
  uint8_t add;
};

// backward bitstream: bits [0, nbits) of the stream's little-endian value
// are still unread and come out top first; cont holds bits [cbase, cbase+64)
struct BR {
  uint64_t cont;
  int32_t nbits;
  int32_t cbase;
  uint32_t beg;
  uint32_t pad;
};

struct Win {                 // an LDS copy of input bytes [lo, lo + n) at
  uint32_t off;              // byte offset off of Smem (an offset, not a pointer:
  uint32_t lo, n;            // reads through &s keep the LDS address space)
};

struct Ctx {
  const uint8_t *in;
  uint8_t *out;
  uint8_t *lit;              // scratch slot (decoded literals of a block)
  uint32_t len;              // input bytes
  uint32_t cap;              // output capacity
};

// Per-stream LDS, phase-shared so that more streams fit a CU (the decode is
// latency-bound per stream: throughput follows the streams in flight).  A
// block's Huffman table lives in the table area only during its literal
// phase, its FSE tables during its sequence phase; treeless literals and
// repeat-mode tables are rebuilt from the saved descriptions (their input
// positions) instead of being kept.
struct Smem {
  union {
    struct {
      SeqEnt tll[512];
      SeqEnt tml[512];
      SeqEnt tof[256];
    };
    struct {                 // indexed by the next hbits bits: no index scaling,
      uint8_t hsym[2048];    // and the length is one byte load off the chain
      uint8_t hlen[2048];
    };
  };
  union {
    struct {                 // building a table (Huffman weights + FSE counts)
      SeqEnt hwt[64];        //   the Huffman-weight FSE table
      uint8_t hw[256];       //   Huffman weights
      int16_t norm[64];
      uint16_t snext[64];
      uint32_t wrank[16];
    };
    struct {                 // literal phase
      alignas(4) uint8_t lwin[4][LWIN];
      alignas(4) uint8_t lstage[4 * LSYM];   // a round's decoded literals, copied out coalesced
    };
    struct {                 // sequence + execution phase
      alignas(4) uint8_t swin[SWIN];
      uint32_t ost[SEQN + 2];     // chunk entry i: output start (relative to the chunk)
      uint32_t lst[SEQN + 1];     //   literal index of its first literal
      uint32_t sll[SEQN + 1];     //   literal length
      uint32_t soff[SEQN + 1];    //   match offset
      uint32_t ptr[OB + OB / EPT];  // batch pointers, bank-skewed (PI)
    };
  };
  BR lbr[4];
  BR sbr;
  uint32_t lcnt[4], lout[4], lwlo[4], lrn[4];
  uint32_t swlo;
  // stream / frame / block scalars (lane 0 writes, all read after a barrier)
  uint32_t ip, op, fstart, fcs_set, fcs, cksum, state;
  uint32_t rep[3];
  int32_t err;
  uint32_t btype, bsize, bstart, bend, blast;
  uint32_t lit_kind, lit_base, lit_n, lit_used, lit_rle;
  uint32_t lit_direct;        // a literals-only block: literals decode into the output
  uint32_t hbits, nls;
  uint32_t hdesc, hdesc_end;           // the frame's last Huffman tree description
  uint32_t tmode[3], tpos[3], tend[3]; // ... and LL / OF / ML table definitions
  uint32_t nseq, seq_done, st_ll, st_of, st_ml, al_ll, al_of, al_ml;
  uint32_t have_ll, have_of, have_ml;
  uint32_t cn, ctot;
  uint32_t ck_pos, ck_need;  // the frame's content checksum (XXH64 low 32 bits)
  uint64_t xacc[4];
  int64_t expect;            // Arrow length prefix, or -1
};

// ------------------------------------------------------------- constants
// predefined distributions (RFC 8878 3.1.1.3.2.2)
#ifdef __HIP_DEVICE_COMPILE__
#define ZTAB __constant__ static const
#else
#define ZTAB static const
#endif
ZTAB int8_t kNormLL[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                           2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
ZTAB int8_t kNormML[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                           1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                           1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
ZTAB int8_t kNormOF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                           1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// baseline + extra bits of a literal-length / match-length / offset code
// (RFC 8878 3.1.1.3.2.1.1): arithmetic plus packed constants, no tables
// (it runs once per code in the wave-uniform sequence loop)
HD void code_base(uint32_t kind, uint32_t c, uint32_t &base, uint32_t &add) {
  if (kind == kOF) {
    add = c;
    base = 1u << c;
  } else if (kind == kLL) {
    // 16..24: 16/1 18/1 20/1 22/1 24/2 28/2 32/3 40/3 48/4
    const uint32_t i = c - 16;
    const uint32_t mid_add = (uint32_t)(0x433221111ull >> (4 * (i & 15))) & 15;
    const uint64_t b0 = 0x28201C1816141210ull;   // bases of 16..23, one byte each
    const uint32_t mid_base = i < 8 ? (uint32_t)(b0 >> (8 * i)) & 255 : 48;
    add = c < 16 ? 0 : c >= 25 ? c - 19 : mid_add;
    base = c < 16 ? c : c >= 25 ? 1u << (c - 19) : mid_base;
  } else if (kind == kML) {
    // 32..42: 35/1 37/1 39/1 41/1 43/2 47/2 51/3 59/3 67/4 83/4 99/5
    const uint32_t i = c - 32;
    const uint32_t mid_add = (uint32_t)(0x54433221111ull >> (4 * (i & 15))) & 15;
    const uint64_t b0 = 0x3B332F2B29272523ull;   // bases of 32..39
    const uint32_t b1 = 0x00635343u;              // bases of 40..42
    const uint32_t mid_base = i < 8 ? (uint32_t)(b0 >> (8 * i)) & 255 : (b1 >> (8 * ((i - 8) & 3))) & 255;
    add = c < 32 ? 0 : c >= 43 ? c - 36 : mid_add;
    base = c < 32 ? c + 3 : c >= 43 ? (1u << (c - 36)) + 3 : mid_base;
  } else {
    base = c;
    add = 0;
  }
}

// ------------------------------------------------------------- input
HD uint32_t gbyte(const Ctx &c, uint32_t p) { return p < c.len ? c.in[p] : 0u; }

template <class S>
HD const uint8_t *sbytes(const S &s) { return (const uint8_t *)&s; }

template <class S>
HD uint32_t wbyte(const S &s, const Win &w, const Ctx &c, uint32_t p) {
  const uint32_t r = p - w.lo;
  return r < w.n ? sbytes(s)[w.off + r] : gbyte(c, p);
}

HD uint32_t rd16(const Ctx &c, uint32_t p) { return gbyte(c, p) | (gbyte(c, p + 1) << 8); }
HD uint32_t rd32(const Ctx &c, uint32_t p) { return rd16(c, p) | (rd16(c, p + 2) << 16); }

HD uint32_t hibit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }   // v > 0

HD bool br_init(BR &b, const Ctx &c, uint32_t beg, uint32_t len) {
  if (len == 0) return ZF(false);
  const uint32_t last = gbyte(c, beg + len - 1);
  if (last == 0) return ZF(false);          // no end marker
  b.beg = beg;
  b.nbits = (int32_t)(8 * (len - 1) + hibit(last));
  b.cbase = 0x7fffffff;                 // first read fills
  b.cont = 0;
  b.pad = 0;
  return true;
}

template <class S>
HD void br_fill(BR &b, const S &s, const Win &w, const Ctx &c) {
  const int32_t nb = b.nbits > 0 ? b.nbits : 0;
  int32_t base = nb - 57;
  base = base > 0 ? (base + 7) & ~7 : 0;    // >= 50 readable bits after a fill
  const uint32_t p = b.beg + (uint32_t)(base >> 3);
  const uint32_t r = p - w.lo;
  uint64_t v = 0;
  if (r + 12 <= w.n) {
    // inside the LDS window: three aligned dwords and a funnel shift
    // (windows start 4-byte aligned in Smem)
    const uint32_t *d = (const uint32_t *)(sbytes(s) + w.off + (r & ~3u));
    const uint64_t lo = (uint64_t)d[0] | ((uint64_t)d[1] << 32);
    const uint32_t sh = 8 * (r & 3);
    v = sh ? (lo >> sh) | ((uint64_t)d[2] << (64 - sh)) : lo;
  } else {
    for (uint32_t j = 0; j < 8; ++j) v |= (uint64_t)wbyte(s, w, c, p + j) << (8 * j);
  }
  b.cont = v;
  b.cbase = base;
}

// the next k (<= 32) bits without consuming them; past the stream start
// the bits read as zeros (the caller sees nbits < 0 afterwards)
template <class S>
HD uint32_t br_peek(BR &b, const S &s, const Win &w, const Ctx &c, uint32_t k) {
  if (b.nbits - (int32_t)k < b.cbase && b.cbase != 0) br_fill(b, s, w, c);
  const int32_t lo = b.nbits - (int32_t)k - b.cbase;
  const uint64_t m = (1ull << k) - 1;
  if (lo >= 0) return (uint32_t)((b.cont >> lo) & m);
  if (b.nbits <= 0) return 0;
  return (uint32_t)((b.cont << (-lo)) & m);
}

template <class S>
HD uint32_t br_read(BR &b, const S &s, const Win &w, const Ctx &c, uint32_t k) {
  if (k == 0) return 0;
  const uint32_t v = br_peek(b, s, w, c, k);
  b.nbits -= (int32_t)k;
  return v;
}

// Hot loops (literal and sequence chunks): the chunk's LDS window covers
// every byte a fill can touch (win_lo: 8 bytes above the position, a
// chunk's worth below, 16 bytes under the stream start), so a
// fill is three aligned LDS dwords.  The container may start below the
// stream (cbase < 0, those bits zeroed), so an extraction is one shift and
// mask with no branch; the fill offset is clamped into the window so that
// even a corrupt stream cannot read outside it.  br_need(k) makes k <= 56
// bits available, br_take then extracts them.
// bits [off, off + w) of v, w <= 31, off + w <= 32; w = 0 gives 0
HD uint32_t ubfe(uint32_t v, uint32_t off, uint32_t w) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_ubfe(v, off, w);
#else
  return (v >> off) & ((1u << w) - 1);
#endif
}

// the low 32 bits of ({hi, lo} >> sh), sh < 32
HD uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t sh) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
#endif
}

template <class S>
HD void br_wfill(BR &b, const S &s, const Win &w) {
  const int32_t nb = b.nbits > 0 ? b.nbits : 0;
  const int32_t base = (nb - 57) & ~7;             // floor to a byte: 57..64 bits readable
  int32_t r = (int32_t)(b.beg - w.lo) + (base >> 3);
  r = r < 0 ? 0 : r > (int32_t)w.n - 12 ? (int32_t)w.n - 12 : r;
  const uint32_t *d = (const uint32_t *)(sbytes(s) + w.off + ((uint32_t)r & ~3u));
  const uint32_t sh = 8 * ((uint32_t)r & 3);
#if ZS_WZERO
  const uint64_t lo = (uint64_t)d[0] | ((uint64_t)d[1] << 32);
  uint64_t v = sh ? (lo >> sh) | ((uint64_t)d[2] << (64 - sh)) : lo;
  if (base < 0) v = base > -64 ? v & (~0ull << (-base)) : 0;   // bits below the stream: 0
  b.cont = v;
#else
  // two funnel shifts; the bits below a stream's start are whatever
  // bytes precede it in the window: a valid stream never consumes them
  // (lookups past a literal stream's end consume nothing, a block's last
  // sequence reads no state bits, Huffman entries are replicated over the
  // unread low bits), and a malformed one ends with nbits != 0
  const uint32_t d0 = d[0], d1 = d[1], d2 = d[2];
  b.cont = (uint64_t)alignbit(d1, d0, sh) | ((uint64_t)alignbit(d2, d1, sh) << 32);
#endif
  b.cbase = base;
}

template <class S>
HD void br_need(BR &b, const S &s, const Win &w, uint32_t k) {
  if (b.nbits - (int32_t)k < b.cbase) br_wfill(b, s, w);
}

// consume k bits (after br_need(>= k)) and return the container shifted
// so that they are its low bits, unmasked: the caller cuts its fields
// out with ubfe (one v_bfe_u32 each)
HD uint64_t br_take(BR &b, uint32_t k) {
  const uint32_t lo = (uint32_t)(b.nbits - (int32_t)k - b.cbase) & 63;
  b.nbits -= (int32_t)k;
  return b.cont >> lo;
}



// forward bits (table descriptions): bytes [p, end), bit offset from p
struct FR {
  uint32_t p, end, bit;
};

HD uint32_t fr_peek(const Ctx &c, const FR &f, uint32_t k) {   // k <= 24
  const uint32_t q = f.p + (f.bit >> 3);
  uint32_t v = 0;
  for (uint32_t j = 0; j < 4; ++j) v |= (q + j < f.end ? gbyte(c, q + j) : 0u) << (8 * j);
  return (v >> (f.bit & 7)) & ((1u << k) - 1);
}

// ------------------------------------------------------------- FSE tables
// FSE table description (RFC 8878 4.1.1) -> normalized counts
HD bool fse_norm(const Ctx &c, FR &f, int16_t *norm, uint32_t maxsym, uint32_t maxal,
                 uint32_t &nsym, uint32_t &al) {
  const uint32_t limit = (f.end - f.p) * 8;
  al = fr_peek(c, f, 4) + 5;
  f.bit += 4;
  if (al > maxal) return ZF(false);
  int32_t remaining = (1 << al) + 1, threshold = 1 << al;
  uint32_t nbits = al + 1, sym = 0;
  bool prev0 = false;
  while (remaining > 1 && sym <= maxsym) {
    if (prev0) {
      uint32_t n0 = sym;
      while (fr_peek(c, f, 2) == 3) {
        n0 += 3;
        f.bit += 2;
        if (f.bit > limit || n0 > maxsym) return ZF(false);
      }
      n0 += fr_peek(c, f, 2);
      f.bit += 2;
      if (n0 > maxsym) return ZF(false);
      while (sym < n0) norm[sym++] = 0;
    }
    const int32_t max = 2 * threshold - 1 - remaining;
    const uint32_t v = fr_peek(c, f, nbits);
    int32_t count;
    if ((int32_t)(v & (uint32_t)(threshold - 1)) < max) {
      count = (int32_t)(v & (uint32_t)(threshold - 1));
      f.bit += nbits - 1;
    } else {
      count = (int32_t)(v & (uint32_t)(2 * threshold - 1));
      if (count >= threshold) count -= max;
      f.bit += nbits;
    }
    --count;
    remaining -= count < 0 ? -count : count;
    if (remaining < 1) return ZF(false);
    norm[sym++] = (int16_t)count;
    prev0 = count == 0;
    while (remaining < threshold) {
      --nbits;
      threshold >>= 1;
    }
    if (f.bit > limit) return ZF(false);
  }
  if (remaining != 1) return ZF(false);
  nsym = sym;
  f.bit = (f.bit + 7) & ~7u;
  return true;
}

// decoding table from normalized counts (RFC 8878 4.1.1: symbol spread,
// then state numbering)
HD bool fse_build(SeqEnt *tab, const int16_t *norm, uint32_t nsym, uint32_t al, uint32_t kind,
                  uint16_t *snext) {
  const uint32_t size = 1u << al, mask = size - 1;
  uint32_t high = size - 1;
  for (uint32_t s = 0; s < nsym; ++s) {
    if (norm[s] == -1) {
      tab[high--].nb = (uint8_t)s;
      snext[s] = 1;
    } else {
      snext[s] = (uint16_t)norm[s];
    }
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3;
  uint32_t pos = 0;
  for (uint32_t s = 0; s < nsym; ++s)
    for (int32_t i = 0; i < norm[s]; ++i) {
      tab[pos].nb = (uint8_t)s;
      do pos = (pos + step) & mask;
      while (pos > high);
    }
  if (pos != 0) return ZF(false);
  for (uint32_t u = 0; u < size; ++u) {
    const uint32_t s = tab[u].nb;
    const uint32_t nx = snext[s]++;
    const uint32_t nb = al - hibit(nx);
    uint32_t base, add;
    code_base(kind, s, base, add);
    // sequence tables number their states as byte offsets (8-byte entries):
    // a state update is one v_lshl_add and indexes LDS without a shift
    tab[u].next = (uint16_t)(((nx << nb) - size) << (kind == kPlain ? 0 : 3));
    tab[u].nb = (uint8_t)nb;
    tab[u].add = (uint8_t)add;
    tab[u].base = base;
  }
  return true;
}

HD void fse_rle(SeqEnt *tab, uint32_t sym, uint32_t kind) {
  uint32_t base, add;
  code_base(kind, sym, base, add);
  tab[0].base = base;
  tab[0].add = (uint8_t)add;
  tab[0].nb = 0;
  tab[0].next = 0;
}

HD void fse_predef(Smem &s, SeqEnt *tab, uint32_t kind, uint32_t &al) {
  const int8_t *src = kind == kLL ? kNormLL : kind == kML ? kNormML : kNormOF;
  const uint32_t n = kind == kLL ? 36 : kind == kML ? 53 : 29;
  for (uint32_t i = 0; i < n; ++i) s.norm[i] = src[i];
  al = kind == kOF ? 5 : 6;
  fse_build(tab, s.norm, n, al, kind, s.snext);
}

// ------------------------------------------------------------- Huffman
// Huffman tree description (RFC 8878 4.2.1) -> weights hw[0..nw)
template <class S>
HD bool huf_weights(S &s, const Ctx &c, uint32_t p, uint32_t end, uint32_t &used,
                    uint32_t &nw) {
  if (p >= end) return ZF(false);
  const uint32_t hb = gbyte(c, p);
  if (hb >= 128) {
    nw = hb - 127;
    const uint32_t nbytes = (nw + 1) / 2;
    if (p + 1 + nbytes > end) return ZF(false);
    for (uint32_t i = 0; i < nw; ++i) {
      const uint32_t b = gbyte(c, p + 1 + i / 2);
      s.hw[i] = (uint8_t)(i & 1 ? b & 15 : b >> 4);
    }
    used = 1 + nbytes;
    return true;
  }
  if (hb == 0 || p + 1 + hb > end) return ZF(false);
  FR f{p + 1, p + 1 + hb, 0};
  uint32_t nsym, al;
  if (!fse_norm(c, f, s.norm, 12, 6, nsym, al)) return ZF(false);
  SeqEnt *wt = s.hwt;
  if (!fse_build(wt, s.norm, nsym, al, kPlain, s.snext)) return ZF(false);
  const uint32_t bp = f.p + (f.bit >> 3);
  BR b;
  if (bp >= f.end || !br_init(b, c, bp, f.end - bp)) return ZF(false);
  const Win w{0, 0, 0};
  uint32_t s1 = br_read(b, s, w, c, al), s2 = br_read(b, s, w, c, al);
  uint32_t n = 0;
  // two interleaved states until the stream is over-read; then the other
  // state's symbol is the last weight (RFC 8878 4.2.1.2)
  for (;;) {
    if (n + 2 > 255) return ZF(false);
    s.hw[n++] = (uint8_t)wt[s1].base;
    s1 = wt[s1].next + br_read(b, s, w, c, wt[s1].nb);
    if (b.nbits < 0) {
      s.hw[n++] = (uint8_t)wt[s2].base;
      break;
    }
    if (n + 2 > 255) return ZF(false);
    s.hw[n++] = (uint8_t)wt[s2].base;
    s2 = wt[s2].next + br_read(b, s, w, c, wt[s2].nb);
    if (b.nbits < 0) {
      s.hw[n++] = (uint8_t)wt[s1].base;
      break;
    }
  }
  nw = n;
  used = 1 + hb;
  return true;
}

// decode table: entries ordered by weight, then symbol; a weight-w symbol
// covers 2^(w-1) entries and has code length hbits + 1 - w
template <class S>
HD bool huf_build(S &s, uint32_t nw) {
  uint32_t total = 0;
  for (uint32_t i = 0; i < nw; ++i) {
    const uint32_t w = s.hw[i];
    if (w > 11) return ZF(false);
    if (w) total += 1u << (w - 1);
  }
  if (!total) return ZF(false);
  const uint32_t maxb = hibit(total) + 1;
  if (maxb > 11) return ZF(false);
  const uint32_t rest = (1u << maxb) - total;
  if (rest & (rest - 1)) return ZF(false);
  s.hw[nw] = (uint8_t)(hibit(rest) + 1);
  const uint32_t nsym = nw + 1;
  for (uint32_t w = 0; w < 16; ++w) s.wrank[w] = 0;
  for (uint32_t i = 0; i < nsym; ++i) s.wrank[s.hw[i]]++;
  uint32_t pos = 0;
  for (uint32_t w = 1; w <= maxb; ++w) {
    const uint32_t n = s.wrank[w];
    s.wrank[w] = pos;
    pos += n << (w - 1);
  }
  if (pos != (1u << maxb)) return ZF(false);
  for (uint32_t i = 0; i < nsym; ++i) {
    const uint32_t w = s.hw[i];
    if (!w) continue;
    const uint32_t n = 1u << (w - 1), st = s.wrank[w];
    for (uint32_t j = 0; j < n; ++j) {
      s.hsym[st + j] = (uint8_t)i;
      s.hlen[st + j] = (uint8_t)(maxb + 1 - w);
    }
    s.wrank[w] = st + n;
  }
  s.hbits = maxb;
  return true;
}

// ------------------------------------------------------------- lane 0: headers
template <class S>
HD void stream_init(S &s, const Ctx &c, int codec) {
  s.err = 0;
  s.op = 0;
  s.ip = 0;
  s.state = kFrame;
  s.expect = -1;
  s.hbits = 0;
  s.ck_need = 0;
  if (c.cap >= kPosMax || c.len >= kPosMax) {
    s.err = kErrOverflow;
    return;
  }
  if (codec == STROM_CODEC_ARROW_ZSTD) {
    if (c.len < 8) {
      s.err = ZF(kErrFormat);
      return;
    }
    const int64_t pre = (int64_t)((uint64_t)rd32(c, 0) | ((uint64_t)rd32(c, 4) << 32));
    s.ip = 8;
    if (pre == -1) {               // stored uncompressed: one raw unit
      s.state = kStored;
      return;
    }
    if (pre < 0 || pre > (int64_t)c.cap) {
      s.err = pre < 0 ? kErrFormat : kErrOverflow;
      return;
    }
    s.expect = pre;
  }
}

// Parse frame headers (skipping skippable frames) and the next block
// header.  Sets s.state = kDone at the end of the input.
template <class S>
HD void next_block(S &s, const Ctx &c) {
  if (s.state == kStored) {        // Arrow buffer stored uncompressed
    s.state = kBlock;
    s.btype = kRaw;
    s.bstart = 8;
    s.bend = c.len;
    s.bsize = c.len - 8;
    s.blast = 1;
    s.cksum = 0;
    s.fcs_set = 0;
    if ((uint64_t)s.op + s.bsize > c.cap) s.err = kErrOverflow;
    return;
  }
  while (s.state == kFrame) {
    const uint32_t p = s.ip;
    if (p == c.len) {
      s.state = kDone;
      return;
    }
    if (p + 4 > c.len) {
      s.err = ZF(kErrFormat);
      return;
    }
    const uint32_t magic = rd32(c, p);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {   // skippable frame
      const uint64_t n = (uint64_t)p + 8 + rd32(c, p + 4);
      if (p + 8 > c.len || n > c.len) {
        s.err = ZF(kErrFormat);
        return;
      }
      s.ip = (uint32_t)n;
      continue;
    }
    if (magic != 0xFD2FB528u || p + 5 > c.len) {
      s.err = ZF(kErrFormat);
      return;
    }
    const uint32_t fhd = gbyte(c, p + 4);
    if (fhd & 0x08) {              // reserved bit
      s.err = ZF(kErrFormat);
      return;
    }
    const uint32_t fcsf = fhd >> 6, single = (fhd >> 5) & 1, didf = fhd & 3;
    uint32_t q = p + 5 + (single ? 0 : 1);
    const uint32_t dsz = didf == 3 ? 4 : didf;
    uint32_t did = 0;
    for (uint32_t j = 0; j < dsz; ++j) did |= gbyte(c, q + j) << (8 * j);
    q += dsz;
    if (did != 0) {
      s.err = kErrUnsupported;     // dictionaries: Arrow writes none
      return;
    }
    const uint32_t fsz = fcsf == 0 ? single : fcsf == 1 ? 2 : fcsf == 2 ? 4 : 8;
    uint64_t fcs = 0;
    for (uint32_t j = 0; j < fsz; ++j) fcs |= (uint64_t)gbyte(c, q + j) << (8 * j);
    if (fsz == 2) fcs += 256;
    q += fsz;
    if (q > c.len) {
      s.err = ZF(kErrFormat);
      return;
    }
    s.fcs_set = fsz != 0;
    if (s.fcs_set && (uint64_t)s.op + fcs > c.cap) {
      s.err = kErrOverflow;
      return;
    }
    s.fcs = (uint32_t)fcs;
    s.cksum = (fhd >> 2) & 1;
    s.fstart = s.op;
    s.rep[0] = 1;
    s.rep[1] = 4;
    s.rep[2] = 8;
    s.hbits = 0;
    s.have_ll = s.have_of = s.have_ml = 0;
    s.ip = q;
    s.state = kBlock;
  }
  const uint32_t p = s.ip;
  if (p + 3 > c.len) {
    s.err = ZF(kErrFormat);
    return;
  }
  const uint32_t h = gbyte(c, p) | (gbyte(c, p + 1) << 8) | (gbyte(c, p + 2) << 16);
  s.blast = h & 1;
  s.btype = (h >> 1) & 3;
  s.bsize = h >> 3;
  s.bstart = p + 3;
  if (s.btype == 3 || s.bsize > MAXB) {
    s.err = ZF(kErrFormat);
    return;
  }
  const uint64_t in_end = (uint64_t)s.bstart + (s.btype == kRle ? 1 : s.bsize);
  if (in_end > c.len) {
    s.err = ZF(kErrFormat);
    return;
  }
  s.bend = (uint32_t)in_end;
  s.ip = s.bstart;
  if (s.btype != kComp && (uint64_t)s.op + s.bsize > c.cap) s.err = kErrOverflow;
}

// after a block: advance; at the end of a frame skip the checksum and
// check the content size
template <class S>
HD void end_block(S &s, const Ctx &c) {
  s.ip = s.bend;
  if (!s.blast) return;
  if (s.cksum) {
    if (s.ip + 4 > c.len) {
      s.err = ZF(kErrFormat);
      return;
    }
    s.ck_pos = s.ip;               // verified by the xxh phase (run())
    s.ck_need = 1;
    s.ip += 4;
  }
  if (s.fcs_set && s.op - s.fstart != s.fcs) s.err = ZF(kErrFormat);
  s.state = kFrame;                // the next frame, or the end of the input
}

template <class S>
HD bool lit_header(S &s, const Ctx &c) {
  const uint32_t p = s.ip, end = s.bend;
  const uint32_t b0 = gbyte(c, p), type = b0 & 3, sf = (b0 >> 2) & 3;
  s.lit_used = 0;
  s.lit_direct = 0;
  for (uint32_t j = 0; j < 4; ++j) s.lcnt[j] = s.lrn[j] = 0;
  if (type <= 1) {
    uint32_t R, hl;
    if ((sf & 1) == 0) {
      R = b0 >> 3;
      hl = 1;
    } else if (sf == 1) {
      R = (b0 >> 4) + (gbyte(c, p + 1) << 4);
      hl = 2;
    } else {
      R = (b0 >> 4) + (gbyte(c, p + 1) << 4) + (gbyte(c, p + 2) << 12);
      hl = 3;
    }
    if (R > MAXB) return ZF(false);
    s.lit_n = R;
    if (type == 0) {
      if ((uint64_t)p + hl + R > end) return ZF(false);
      s.lit_kind = kLitInput;
      s.lit_base = p + hl;
      s.ip = p + hl + R;
    } else {
      if (p + hl + 1 > end) return ZF(false);
      s.lit_kind = kLitRle;
      s.lit_rle = gbyte(c, p + hl);
      s.ip = p + hl + 1;
    }
    return true;
  }
  const uint32_t hl = sf <= 1 ? 3 : sf == 2 ? 4 : 5, bits = sf <= 1 ? 10 : sf == 2 ? 14 : 18;
  uint64_t h = 0;
  for (uint32_t j = 0; j < hl; ++j) h |= (uint64_t)gbyte(c, p + j) << (8 * j);
  const uint32_t R = (uint32_t)(h >> 4) & ((1u << bits) - 1);
  const uint32_t C = (uint32_t)(h >> (4 + bits)) & ((1u << bits) - 1);
  if (R > MAXB || (uint64_t)p + hl + C > end) return ZF(false);
  uint32_t d = p + hl;
  const uint32_t dend = d + C;
  if (type == 2) {
    uint32_t used, nw;
    if (!huf_weights(s, c, d, dend, used, nw) || !huf_build(s, nw)) return ZF(false);
    s.hdesc = d;
    s.hdesc_end = dend;
    d += used;
  } else {
    // treeless: the frame's previous table, rebuilt from its description
    // (the table area held this frame's FSE tables since)
    uint32_t used, nw;
    if (!s.hbits || !huf_weights(s, c, s.hdesc, s.hdesc_end, used, nw) || !huf_build(s, nw))
      return ZF(false);
  }
  s.nls = sf == 0 ? 1 : 4;
  if (s.nls == 1) {
    if (!br_init(s.lbr[0], c, d, dend - d)) return ZF(false);
    s.lcnt[0] = R;
    s.lout[0] = 0;
  } else {
    if (d + 6 > dend) return ZF(false);
    const uint32_t l1 = rd16(c, d), l2 = rd16(c, d + 2), l3 = rd16(c, d + 4);
    d += 6;
    const uint32_t tot = dend - d;
    if (l1 + l2 + l3 >= tot) return ZF(false);
    const uint32_t seg = (R + 3) / 4;
    if (3 * seg > R) return ZF(false);
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t lj = j == 0 ? l1 : j == 1 ? l2 : j == 2 ? l3 : tot - l1 - l2 - l3;
      if (!br_init(s.lbr[j], c, d, lj)) return ZF(false);
      d += lj;
      s.lout[j] = j * seg;
      s.lcnt[j] = j < 3 ? seg : R - 3 * seg;
    }
  }
  s.lit_kind = kLitScratch;
  s.lit_n = R;
  s.ip = dend;
  // Number_of_Sequences = 0 as the block's last byte (an incompressible
  // column's blocks): the literals are the block's output, so they are
  // flushed straight into it and the block has no execution phase
  s.lit_direct = ZS_LITDIRECT && dend + 1 == end && gbyte(c, dend) == 0 &&
                 (uint64_t)s.op + R <= c.cap;
  return true;
}

// One of the LL / OF / ML tables.  Every block with sequences builds all
// three (its literal phase reused the table area); a repeat-mode table is
// rebuilt from the frame's saved definition of that table.
HD bool seq_table(Smem &s, const Ctx &c, uint32_t mode, uint32_t kind, uint32_t &p,
                  uint32_t end, SeqEnt *tab, uint32_t &al, uint32_t &have) {
  const uint32_t maxsym = kind == kLL ? 35 : kind == kML ? 52 : 31;
  const uint32_t maxal = kind == kOF ? 8 : 9;
  const bool repeat = mode == 3;
  if (repeat && !have) return ZF(false);
  const uint32_t m = repeat ? s.tmode[kind] : mode;
  const uint32_t q0 = repeat ? s.tpos[kind] : p;
  const uint32_t qend = repeat ? s.tend[kind] : end;
  uint32_t q = q0;
  if (m == 0) {
    fse_predef(s, tab, kind, al);
  } else if (m == 1) {
    if (q >= qend) return ZF(false);
    const uint32_t sym = gbyte(c, q++);
    if (sym > maxsym) return ZF(false);
    fse_rle(tab, sym, kind);
    al = 0;
  } else {
    FR f{q, qend, 0};
    uint32_t nsym;
    if (!fse_norm(c, f, s.norm, maxsym, maxal, nsym, al)) return ZF(false);
    if (!fse_build(tab, s.norm, nsym, al, kind, s.snext)) return ZF(false);
    q += f.bit >> 3;
  }
  if (!repeat) {
    s.tmode[kind] = m;
    s.tpos[kind] = q0;
    s.tend[kind] = end;
    p = q;
  }
  have = 1;
  return true;
}

HD bool seq_header(Smem &s, const Ctx &c) {
  uint32_t p = s.ip;
  const uint32_t end = s.bend;
  if (p >= end) return ZF(false);
  const uint32_t b0 = gbyte(c, p);
  uint32_t n;
  if (b0 == 0) {
    s.nseq = 0;
    s.seq_done = 0;
    return p + 1 == end ? true : ZF(false);
  }
  if (b0 < 128) {
    n = b0;
    p += 1;
  } else if (b0 < 255) {
    n = ((b0 - 128) << 8) + gbyte(c, p + 1);
    p += 2;
  } else {
    n = gbyte(c, p + 1) + (gbyte(c, p + 2) << 8) + 0x7F00;
    p += 3;
  }
  if (p >= end) return ZF(false);
  const uint32_t modes = gbyte(c, p++);
  if (modes & 3) return ZF(false);
  if (!seq_table(s, c, modes >> 6, kLL, p, end, s.tll, s.al_ll, s.have_ll) ||
      !seq_table(s, c, (modes >> 4) & 3, kOF, p, end, s.tof, s.al_of, s.have_of) ||
      !seq_table(s, c, (modes >> 2) & 3, kML, p, end, s.tml, s.al_ml, s.have_ml))
    return ZF(false);
  if (p >= end || !br_init(s.sbr, c, p, end - p)) return ZF(false);
  const Win w{0, 0, 0};
  s.st_ll = br_read(s.sbr, s, w, c, s.al_ll) << 3;   // byte offsets
  s.st_of = br_read(s.sbr, s, w, c, s.al_of) << 3;
  s.st_ml = br_read(s.sbr, s, w, c, s.al_ml) << 3;
  s.nseq = n;
  s.seq_done = 0;
  return s.sbr.nbits >= 0 ? true : ZF(false);
}

// ------------------------------------------------------------- phases
// window origin of a backward stream: its top 8 bytes above the current
// position (a fill reads up to 12 bytes from 57-64 bits below it), the
// chunk's reads below, and at least 16 bytes under the stream start
HD uint32_t win_lo(const BR &b, uint32_t wsize) {
  const int32_t nb = b.nbits > 0 ? b.nbits : 0;
  const int32_t back = (nb >> 3) + 8 - (int32_t)wsize;
  return b.beg + (uint32_t)(back > -16 ? back : -16);
}

// (1) literal windows: lane t copies every NT-th byte of each stream window
HD void lit_load(Smem &s, const Ctx &c, uint32_t t) {
  for (uint32_t j = 0; j < s.nls; ++j) {
    if (!s.lcnt[j]) continue;
    const uint32_t lo = s.lwlo[j];
    uint8_t r[LWIN / NT];
#pragma unroll
    for (uint32_t k = 0; k < LWIN / NT; ++k) r[k] = (uint8_t)gbyte(c, lo + t + k * NT);
#pragma unroll
    for (uint32_t k = 0; k < LWIN / NT; ++k) s.lwin[j][t + k * NT] = r[k];
  }
}

// (1) up to LSYM symbols of literal stream j
HD void lit_chunk(Smem &s, const Ctx &c, uint32_t j) {
  const uint32_t left = s.lcnt[j];
  if (!left) return;
  BR b = s.lbr[j];
  const Win w{(uint32_t)offsetof(Smem, lwin) + j * LWIN, s.lwlo[j], LWIN};
  const uint32_t n = left < LSYM ? left : LSYM, mb = s.hbits;
  uint8_t *stage = s.lstage + j * LSYM;
  // four symbols per container check (4 x 11 <= 56 readable bits): the
  // lanes' refills fall on the same iterations far more often, and three
  // of four lookups carry no check at all
  // and one dword store of the four; the last, partial group's lookups
  // past the stream's end consume nothing (their bytes are never flushed)
  const uint32_t nf = n & ~3u;
  for (uint32_t k = 0; k < nf; k += 4) {
    br_need(b, s, w, 4 * mb);
    uint32_t word = 0;
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const uint32_t lo = (uint32_t)(b.nbits - (int32_t)mb - b.cbase) & 63;
      const uint32_t x = ubfe((uint32_t)(b.cont >> lo), 0, mb);
      b.nbits -= (int32_t)s.hlen[x];
      word |= (uint32_t)s.hsym[x] << (8 * g);
    }
    *(uint32_t *)(stage + k) = word;
  }
  if (nf < n) {
    br_need(b, s, w, 4 * mb);
    uint32_t word = 0;
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const uint32_t lo = (uint32_t)(b.nbits - (int32_t)mb - b.cbase) & 63;
      const uint32_t x = ubfe((uint32_t)(b.cont >> lo), 0, mb);
      b.nbits -= nf + g < n ? (int32_t)s.hlen[x] : 0;
      word |= (uint32_t)s.hsym[x] << (8 * g);
    }
    *(uint32_t *)(stage + nf) = word;
  }
  s.lrn[j] = n;
  s.lcnt[j] = left - n;
  s.lbr[j] = b;
  if (left == n && b.nbits != 0) s.err = ZF(kErrFormat);   // a stream ends exactly
}

// (1) the round's staged literals -> the scratch slot (lane-strided)
HD void lit_flush(Smem &s, const Ctx &c, uint32_t t) {
  uint8_t *dst = s.lit_direct ? c.out + s.op : c.lit;
  for (uint32_t j = 0; j < s.nls; ++j) {
    const uint32_t n = s.lrn[j], o = s.lout[j];
    for (uint32_t i = t; i < n; i += NT) dst[o + i] = s.lstage[j * LSYM + i];
  }
}

// (2) sequence window: lane t copies every NT-th byte
HD void seq_load(Smem &s, const Ctx &c, uint32_t t) {
  const uint32_t lo = s.swlo;
  uint8_t r[SWIN / NT];
#pragma unroll
  for (uint32_t k = 0; k < SWIN / NT; ++k) r[k] = (uint8_t)gbyte(c, lo + t + k * NT);
#pragma unroll
  for (uint32_t k = 0; k < SWIN / NT; ++k) s.swin[t + k * NT] = r[k];
}

// one FSE entry as a single 64-bit LDS load (a field-wise copy splits it)
HD SeqEnt ld_ent(const SeqEnt *tab, uint32_t off) {   // off: state x 8
  const uint64_t v = *(const uint64_t *)((const uint8_t *)tab + off);
  SeqEnt e;
  e.base = (uint32_t)v;
  e.next = (uint16_t)(v >> 32);
  e.nb = (uint8_t)(v >> 48);
  e.add = (uint8_t)(v >> 56);
  return e;
}

// (2) up to SEQN sequences -> chunk entries; the block's last chunk also
// gets the trailing literals as an entry without a match.  Run by every
// lane of the wave on the same values (wave-uniform: scalar registers and
// scalar branches, no exec-mask juggling around a one-lane loop); lane 0
// stores.
//
// SYM: a block decoded ahead of its predecessors (the frame-parallel
// decoder, run_fp): the repeat offsets it starts from are not known yet,
// so they start as symbols — kSym | index << 26 | k meaning "incoming
// repeat offset `index`, minus k" (RFC 8878 3.1.2.5: the only arithmetic on
// a repeat offset is the LL = 0, code 3 "first repeat minus one") — and
// resolve when the block executes (exec_fp).  Offsets are then checked
// against the output there, not here; a new offset >= kPosMax is an error
// at once (it would read as a symbol).
HD bool is_sym(uint32_t off) { return off >= kPosMax; }

template <bool SYM = false>
HD void seq_chunk(Smem &s, const Ctx &c, uint32_t t) {
  const uint32_t left = s.nseq - s.seq_done;
  const uint32_t m = left < SEQN ? left : SEQN;
  BR b = s.sbr;
  const Win w{(uint32_t)offsetof(Smem, swin), s.swlo, SWIN};
  uint32_t sll = s.st_ll, sof = s.st_of, sml = s.st_ml;
  uint32_t r0 = s.rep[0], r1 = s.rep[1], r2 = s.rep[2];
  const uint32_t pos0 = s.op - s.fstart;    // frame output before this chunk
  const uint32_t lit_n = s.lit_n, last = s.nseq - s.seq_done;
  uint32_t n = 0, out = 0, lit = s.lit_used;
  int32_t err = 0;
  // the offset-distance check accumulates into a flag that ends the stream
  // after the chunk (its entries are then never executed); literal and
  // output totals only grow, so their bounds are checked once after it
  bool bad_dist = false;
  // one sequence; MORE (every sequence but a block's last): the three
  // state updates follow its literal-length bits
  auto step = [&](auto more) __attribute__((always_inline)) {
    constexpr bool MORE = decltype(more)::value;
    const SeqEnt eo = ld_ent(s.tof, sof), em = ld_ent(s.tml, sml), el = ld_ent(s.tll, sll);
    // offset + match-length extra bits in one extraction (<= 47 bits)
    br_need(b, s, w, 47);
    const uint64_t x1 = br_take(b, eo.add + em.add);
    const uint32_t ml = em.base + ubfe((uint32_t)x1, 0, em.add);
    const uint32_t ofv = eo.base + ubfe((uint32_t)(x1 >> em.add), 0, eo.add);
    // literal-length extra bits + the three state updates (<= 42 bits)
    br_need(b, s, w, 42);
    const uint32_t nst = MORE ? el.nb + em.nb + eo.nb : 0;
    const uint64_t x2 = br_take(b, el.add + nst);
    const uint32_t ll = el.base + ubfe((uint32_t)(x2 >> nst), 0, el.add);
    if (MORE) {
      const uint32_t y = (uint32_t)x2;      // ll state | ml state | of state, high to low
      sof = eo.next + (ubfe(y, 0, eo.nb) << 3);
      sml = em.next + (ubfe(y, eo.nb, em.nb) << 3);
      sll = el.next + (ubfe(y, eo.nb + em.nb, el.nb) << 3);
    }
    // repeat offsets (RFC 8878 3.1.2.5): the first repeat offset after a
    // literal run is the common case and changes nothing; otherwise k =
    // repeat index, shifted by one when the literal length is 0, k = 3 is
    // "first repeat minus one"
    uint32_t off = r0;
    if (ofv != 1 || ll == 0) {
      const bool isnew = ofv > 3;
      const uint32_t k = ofv - 1 + (ll == 0 ? 1 : 0);
      const uint32_t rep01 = k == 1 ? r1 : r0;
      const uint32_t rep012 = k == 2 ? r2 : rep01;
      const uint32_t rep = k == 3 ? (SYM && is_sym(r0) ? r0 + 1 : r0 - 1) : rep012;
      off = isnew ? ofv - 3 : rep;
      if (SYM) bad_dist |= isnew && is_sym(off);
      const bool shift2 = isnew || k >= 2;
      r2 = shift2 ? r1 : r2;
      r1 = r0;                             // k >= 1 or new here
      r0 = off;
    }
    if (!SYM) bad_dist |= off - 1 >= pos0 + out + ll;  // off == 0 wraps
    // lane 0 stores (the CPU runs the phase once, HostTeam::uni, as t = 0)
    if (t == 0) {
      s.sll[n] = ll;
      s.soff[n] = off;
      s.lst[n] = lit;
      s.ost[n] = out;
    }
    lit += ll;
    out += ll + ml;
    ++n;
  };
  const bool tail = m && m == last;         // the chunk ends the block
  for (uint32_t i = 0, e = tail ? m - 1 : m; i < e; ++i) step(std::true_type{});
  if (tail) step(std::false_type{});
  if (lit > lit_n || out > MAXB) err = ZF(kErrFormat);
  else if (bad_dist) err = ZF(kErrDistance);
  const bool w0 = t == 0;
  if (!err && m == last) {
    if (s.nseq && b.nbits != 0) err = ZF(kErrFormat);
    const uint32_t rest = lit_n - lit;
    if (rest) {
      if (w0) {
        s.sll[n] = rest;
        s.soff[n] = 0;
        s.lst[n] = lit;
        s.ost[n] = out;
      }
      out += rest;
      lit += rest;
      ++n;
    }
  }
  if (!SYM && !err && (uint64_t)s.op + out > c.cap) err = kErrOverflow;
  if (w0) {
    s.seq_done += m;
    s.ost[n] = out;
    s.cn = n;
    s.ctot = out;
    s.lit_used = lit;
    s.sbr = b;
    s.st_ll = sll;
    s.st_of = sof;
    s.st_ml = sml;
    s.rep[0] = r0;
    s.rep[1] = r1;
    s.rep[2] = r2;
    if (err) s.err = err;
  }
}

// chunk entry holding output byte pos (ost strictly increases)
HD uint32_t entry_of(const Smem &s, uint32_t pos) {
  uint32_t lo = 0, hi = s.cn;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s.ost[mid] <= pos) lo = mid;
    else hi = mid;
  }
  return lo;
}

// (3a) source pointer of every byte of the batch [b0, b0 + nb): lane t
// fills the EPT contiguous entries from t * EPT — one binary search for
// the first, then a walk along the chunk entries (the write phase reads
// the pointers strided, so its stores stay coalesced)
HD void ex_fill(Smem &s, uint32_t t, uint32_t b0, uint32_t nb) {
  const uint32_t abs0 = s.op, e0 = t * EPT;
  if (e0 >= nb) return;
  uint32_t i = entry_of(s, b0 + e0);
  uint32_t start = s.ost[i], next = s.ost[i + 1];
  uint32_t ll = s.sll[i], off = s.soff[i], lst = s.lst[i];
  for (uint32_t k = 0; k < EPT; ++k) {
    const uint32_t e = e0 + k;
    if (e >= nb) break;
    const uint32_t pos = b0 + e;
    while (pos >= next) {                  // the next chunk entry (ost strictly increases)
      ++i;
      start = next;
      next = s.ost[i + 1];
      ll = s.sll[i];
      off = s.soff[i];
      lst = s.lst[i];
    }
    const uint32_t r = pos - start;
    uint32_t v;
    if (r < ll) {
      v = kLit | (lst + r);
    } else {
      const uint32_t src = abs0 + pos - off;
      v = src < abs0 + b0 ? (kHist | src) : src - abs0 - b0;
    }
    s.ptr[PI(e)] = v;
  }
}

// (3b) one doubling round; true while some pointer is still in the batch
// (concurrent rounds only ever replace a pointer by one further down its
// chain: any value a lane reads is a valid ancestor)
HD bool ex_double(Smem &s, uint32_t t, uint32_t nb) {
  bool more = false;
  for (uint32_t k = 0; k < EPT; ++k) {
    const uint32_t e = k * NT + t;
    if (e >= nb) break;
    const uint32_t v = s.ptr[PI(e)];
    if (v & kTag) continue;
    const uint32_t x = s.ptr[PI(v)];
    s.ptr[PI(e)] = x;
    more |= !(x & kTag);
  }
  return more;
}

// A byte stored by this workgroup in an earlier phase: visible to a plain
// load after the release fence + barrier that ended that phase — the
// workgroup's waves share the CU's vector L1 (write-through), so no
// L1-bypassing atomic is needed, and plain loads pipeline (EPT per lane in
// flight instead of one atomic round trip each)
HD uint8_t ld_stored(const uint8_t *base, uint32_t pos) { return base[pos]; }

// (3c) gather + store
HD void ex_write(const Smem &s, const Ctx &c, uint32_t t, uint32_t b0, uint32_t nb) {
  const uint32_t o = s.op + b0;
  for (uint32_t k = 0; k < EPT; ++k) {
    const uint32_t e = k * NT + t;
    if (e >= nb) break;
    const uint32_t v = s.ptr[PI(e)], x = v & ~kTag;
    uint8_t y;
    if (v & kLit)
      y = s.lit_kind == kLitInput ? c.in[s.lit_base + x]
        : s.lit_kind == kLitRle ? (uint8_t)s.lit_rle : ld_stored(c.lit, x);
    else
      y = ld_stored(c.out, x);
    c.out[o + e] = y;
  }
}

// raw / RLE block (or a stored Arrow buffer): lane-strided copy
HD void copy_block(const Smem &s, const Ctx &c, uint32_t t) {
  uint8_t *o = c.out + s.op;
  if (s.btype == kRle) {
    const uint8_t v = (uint8_t)gbyte(c, s.bstart);
    for (uint32_t i = t; i < s.bsize; i += NT) o[i] = v;
  } else {
    const uint8_t *in = c.in + s.bstart;
    for (uint32_t i = t; i < s.bsize; i += NT) o[i] = in[i];
  }
}

// ------------------------------------------------------------- XXH64
// The content checksum of a frame (RFC 8878 3.1.1: the low 32 bits of
// XXH64, seed 0, over the frame's decoded bytes): lanes 0..3 each run one
// of the four stripe accumulators over the frame's output, lane 0 merges
// them and the tail.
constexpr uint64_t kP1 = 0x9E3779B185EBCA87ull, kP2 = 0xC2B2AE3D27D4EB4Full,
                   kP3 = 0x165667B19E3779F9ull, kP4 = 0x85EBCA77C2B2AE63ull,
                   kP5 = 0x27D4EB2F165667C5ull;

HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
HD uint64_t xround(uint64_t acc, uint64_t in) { return rotl64(acc + in * kP2, 31) * kP1; }

HD uint64_t rd64(const uint8_t *p) {
  if (((uintptr_t)p & 7) == 0) return *(const uint64_t *)p;
  uint64_t v = 0;
  for (int j = 0; j < 8; ++j) v |= (uint64_t)p[j] << (8 * j);
  return v;
}

HD void xxh_lane(Smem &s, const Ctx &c, uint32_t t) {
  if (t >= 4) return;
  const uint8_t *p = c.out + s.fstart;
  const uint32_t len = s.op - s.fstart, stripes = len / 32;
  uint64_t v = t == 0 ? kP1 + kP2 : t == 1 ? kP2 : t == 2 ? 0 : 0 - kP1;
  for (uint32_t j = 0; j < stripes; ++j) v = xround(v, rd64(p + 32 * j + 8 * t));
  s.xacc[t] = v;
}

HD void xxh_finish(Smem &s, const Ctx &c) {
  const uint8_t *p = c.out + s.fstart;
  const uint32_t len = s.op - s.fstart;
  uint64_t h;
  uint32_t i = 0;
  if (len >= 32) {
    const uint64_t v1 = s.xacc[0], v2 = s.xacc[1], v3 = s.xacc[2], v4 = s.xacc[3];
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = (h ^ xround(0, v1)) * kP1 + kP4;
    h = (h ^ xround(0, v2)) * kP1 + kP4;
    h = (h ^ xround(0, v3)) * kP1 + kP4;
    h = (h ^ xround(0, v4)) * kP1 + kP4;
    i = len / 32 * 32;
  } else {
    h = kP5;
  }
  h += len;
  for (; i + 8 <= len; i += 8) h = rotl64(h ^ xround(0, rd64(p + i)), 27) * kP1 + kP4;
  if (i + 4 <= len) {
    const uint64_t w = (uint64_t)p[i] | ((uint64_t)p[i + 1] << 8) | ((uint64_t)p[i + 2] << 16) |
                       ((uint64_t)p[i + 3] << 24);
    h = rotl64(h ^ (w * kP1), 23) * kP2 + kP3;
    i += 4;
  }
  for (; i < len; ++i) h = rotl64(h ^ (p[i] * kP5), 11) * kP1;
  h ^= h >> 33;
  h *= kP2;
  h ^= h >> 29;
  h *= kP3;
  h ^= h >> 32;
  s.ck_need = 0;
  if ((uint32_t)h != rd32(c, s.ck_pos)) s.err = ZF(kErrChecksum);
}

// ------------------------------------------------------------- driver
template <class TM>
HD void verify_frame(TM &tm, Smem &s, const Ctx &c) {
  tm.fence();                      // the frame's last output stores
  tm.sync();
  tm.each([&](uint32_t t) { xxh_lane(s, c, t); });
  tm.sync();
  tm.one([&] { xxh_finish(s, c); });
  tm.sync();
}

// (3) one chunk's entries, executed: batches of OB output bytes
template <class TM>
HD void exec_chunk(TM &tm, Smem &s, const Ctx &c) {
  const uint32_t total = s.ctot;
  for (uint32_t b0 = 0; b0 < total; b0 += OB) {
    const uint32_t nb = total - b0 < OB ? total - b0 : OB;
    tm.count(kZpNBatch);
    tm.each([&](uint32_t t) { ex_fill(s, t, b0, nb); });
    tm.sync();
    tm.mark(kZpFill);
    while (tm.any([&](uint32_t t) { return ex_double(s, t, nb); })) {
      tm.count(kZpNDouble);
    }
    tm.mark(kZpDouble);
    tm.each([&](uint32_t t) { ex_write(s, c, t, b0, nb); });
    tm.fence();
    tm.sync();
    tm.mark(kZpWrite);
  }
}

// (1) a compressed block's literal section: header, then the Huffman
// rounds into the scratch slot (or, for a literals-only block, into the
// output).  False when the block is done (literals-only) or failed.
template <class TM>
HD bool block_literals(TM &tm, Smem &s, const Ctx &c, bool allow_direct) {
  tm.one([&] {
    if (!lit_header(s, c)) s.err = ZF(kErrFormat);
    if (!allow_direct) s.lit_direct = 0;
  });
  tm.sync();
  tm.mark(kZpHdr);
  if (s.err) return false;
  if (s.lit_kind == kLitScratch) {
    for (;;) {
      tm.each([&](uint32_t t) {
        if (t < s.nls) s.lwlo[t] = win_lo(s.lbr[t], LWIN);
      });
      tm.sync();
      tm.each([&](uint32_t t) { lit_load(s, c, t); });
      tm.sync();
      tm.mark(kZpLitLoad);
      tm.count(kZpNLitRound);
      tm.each([&](uint32_t t) {
        if (t < s.nls) lit_chunk(s, c, t);
      });
      tm.sync();
      tm.each([&](uint32_t t) { lit_flush(s, c, t); });
      tm.sync();
      tm.each([&](uint32_t t) {
        if (t < s.nls) s.lout[t] += s.lrn[t];
      });
      tm.sync();
      tm.mark(kZpLitDec);
      if (s.err || !(s.lcnt[0] | s.lcnt[1] | s.lcnt[2] | s.lcnt[3])) break;
    }
    tm.fence();
    tm.sync();
    if (s.err) return false;
    if (s.lit_direct) {
      tm.one([&] {
        if (!seq_header(s, c)) s.err = ZF(kErrFormat);   // the 0 sequences byte
        s.op += s.lit_n;
      });
      tm.sync();
      return false;
    }
  }
  return true;
}

// One block after next_block() found it, decoded and executed in place
// (the serial path, and block 0 of a frame-parallel group): s.op advances
// by its output; end_block() is the caller's.
template <class TM>
HD void block_body(TM &tm, Smem &s, const Ctx &c) {
  if (s.btype != kComp) {
    tm.each([&](uint32_t t) { copy_block(s, c, t); });
    tm.fence();
    tm.sync();
    tm.one([&] { s.op += s.bsize; });
    tm.sync();
    tm.mark(kZpCopy);
    return;
  }
  if (!block_literals(tm, s, c, true)) return;
  tm.one([&] {
    if (!seq_header(s, c)) s.err = ZF(kErrFormat);
  });
  tm.sync();
  tm.mark(kZpHdr);
  if (s.err) return;
  do {
    tm.one([&] { s.swlo = win_lo(s.sbr, SWIN); });
    tm.sync();
    if (s.nseq) {
      tm.each([&](uint32_t t) { seq_load(s, c, t); });
      tm.sync();
    }
    tm.mark(kZpSeqLoad);
    tm.count(kZpNChunk);
    tm.uni([&](uint32_t t) { seq_chunk(s, c, t); });
    tm.sync();
    tm.mark(kZpSeqDec);
    if (s.err) return;
    exec_chunk(tm, s, c);
    tm.one([&] { s.op += s.ctot; });
    tm.sync();
  } while (s.seq_done < s.nseq);
}

template <class TM>
HD void run(TM &tm, Smem &s, const Ctx &c, int codec) {
  tm.one([&] { stream_init(s, c, codec); });
  tm.sync();
  while (!s.err) {
    tm.one([&] { next_block(s, c); });
    tm.sync();
    tm.mark(kZpHdr);
    if (s.err || s.state == kDone) break;
    block_body(tm, s, c);
    if (s.err) break;
    tm.one([&] { end_block(s, c); });
    tm.sync();
    if (s.ck_need && !s.err) verify_frame(tm, s, c);
  }
  tm.one([&] {
    if (!s.err && s.expect >= 0 && (int64_t)s.op != s.expect) s.err = ZF(kErrFormat);
  });
  tm.sync();
}

// ------------------------------------------------------------- frame-parallel
// The blocks of a frame decode on different waves of one workgroup (NW
// waves per stream).  A compressed block's entropy stages — literal
// Huffman streams, FSE tables and the sequence bitstream — depend only on
// its own bytes, except for the frame's repeat offsets, a treeless
// literal section (the previous Huffman tree) and a repeat-mode FSE table
// (the previous definition).  So, per group of up to NW blocks:
//   prewalk   wave 0, one lane: the group's block headers, and whether any
//             block needs a previous block's tree or table (then the
//             group runs serially on wave 0 instead);
//   decode    wave 0 decodes and executes block 0 in place; wave w > 0
//             decodes block w's literals into its own scratch slot and its
//             sequences (repeat offsets symbolic, seq_chunk<true>) into its
//             own entry buffer in HBM;
//   execute   waves 1.. in block order: the entries come back chunk by
//             chunk, symbolic offsets resolve against the repeat offsets
//             the previous block ended with, every offset is checked
//             against the output written so far, and the chunk executes
//             as in the serial path (history of earlier blocks is in the
//             output, written before the workgroup barrier that ordered
//             the executions).
// Wave 0's Smem holds the frame (op, repeat offsets, table definitions for
// later treeless / repeat-mode blocks).  The same code runs on the CPU,
// wave after wave (strom_zstd_host_fp), as the algorithm's reference.
constexpr uint32_t NWMAX = 8;
constexpr uint32_t kMaxSeq = MAXB / 3;          // a sequence outputs >= 3 bytes
constexpr uint32_t kMaxEnt = kMaxSeq + 2;       // + the trailing literals
constexpr uint32_t kSym = 0xC0000000u;

struct alignas(16) Ent {                        // a decoded sequence (HBM)
  uint32_t ll, off, lst, ost;                   // ost: output start in the block
};

// a block of a group, with the frame's Huffman-tree and FSE-table
// definitions as that block sees them (positions in the input, resolved by
// the prewalk: a treeless / repeat-mode block rebuilds its tables from
// them on whatever wave decodes it)
struct FpDefs {
  uint32_t hbits, hdesc, hdesc_end;
  uint32_t have[3], tmode[3], tpos[3], tend[3];
};

struct FpBlk {
  uint32_t bstart, bend, btype, bsize, blast;
  FpDefs d;
};

// the frame's state while its blocks decode on every wave (wave 0's Smem
// holds it otherwise): output position, repeat offsets, and the latest
// Huffman-tree / FSE-table definitions
struct FpFrame {
  uint32_t op, fstart, rep[3];
  uint32_t hbits, hdesc, hdesc_end, have_ll, have_of, have_ml;
  uint32_t tmode[3], tpos[3], tend[3];
};

struct FpShared {
  FpBlk blk[NWMAX];
  uint32_t nblk, serial, nent[NWMAX], bout[NWMAX];
  int32_t err;
  FpFrame fr;
};

HD void frame_save(FpFrame &f, const Smem &s) {
  f.op = s.op;
  f.fstart = s.fstart;
  for (uint32_t k = 0; k < 3; ++k) {
    f.rep[k] = s.rep[k];
    f.tmode[k] = s.tmode[k];
    f.tpos[k] = s.tpos[k];
    f.tend[k] = s.tend[k];
  }
  f.hbits = s.hbits;
  f.hdesc = s.hdesc;
  f.hdesc_end = s.hdesc_end;
  f.have_ll = s.have_ll;
  f.have_of = s.have_of;
  f.have_ml = s.have_ml;
}

HD void frame_restore(Smem &s, const FpFrame &f) {
  s.op = f.op;
  s.fstart = f.fstart;
  for (uint32_t k = 0; k < 3; ++k) {
    s.rep[k] = f.rep[k];
    s.tmode[k] = f.tmode[k];
    s.tpos[k] = f.tpos[k];
    s.tend[k] = f.tend[k];
  }
  s.hbits = f.hbits;
  s.hdesc = f.hdesc;
  s.hdesc_end = f.hdesc_end;
  s.have_ll = f.have_ll;
  s.have_of = f.have_of;
  s.have_ml = f.have_ml;
}

HD uint32_t sym_resolve(uint32_t v, const uint32_t *rin) {
  if (!is_sym(v)) return v;
  const uint32_t idx = (v >> 26) & 15;
  // selects, not an index: a dynamically indexed array lives in private memory
  const uint32_t r = idx == 0 ? rin[0] : idx == 1 ? rin[1] : rin[2];
  return idx < 3 ? r - (v & 0x3FFFFFFu) : 0u;   // 0: rejected by the distance check
}

// lane 0 of wave 0: the next up to nw block headers of the current frame
// (parsing the frame header first when one starts).  serial = 1 when a
// block needs a predecessor's tree / table, or the stream is stored.
// the definitions block s.bstart.. leaves for its successors: a Huffman
// description (literals type 2) and the LL / OF / ML table definitions of
// its sequence section (the table descriptions are walked with fse_norm to
// find where each ends).  false: a header it cannot follow.
template <class S>
HD bool prewalk_defs(S &s, const Ctx &c, FpDefs &d) {
  const uint32_t p = s.bstart, end = s.bend, b0 = gbyte(c, p), lt = b0 & 3, sf = (b0 >> 2) & 3;
  uint32_t q;
  if (lt <= 1) {
    const uint32_t hl = (sf & 1) == 0 ? 1 : sf == 1 ? 2 : 3;
    const uint32_t R = hl == 1 ? b0 >> 3 : hl == 2 ? (b0 >> 4) + (gbyte(c, p + 1) << 4)
                               : (b0 >> 4) + (gbyte(c, p + 1) << 4) + (gbyte(c, p + 2) << 12);
    q = p + hl + (lt == 0 ? R : 1);
  } else {
    const uint32_t hl = sf <= 1 ? 3 : sf == 2 ? 4 : 5, bits = sf <= 1 ? 10 : sf == 2 ? 14 : 18;
    uint64_t h = 0;
    for (uint32_t j = 0; j < hl; ++j) h |= (uint64_t)gbyte(c, p + j) << (8 * j);
    const uint32_t C = (uint32_t)(h >> (4 + bits)) & ((1u << bits) - 1);
    if (lt == 2) {                                 // a new tree: lit_header's hdesc / hdesc_end
      d.hbits = 1;
      d.hdesc = p + hl;
      d.hdesc_end = p + hl + C;
    } else if (!d.hbits) {
      return false;                                // treeless with no tree before it
    }
    q = p + hl + C;
  }
  if (q >= end) return false;
  const uint32_t n0 = gbyte(c, q);
  if (n0 == 0) return true;                        // no sequences: no tables
  q += n0 < 128 ? 1 : n0 < 255 ? 2 : 3;
  if (q >= end) return false;
  const uint32_t modes = gbyte(c, q++);
  for (uint32_t k = 0; k < 3; ++k) {               // LL, OF, ML (seq_header's order)
    const uint32_t kind = k == 0 ? kLL : k == 1 ? kOF : kML;
    const uint32_t mode = (modes >> (6 - 2 * k)) & 3;
    if (mode == 3) {
      if (!d.have[kind]) return false;
      continue;
    }
    d.tmode[kind] = mode;
    d.tpos[kind] = q;
    d.tend[kind] = end;
    d.have[kind] = 1;
    if (mode == 1) {
      ++q;
    } else if (mode == 2) {
      FR fr{q, end, 0};
      uint32_t nsym, al;
      const uint32_t maxsym = kind == kLL ? 35 : kind == kML ? 52 : 31;
      if (!fse_norm(c, fr, s.norm, maxsym, kind == kOF ? 8 : 9, nsym, al)) return false;
      q += fr.bit >> 3;
    }
  }
  return true;
}

template <class S>
HD void defs_of(FpDefs &d, const S &s) {
  d.hbits = s.hbits ? 1u : 0u;
  d.hdesc = s.hdesc;
  d.hdesc_end = s.hdesc_end;
  d.have[kLL] = s.have_ll;
  d.have[kOF] = s.have_of;
  d.have[kML] = s.have_ml;
  for (uint32_t k = 0; k < 3; ++k) {
    d.tmode[k] = s.tmode[k];
    d.tpos[k] = s.tpos[k];
    d.tend[k] = s.tend[k];
  }
}

HD void prewalk(Smem &s, const Ctx &c, FpShared &f, uint32_t nw) {
  f.nblk = 0;
  f.serial = 0;
  FpDefs d;
  bool fresh = true;                               // definitions not read yet
  for (uint32_t k = 0; k < nw; ++k) {
    next_block(s, c);
    if (s.err || s.state == kDone) break;
    if (fresh) {                                   // the frame's (a new frame reset them)
      defs_of(d, s);
      fresh = false;
    }
    FpBlk &b = f.blk[k];
    b.bstart = s.bstart;
    b.bend = s.bend;
    b.btype = s.btype;
    b.bsize = s.bsize;
    b.blast = s.blast;
    b.d = d;
    if (s.btype == kComp && !prewalk_defs(s, c, d)) {
      // a header the walk cannot follow: the block runs alone on wave 0,
      // whose own decode reports the error
      if (k) break;
      f.serial = 1;
    }
    f.nblk = k + 1;
    if (s.blast) break;
    s.ip = s.bend;                                 // the next block header
  }
  if (!f.nblk || s.err) return;
  // wave 0 decodes the first block from its header fields; the frame's
  // header (fstart, repeat offsets, ...) was parsed here once
  const FpBlk &b = f.blk[0];
  s.bstart = b.bstart;
  s.bend = b.bend;
  s.btype = b.btype;
  s.bsize = b.bsize;
  s.blast = b.blast;
  s.ip = b.bstart;
  s.state = kBlock;
  if (f.nblk == 1) f.serial = 1;                   // nothing to overlap
}

// wave w > 0: decode block f.blk[w] — literals into its slot, sequences
// into its entry buffer (HBM), repeat offsets symbolic
template <class TM>
HD void decode_fp(TM &tm, Smem &s, const Ctx &c, const FpBlk &b, Ent *ent, uint32_t &nent,
                  uint32_t &bout) {
  tm.one([&] {
    s.err = 0;
    s.bstart = b.bstart;
    s.bend = b.bend;
    s.btype = b.btype;
    s.bsize = b.bsize;
    s.blast = b.blast;
    s.ip = b.bstart;
    s.op = 0;                                      // block-relative until it executes
    s.fstart = 0;
    // the definitions this block may refer to (treeless literals,
    // repeat-mode tables), as the prewalk resolved them
    s.hbits = b.d.hbits;
    s.hdesc = b.d.hdesc;
    s.hdesc_end = b.d.hdesc_end;
    s.have_ll = b.d.have[kLL];
    s.have_of = b.d.have[kOF];
    s.have_ml = b.d.have[kML];
    for (uint32_t k = 0; k < 3; ++k) {
      s.tmode[k] = b.d.tmode[k];
      s.tpos[k] = b.d.tpos[k];
      s.tend[k] = b.d.tend[k];
    }
    s.rep[0] = kSym | (0u << 26);
    s.rep[1] = kSym | (1u << 26);
    s.rep[2] = kSym | (2u << 26);
    s.nseq = 0;
    s.seq_done = 0;
  });
  tm.sync();
  nent = 0;
  bout = 0;
  if (b.btype != kComp) {
    bout = b.bsize;
    return;
  }
  if (!block_literals(tm, s, c, false)) return;   // never literals-direct here
  tm.one([&] {
    if (!seq_header(s, c) || s.nseq > kMaxSeq) s.err = ZF(kErrFormat);
  });
  tm.sync();
  if (s.err) return;
  uint32_t n = 0, out = 0;
  do {
    tm.one([&] { s.swlo = win_lo(s.sbr, SWIN); });
    tm.sync();
    if (s.nseq) {
      tm.each([&](uint32_t t) { seq_load(s, c, t); });
      tm.sync();
    }
    tm.uni([&](uint32_t t) { seq_chunk<true>(s, c, t); });
    tm.sync();
    if (s.err) return;
    if (n + s.cn > kMaxEnt) {
      tm.one([&] { s.err = ZF(kErrFormat); });
      tm.sync();
      return;
    }
    const uint32_t cn = s.cn, n0 = n, o0 = out;
    tm.each([&](uint32_t t) {
      for (uint32_t i = t; i < cn; i += NT) {
        Ent e;
        e.ll = s.sll[i];
        e.off = s.soff[i];
        e.lst = s.lst[i];
        e.ost = o0 + s.ost[i];
        ent[n0 + i] = e;
      }
    });
    n += cn;
    out += s.ctot;
    tm.sync();
  } while (s.seq_done < s.nseq);
  tm.fence();
  tm.sync();
  nent = n;
  bout = out;
}

// Block executions of the frame-parallel decoder run on the whole
// workgroup (TN = NW x 64 lanes, batches of TN x EPT output bytes): the
// batch pointers live in the waves' own execution areas, 1024 entries (+
// skew) per wave, idle by then — entry e is sm[e / 1024].ptr[PI(e % 1024)].
HD uint32_t &gptr(Smem *sm, uint32_t e) { return sm[e >> 10].ptr[PI(e & 1023u)]; }

// a group chunk: up to (TN / 64) x SEQN entries, entry i in wave i / SEQN's
// chunk arrays at i % SEQN (idle there by then), its end in `end`
struct GChunk {
  Smem *sm;
  uint32_t m, end;
  HD uint32_t ost(uint32_t i) const { return i >= m ? end : sm[i / SEQN].ost[i % SEQN]; }
  HD uint32_t sll(uint32_t i) const { return sm[i / SEQN].sll[i % SEQN]; }
  HD uint32_t soff(uint32_t i) const { return sm[i / SEQN].soff[i % SEQN]; }
  HD uint32_t lst(uint32_t i) const { return sm[i / SEQN].lst[i % SEQN]; }
  HD uint32_t entry_of(uint32_t pos) const {   // ost strictly increases
    uint32_t lo = 0, hi = m;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (ost(mid) <= pos) lo = mid;
      else hi = mid;
    }
    return lo;
  }
};

HD void gx_fill(const Smem &s, const GChunk &g, uint32_t t, uint32_t b0, uint32_t nb) {
  const uint32_t abs0 = s.op, e0 = t * EPT;
  if (e0 >= nb) return;
  uint32_t i = g.entry_of(b0 + e0);
  uint32_t start = g.ost(i), next = g.ost(i + 1);
  uint32_t ll = g.sll(i), off = g.soff(i), lst = g.lst(i);
  for (uint32_t k = 0; k < EPT; ++k) {
    const uint32_t e = e0 + k;
    if (e >= nb) break;
    const uint32_t pos = b0 + e;
    while (pos >= next) {
      ++i;
      start = next;
      next = g.ost(i + 1);
      ll = g.sll(i);
      off = g.soff(i);
      lst = g.lst(i);
    }
    const uint32_t r = pos - start;
    uint32_t v;
    if (r < ll) {
      v = kLit | (lst + r);
    } else {
      const uint32_t src = abs0 + pos - off;
      v = src < abs0 + b0 ? (kHist | src) : src - abs0 - b0;
    }
    gptr(g.sm, e) = v;
  }
}

HD bool gx_double(Smem *sm, uint32_t t, uint32_t tn, uint32_t nb) {
  bool more = false;
  for (uint32_t k = 0; k < EPT; ++k) {
    const uint32_t e = k * tn + t;
    if (e >= nb) break;
    const uint32_t v = gptr(sm, e);
    if (v & kTag) continue;
    const uint32_t x = gptr(sm, v);
    gptr(sm, e) = x;
    more |= !(x & kTag);
  }
  return more;
}

HD void gx_write(const Smem &s, Smem *sm, const Ctx &c, uint32_t t, uint32_t tn, uint32_t b0,
                 uint32_t nb) {
  const uint32_t o = s.op + b0;
  for (uint32_t k = 0; k < EPT; ++k) {
    const uint32_t e = k * tn + t;
    if (e >= nb) break;
    const uint32_t v = gptr(sm, e), x = v & ~kTag;
    uint8_t y;
    if (v & kLit)
      y = s.lit_kind == kLitInput ? c.in[s.lit_base + x]
        : s.lit_kind == kLitRle ? (uint8_t)s.lit_rle : ld_stored(c.lit, x);
    else
      y = ld_stored(c.out, x);
    c.out[o + e] = y;
  }
}

// the workgroup, in block order: execute block w at the frame's output
// position, resolving its symbolic repeat offsets; the frame state in s0
// (wave 0's Smem) advances.  c: wave w's view (its literal slot).
template <class TM>
HD void exec_fp(TM &tm, Smem *sm, uint32_t w, FpFrame &s0, const Ctx &c, const Ent *ent,
                uint32_t nent, uint32_t bout) {
  Smem &s = sm[w];
  const uint32_t tn = tm.size(), gob = tn * EPT;
  tm.one([&] {
    s.op = s0.op;
    if ((uint64_t)s0.op + bout > c.cap) s.err = kErrOverflow;
  });
  tm.sync();
  if (s.err) return;
  if (s.btype != kComp) {
    tm.each([&](uint32_t t) {
      uint8_t *o = c.out + s.op;
      if (s.btype == kRle) {
        const uint8_t v = (uint8_t)gbyte(c, s.bstart);
        for (uint32_t i = t; i < s.bsize; i += tn) o[i] = v;
      } else {
        const uint8_t *in = c.in + s.bstart;
        for (uint32_t i = t; i < s.bsize; i += tn) o[i] = in[i];
      }
    });
  } else if (s.nseq == 0 && s.lit_kind == kLitScratch) {
    // literals-only: the slot is the block's output
    tm.each([&](uint32_t t) {
      for (uint32_t i = t; i < s.lit_n; i += tn) c.out[s.op + i] = ld_stored(c.lit, i);
    });
  } else {
    const uint32_t rin[3] = {s0.rep[0], s0.rep[1], s0.rep[2]};
    const uint32_t fpos = s0.op - s0.fstart;     // frame output before the block
    // chunks of (tn / 64) x SEQN entries over every wave's chunk arrays:
    // about one batch of output each (the block's ~16k sequences in 32
    // chunks, not 128 of a quarter batch)
    const uint32_t gseq = tn / NT * SEQN;
    for (uint32_t i0 = 0; i0 < nent; i0 += gseq) {
      const uint32_t m = nent - i0 < gseq ? nent - i0 : gseq;
      const uint32_t base = ent[i0].ost;
      const uint32_t end = (i0 + m < nent ? ent[i0 + m].ost : bout) - base;
      tm.each([&](uint32_t t) {
        bool bad = false;
        for (uint32_t i = t; i < m; i += tn) {
          const Ent e = ent[i0 + i];
          const uint32_t off = sym_resolve(e.off, rin);
          // the serial path's check (seq_chunk): a match reaches back at
          // most to the frame start; the trailing-literals entry has no match
          const bool has_match = (i0 + i + 1 < nent ? ent[i0 + i + 1].ost : bout) - e.ost > e.ll;
          bad |= has_match && off - 1 >= fpos + e.ost + e.ll;
          Smem &q = sm[i / SEQN];
          q.sll[i % SEQN] = e.ll;
          q.soff[i % SEQN] = off;
          q.lst[i % SEQN] = e.lst;
          q.ost[i % SEQN] = e.ost - base;
        }
        if (bad) s.err = ZF(kErrDistance);
      });
      tm.sync();
      if (s.err) return;
      const GChunk gc{sm, m, end};
      const uint32_t total = end;
      for (uint32_t b0 = 0; b0 < total; b0 += gob) {
        const uint32_t nb = total - b0 < gob ? total - b0 : gob;
        tm.each([&](uint32_t t) { gx_fill(s, gc, t, b0, nb); });
        tm.sync();
        while (tm.any([&](uint32_t t) { return gx_double(sm, t, tn, nb); })) {
        }
        tm.each([&](uint32_t t) { gx_write(s, sm, c, t, tn, b0, nb); });
        tm.fence();
        tm.sync();
      }
      tm.one([&] { s.op += total; });
      tm.sync();
    }
  }
  tm.fence();
  tm.sync();
  tm.one([&] {
    s0.op += bout;
    if (s.btype == kComp && s.nseq) {
      const uint32_t rin[3] = {s0.rep[0], s0.rep[1], s0.rep[2]};
      s0.rep[0] = sym_resolve(s.rep[0], rin);
      s0.rep[1] = sym_resolve(s.rep[1], rin);
      s0.rep[2] = sym_resolve(s.rep[2], rin);
    }
  });
  tm.sync();
}

// after a parallel group: the blocks' Huffman tree and FSE table
// definitions, in block order, become the frame's (a treeless /
// repeat-mode block of a later group runs alone on wave 0)
HD void inherit_defs(FpFrame &s0, const Smem &s) {
  if (s.btype != kComp) return;
  if (s.hbits && s.lit_kind == kLitScratch) {
    s0.hdesc = s.hdesc;
    s0.hdesc_end = s.hdesc_end;
    s0.hbits = s.hbits;
  }
  if (s.nseq) {
    for (uint32_t k = 0; k < 3; ++k) {
      s0.tmode[k] = s.tmode[k];
      s0.tpos[k] = s.tpos[k];
      s0.tend[k] = s.tend[k];
    }
    s0.have_ll = s0.have_of = s0.have_ml = 1;
  }
}

// G: a workgroup of NW wave teams (DevGroup) or their CPU emulation
// (HostGroup: the waves one after another — their decodes are independent)
// per-wave views of a workgroup's frame-parallel scratch (computed, not
// kept in arrays indexed by the wave: those would live in private memory)
struct FpCtx {
  Ctx c;                     // lit: wave 0's slot
  uint8_t *scr;              // fp_scratch(nw) bytes
  uint32_t nw;
  HD Ctx wave(uint32_t w) const {
    return Ctx{c.in, c.out, scr + (size_t)w * SLOT, c.len, c.cap};
  }
  HD Ent *ent(uint32_t w) const {
    return (Ent *)(scr + (size_t)nw * SLOT + (size_t)w * kMaxEnt * sizeof(Ent));
  }
};

template <class G>
HD void run_fp(G &g, Smem *sm, FpShared &f, const FpCtx &x, int codec) {
  Smem &s0 = sm[0];
  const uint32_t nw = x.nw;
  const Ctx c0 = x.wave(0);
  g.wave(0, [&](auto &tm) {
    tm.one([&] { stream_init(s0, c0, codec); });
    tm.sync();
  });
  g.sync_all();
  while (!s0.err) {
    g.wave(0, [&](auto &tm) {
      tm.one([&] { prewalk(s0, c0, f, nw); });
      tm.sync();
    });
    g.sync_all();
    if (s0.err || !f.nblk) break;
    const uint32_t nb = f.serial ? 1 : f.nblk;
    g.count_group(nb);
    if (f.serial) {
      // one block, decoded and executed in place on wave 0
      g.wave(0, [&](auto &tm) { block_body(tm, s0, c0); });
      g.sync_all();
    } else {
      // every block of the group on its own wave; wave 0's Smem is a block
      // decoder too meanwhile, the frame waits in f.fr
      g.wave(0, [&](auto &tm) {
        tm.one([&] {
          frame_save(f.fr, s0);
          f.err = 0;
        });
        tm.sync();
      });
      g.sync_all();
      g.waves(nb, [&](uint32_t w, auto &tm) {
        decode_fp(tm, sm[w], x.wave(w), f.blk[w], x.ent(w), f.nent[w], f.bout[w]);
      });
      g.sync_all();
      for (uint32_t w = 0; w < nb; ++w) {
        if (sm[w].err) break;                      // its decode failed
        g.all([&](auto &tm) { exec_fp(tm, sm, w, f.fr, x.wave(w), x.ent(w), f.nent[w], f.bout[w]); });
        g.sync_all();
        if (sm[w].err) break;                      // its execution failed
      }
      g.wave(0, [&](auto &tm) {
        tm.one([&] {
          for (uint32_t w = 0; w < nb && !f.err; ++w) f.err = sm[w].err;
          for (uint32_t w = 0; w < nb; ++w) inherit_defs(f.fr, sm[w]);
          frame_restore(s0, f.fr);
          s0.err = f.err;
        });
        tm.sync();
      });
      g.sync_all();
    }
    if (s0.err) break;
    g.wave(0, [&](auto &tm) {
      tm.one([&] {
        const FpBlk &l = f.blk[nb - 1];
        s0.bend = l.bend;
        s0.blast = l.blast;
        end_block(s0, c0);
      });
      tm.sync();
      if (s0.ck_need && !s0.err) verify_frame(tm, s0, c0);
    });
    g.sync_all();
  }
  g.wave(0, [&](auto &tm) {
    tm.one([&] {
      if (!s0.err && s0.expect >= 0 && (int64_t)s0.op != s0.expect) s0.err = ZF(kErrFormat);
    });
    tm.sync();
  });
  g.sync_all();
}

#define DI __device__ inline __attribute__((always_inline))
// -DZS_PROF (libstrom_zstdprof.so): lane-0 cycle stamps per phase summed
// over all workgroups, plus event counts (tools/zstd_bench.py --prof)
#ifdef ZS_PROF
__device__ unsigned long long g_zprof[kZpN];
#endif
struct DevTeam {
#ifdef ZS_PROF
  uint64_t acc[kZpN] = {0};
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  DI void mark(int k) {
    const uint64_t n = __builtin_amdgcn_s_memtime();
    acc[k] += n - t0;
    t0 = n;
  }
  DI void count(int k) { acc[k] += 1; }
  DI void flush() {
    if (threadIdx.x == 0)
      for (int i = 0; i < kZpN; ++i) atomicAdd(&g_zprof[i], (unsigned long long)acc[i]);
  }
#else
  DI void mark(int) {}
  DI void count(int) {}
  DI void flush() {}
#endif
  DI uint32_t size() const { return blockDim.x; }
  DI void sync() { __syncthreads(); }
  DI void fence() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
  template <class F>
  DI void each(F f) { f(threadIdx.x); }
  template <class F>
  DI void one(F f) {
    if (threadIdx.x == 0) f();
  }
  // wave-uniform phase: every lane computes, lane 0 stores
  template <class F>
  DI void uni(F f) { f(threadIdx.x); }
  template <class F>
  DI bool any(F f) { return __syncthreads_or(f(threadIdx.x)); }
};

struct HostTeam {
  uint32_t n = NT;           // lanes (a workgroup-wide team of the frame-parallel decoder: more)
  uint32_t size() const { return n; }
  void mark(int) {}
  void count(int) {}
  void sync() {}
  void fence() {}
  template <class F>
  void each(F f) {
    for (uint32_t t = 0; t < n; ++t) f(t);
  }
  template <class F>
  void one(F f) { f(); }
  template <class F>
  void uni(F f) { f(0); }
  template <class F>
  bool any(F f) {
    bool v = false;
    for (uint32_t t = 0; t < n; ++t) v |= f(t);
    return v;
  }
};

// One wave of a multi-wave workgroup as a team (the frame-parallel
// decoder): its own barrier is a wave barrier with LDS / memory ordering
// at wavefront scope (a wave's LDS operations complete in order); stores
// another wave reads are ordered by the workgroup fence + barrier of
// DevGroup::sync_all.
struct WaveTeam {
  DI uint32_t size() const { return NT; }
  DI uint32_t lane() const { return threadIdx.x & (NT - 1); }
  DI void mark(int) {}
  DI void count(int) {}
  DI void sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  DI void fence() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
  template <class F>
  DI void each(F f) { f(lane()); }
  template <class F>
  DI void one(F f) {
    if (lane() == 0) f();
  }
  template <class F>
  DI void uni(F f) { f(lane()); }
  template <class F>
  DI bool any(F f) {
    const bool v = f(lane());
    sync();
    return __ballot(v) != 0;
  }
};

struct DevGroup {
  WaveTeam tm;
  DI uint32_t wid() const { return threadIdx.x / NT; }
  template <class F>
  DI void wave(uint32_t k, F f) {
    if (wid() == k) f(tm);
  }
  template <class F>
  DI void waves(uint32_t n, F f) {
    if (wid() < n) f(wid(), tm);
  }
  // the whole workgroup as one team (block executions)
  template <class F>
  DI void all(F f) {
    DevTeam t;
    f(t);
  }
  DI void sync_all() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  DI void count_group(uint32_t) {}
};

struct HostGroup {
  HostTeam tm;
  template <class F>
  void wave(uint32_t, F f) { f(tm); }
  template <class F>
  void waves(uint32_t n, F f) {
    for (uint32_t w = 0; w < n; ++w) f(w, tm);
  }
  uint32_t nw = 1;
  template <class F>
  void all(F f) {
    HostTeam t;
    t.n = NT * nw;
    f(t);
  }
  void sync_all() {}
  uint32_t groups = 0, blocks_par = 0;   // groups, and blocks decoded ahead of their turn
  void count_group(uint32_t nb) {
    ++groups;
    blocks_par += nb - 1;
  }
};

// ------------------------------------------------------------- lane-parallel
// The decoders above run a block's serial entropy stages on a whole wave:
// 64 lanes compute the same values, one symbol / sequence at a time, so a
// stream's latency is ~1,000 cycles per sequence and the chip fills only
// with thousands of streams (profiles/r4/zstd: 2,048 val streams at 34.8
// GB/s, VALU-issue-bound).  The lane-parallel ("LP") decoder gives every
// BLOCK its own lanes instead: several blocks share a wave, a block's four
// Huffman literal streams decode on four of its lanes and its sequence
// bitstream on one, each lane walking its own tables and input window in
// LDS.  Launches:
//   walk     one lane per stream: frame + block headers, every block's
//            literal / sequence counts and the Huffman-tree / FSE-table
//            definitions it may refer to (treeless / repeat-mode blocks
//            rebuild them on their own lanes); blocks go to one list,
//            entries are allocated from a pool
//   lit      LPLB blocks per wave (all of a column's blocks at once, in one
//            or two resident rounds): literals decode straight into the
//            stream's OUTPUT buffer, packed at its tail
//   seq      LPSB blocks per wave, one lane each: sequences into 16-byte
//            entries (repeat offsets symbolic, as the frame-parallel
//            decoder's)
//   exec     one workgroup per stream, blocks in order: exec_fp's batches
//            over the entries, gathers split from stores (a literal's tail
//            position is never below its output position — the in-place
//            decompression argument — but a batch may write where a later
//            byte of the same batch reads), symbolic offsets resolved and
//            every distance checked
// Any stream the walk cannot take (several frames, a stored Arrow buffer,
// a header it cannot follow, pool exhausted) or whose LP decode reports an
// error is decoded again by the serial decoder (run()) in the exec launch,
// so statuses and errors are the serial decoder's.
#ifndef ZS_LPB
#define ZS_LPB 4
#endif
constexpr uint32_t LP_LSYM = 128;             // literal symbols per stream per round
constexpr uint32_t LP_LWIN = 256;             // its input window (one dword per lane)
constexpr uint32_t LP_SEQN = 64;              // sequences per round
constexpr uint32_t LP_SWIN = 768;             // its input window (three dwords per lane)
static_assert(LP_LSYM * 11 / 8 + 24 <= LP_LWIN && LP_SEQN * 89 / 8 + 24 <= LP_SWIN, "LP windows");
static_assert(LP_LWIN == 4 * NT && LP_SWIN % (4 * NT) == 0, "LP window loads");

// compact FSE entry (4 bytes, a third of the LDS the 8-byte SeqEnt takes):
// code | bits << 8 | next state base << 16; the code's baseline and extra
// bits come from code_base()
HD uint32_t lp_ent(uint32_t code, uint32_t nb, uint32_t next) { return code | nb << 8 | next << 16; }

// The LP phases keep their input / output pointers in LDS (per block), so
// the compiler no longer sees that they are global: accesses would become
// FLAT, and a flat op counts in lgkmcnt too — every LDS table lookup would
// then wait for the previous literal / entry store.  The hot loops go
// through these global-address-space views instead.
#ifdef __HIP_DEVICE_COMPILE__
#define ZG __attribute__((address_space(1)))
#else
#define ZG
#endif
template <class T>
HD ZG T *zg(T *p) { return (ZG T *)p; }

HD bool fse_build4(uint32_t *tab, const int16_t *norm, uint32_t nsym, uint32_t al,
                   uint16_t *snext) {
  const uint32_t size = 1u << al, mask = size - 1;
  uint32_t high = size - 1;
  for (uint32_t s = 0; s < nsym; ++s) {
    if (norm[s] == -1) {
      tab[high--] = s;
      snext[s] = 1;
    } else {
      snext[s] = (uint16_t)norm[s];
    }
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3;
  uint32_t pos = 0;
  for (uint32_t s = 0; s < nsym; ++s)
    for (int32_t i = 0; i < norm[s]; ++i) {
      tab[pos] = s;
      do pos = (pos + step) & mask;
      while (pos > high);
    }
  if (pos != 0) return ZF(false);
  for (uint32_t u = 0; u < size; ++u) {
    const uint32_t s = tab[u] & 255;
    const uint32_t nx = snext[s]++;
    const uint32_t nb = al - hibit(nx);
    tab[u] = lp_ent(s, nb, (nx << nb) - size);
  }
  return true;
}

// seq_table with compact entries (the same modes and saved definitions)
template <class S>
HD bool seq_table4(S &s, const Ctx &c, uint32_t mode, uint32_t kind, uint32_t &p, uint32_t end,
                   uint32_t *tab, uint32_t &al, uint32_t &have) {
  const uint32_t maxsym = kind == kLL ? 35 : kind == kML ? 52 : 31;
  const uint32_t maxal = kind == kOF ? 8 : 9;
  const bool repeat = mode == 3;
  if (repeat && !have) return ZF(false);
  const uint32_t m = repeat ? s.tmode[kind] : mode;
  const uint32_t q0 = repeat ? s.tpos[kind] : p;
  const uint32_t qend = repeat ? s.tend[kind] : end;
  uint32_t q = q0;
  if (m == 0) {
    const int8_t *src = kind == kLL ? kNormLL : kind == kML ? kNormML : kNormOF;
    const uint32_t n = kind == kLL ? 36 : kind == kML ? 53 : 29;
    for (uint32_t i = 0; i < n; ++i) s.norm[i] = src[i];
    al = kind == kOF ? 5 : 6;
    fse_build4(tab, s.norm, n, al, s.snext);
  } else if (m == 1) {
    if (q >= qend) return ZF(false);
    const uint32_t sym = gbyte(c, q++);
    if (sym > maxsym) return ZF(false);
    tab[0] = lp_ent(sym, 0, 0);
    al = 0;
  } else {
    FR f{q, qend, 0};
    uint32_t nsym;
    if (!fse_norm(c, f, s.norm, maxsym, maxal, nsym, al)) return ZF(false);
    if (!fse_build4(tab, s.norm, nsym, al, s.snext)) return ZF(false);
    q += f.bit >> 3;
  }
  if (!repeat) {
    s.tmode[kind] = m;
    s.tpos[kind] = q0;
    s.tend[kind] = end;
    p = q;
  }
  have = 1;
  return true;
}

// ---- global records (the pool: header, streams, blocks, fallback slots, entries)
struct LpHdr {
  uint32_t nblk;             // blocks listed (may pass the capacity: those streams fall back)
  uint32_t lp_done;          // streams the LP path decoded (the rest: the serial decoder)
  uint64_t ent_used;         // entry bytes allocated
};

enum : uint32_t { kLpDecode = 0, kLpSerial = 1 };

struct LpStream {
  uint32_t first, nblk, mode, fcs_set, fcs, cksum, ck_pos, pad;
  int64_t expect;
};

struct alignas(16) LpBlock {
  // walk
  uint32_t stream, bstart, bend, btype, bsize, blast, active, lit_off;
  FpDefs d;
  uint64_t ent_off;
  // entropy
  uint32_t lit_kind, lit_n, lit_base, lit_rle, sip, nseq, nent, bout;
  uint32_t rep[3];
  int32_t err;
};

// the walk's per-lane state: what stream_init / next_block / prewalk_defs use
struct LpWalk {
  int32_t err;
  uint32_t op, ip, state;
  int64_t expect;
  uint32_t hbits, hdesc, hdesc_end, ck_need, ck_pos, fcs_set, fcs, cksum, fstart;
  uint32_t rep[3];
  uint32_t have_ll, have_of, have_ml, tmode[3], tpos[3], tend[3];
  uint32_t bstart, bend, btype, bsize, blast;
  int16_t norm[64];
};

// a compressed block's regenerated literal count (R), the literal section's
// type and its sequence count, from the two section headers
HD bool lp_sizes(const Ctx &c, uint32_t p, uint32_t end, uint32_t &R, uint32_t &lt,
                 uint32_t &nseq) {
  if (p >= end) return false;
  const uint32_t b0 = gbyte(c, p), sf = (b0 >> 2) & 3;
  lt = b0 & 3;
  uint32_t q;
  if (lt <= 1) {
    const uint32_t hl = (sf & 1) == 0 ? 1 : sf == 1 ? 2 : 3;
    R = hl == 1 ? b0 >> 3 : hl == 2 ? (b0 >> 4) + (gbyte(c, p + 1) << 4)
                          : (b0 >> 4) + (gbyte(c, p + 1) << 4) + (gbyte(c, p + 2) << 12);
    q = p + hl + (lt == 0 ? R : 1);
  } else {
    const uint32_t hl = sf <= 1 ? 3 : sf == 2 ? 4 : 5, bits = sf <= 1 ? 10 : sf == 2 ? 14 : 18;
    uint64_t h = 0;
    for (uint32_t j = 0; j < hl; ++j) h |= (uint64_t)gbyte(c, p + j) << (8 * j);
    R = (uint32_t)(h >> 4) & ((1u << bits) - 1);
    q = p + hl + ((uint32_t)(h >> (4 + bits)) & ((1u << bits) - 1));
  }
  if (R > MAXB || q >= end) return false;
  const uint32_t n0 = gbyte(c, q);
  nseq = n0 < 128 ? n0 : n0 < 255 ? ((n0 - 128) << 8) + gbyte(c, q + 1)
                                  : gbyte(c, q + 1) + (gbyte(c, q + 2) << 8) + 0x7F00;
  return nseq <= kMaxSeq;
}

// One stream's headers.  rec == nullptr: count (blocks, literal bytes
// packed at the output's tail, entries); else fill rec[0..nblk).  false:
// the LP path does not take the stream (the serial decoder will).
// lit_start: where the tail-packed literal regions begin (cap - the first
// pass's lits); ent_base: the stream's entries in the pool.
HD bool lp_walk(LpWalk &s, const Ctx &c, int codec, uint32_t stream, LpBlock *rec,
                uint32_t lit_start, uint64_t ent_base, uint32_t &nblk, uint32_t &lits,
                uint32_t &nent, LpStream &st) {
  stream_init(s, c, codec);
  if (s.err || s.state == kStored) return false;
  nblk = lits = nent = 0;
  uint32_t frames = 0, pos = lit_start;      // tail packing cursor
  FpDefs d{};
  bool fresh = true;
  for (;;) {
    if (s.state == kFrame) {
      if (s.ip == c.len) break;              // end of the input
      if (++frames > 1) return false;        // several frames: the serial decoder
    }
    next_block(s, c);
    if (s.err) return false;
    if (s.state == kDone) break;
    if (fresh) {
      defs_of(d, s);
      fresh = false;
    }
    uint32_t R = 0, lt = 0, nseq = 0;
    LpBlock b{};
    b.stream = stream;
    b.bstart = s.bstart;
    b.bend = s.bend;
    b.btype = s.btype;
    b.bsize = s.bsize;
    b.blast = s.blast;
    b.d = d;
    if (s.btype == kComp) {
      if (!lp_sizes(c, s.bstart, s.bend, R, lt, nseq) || !prewalk_defs(s, c, d)) return false;
      const uint32_t lr = lt >= 2 ? R : 0;   // Huffman literals: a region at the tail
      if (lr > c.cap - lits) return false;
      lits += lr;
      b.active = 1;
      b.lit_off = pos;
      pos += lr;
      b.ent_off = ent_base + (uint64_t)nent * sizeof(Ent);
      nent += nseq + 1;                      // + the trailing literals
    }
    if (rec) rec[nblk] = b;
    ++nblk;
    s.ip = s.bend;
    if (s.blast) {                           // end_block without its output checks
      st.cksum = s.cksum;
      if (s.cksum) {
        if (s.ip + 4 > c.len) return false;
        st.ck_pos = s.ip;
        s.ip += 4;
      }
      st.fcs_set = s.fcs_set;
      st.fcs = s.fcs;
      s.state = kFrame;
    }
  }
  if (frames != 1 || !nblk || s.state != kFrame) return false;
  st.expect = s.expect;
  return true;
}

// ---- entropy: two launches, literal sections then sequence sections, each
// with its own per-block LDS (a block's Huffman table, or its three FSE
// tables) and blocks per wave — the sequence launch keeps 4 waves per CU,
// one per SIMD, where one launch for both held 3.
// literals: LPLB blocks per wave, 64 / LPLB lanes each (one per stream)
#ifndef ZS_LPLB
#define ZS_LPLB ZS_LPB
#endif
#ifndef ZS_LPSB
#define ZS_LPSB 6
#endif
constexpr uint32_t LPLB = ZS_LPLB;
constexpr uint32_t LPLL = NT / LPLB;
static_assert(NT % LPLB == 0 && LPLL >= 4, "LP literal lanes");
constexpr uint32_t LPSB = ZS_LPSB;            // sequences: blocks per wave, block b on lane b
static_assert(LPSB >= 1 && LPSB <= NT, "LP sequence lanes");

struct alignas(16) LpL {                      // a block's literal section
  uint8_t hsym[2048];
  uint8_t hlen[2048];
  union {
    struct {                                  // building the Huffman table
      SeqEnt hwt[64];
      uint8_t hw[256];
      int16_t norm[64];
      uint16_t snext[64];
      uint32_t wrank[16];
    };
    alignas(4) uint8_t lwin[4][LP_LWIN];     // the four streams' windows
  };
  BR lbr[4];
  uint32_t lcnt[4], lout[4], lwlo[4], lrn[4];
  uint32_t act, lact;                         // decoding; bit j = stream j has symbols left
  // lit_header's state (its field names)
  uint32_t ip, bend, op, lit_used, lit_direct, lit_n, lit_kind, lit_base, lit_rle;
  uint32_t hdesc, hdesc_end, hbits, nls;
  int32_t err;
  uint32_t len, cap;
  const uint8_t *in;
  uint8_t *litp;                              // the block's literal region (in the output)
};

struct alignas(16) LpS {                      // a block's sequence section
  uint32_t tll[512];
  uint32_t tml[512];
  uint32_t tof[256];
  union {
    struct {                                  // building an FSE table
      int16_t norm[64];
      uint16_t snext[64];
    };
    alignas(4) uint8_t swin[LP_SWIN];        // the bitstream's window
  };
  BR sbr;
  uint32_t swlo, act;
  uint32_t tmode[3], tpos[3], tend[3], have_ll, have_of, have_ml;
  uint32_t nseq, seq_done, st_ll, st_of, st_ml, al_ll, al_of, al_ml;
  uint32_t rep[3], lit, out, nent, lit_n, sip, bend;
  int32_t err;
  uint32_t len;
  const uint8_t *in;
  Ent *ent;
};

struct LpLWave {
  LpL b[LPLB];
};

struct LpSWave {
  uint32_t ctab[36 + 53];                     // LL / ML code -> base | extra bits << 24
  LpS b[LPSB];
};

// (L0) a block's lane 0: its record, literal section header + tree
HD void lp_lit_begin(LpL &s, const LpBlock *blk, uint32_t k, uint32_t nlist, const uint8_t *src,
                     uint8_t *dst, const strom_decomp_desc *desc) {
  s.act = 0;
  s.lact = 0;
  s.err = 0;
  if (k >= nlist) return;
  const LpBlock &r = blk[k];
  if (!r.active) return;
  const strom_decomp_desc dd = desc[r.stream];
  s.in = src + dd.src_off;
  s.len = dd.src_len;
  s.cap = dd.dst_len;
  s.litp = dst + dd.dst_off + r.lit_off;
  s.ip = r.bstart;
  s.bend = r.bend;
  s.op = 0;
  s.hbits = r.d.hbits;
  s.hdesc = r.d.hdesc;
  s.hdesc_end = r.d.hdesc_end;
  s.act = 1;
  const Ctx c{s.in, nullptr, nullptr, s.len, s.cap};
  if (!lit_header(s, c)) {
    s.err = ZF(kErrFormat);
    return;
  }
  s.lit_direct = 0;
  if (s.lit_kind == kLitScratch)
    for (uint32_t j = 0; j < s.nls; ++j)
      if (s.lcnt[j]) s.lact |= 1u << j;
}

// (L) the block's results: its literal section, where its sequences start
HD void lp_lit_end(const LpL &s, LpBlock *blk, uint32_t k, uint32_t nlist) {
  if (k >= nlist || !blk[k].active) return;
  LpBlock &r = blk[k];
  r.err = s.err;
  r.lit_kind = s.lit_kind;
  r.lit_n = s.lit_n;
  r.lit_base = s.lit_base;
  r.lit_rle = s.lit_rle;
  r.sip = s.ip;                               // where the sequence section starts
}

// (1) literal windows of every stream with symbols left: one dword per lane
// each, aligned in the input (bytes outside it read as 0)
HD uint32_t lp_ld32(const uint8_t *in, uint32_t len, uint32_t p) {
  const ZG uint8_t *g = zg(in);
  if (p < len && len - p >= 4) return *(const ZG uint32_t *)(g + p);
  uint32_t v = 0;
  for (uint32_t j = 0; j < 4; ++j) v |= (p + j < len ? (uint32_t)g[p + j] : 0u) << (8 * j);
  return v;
}

// a window origin moved down to a dword boundary of the input (the caller
// asked win_lo for 4 bytes less, so the window still reaches as high); below
// the input it wraps and reads as 0
HD uint32_t lp_align_lo(const uint8_t *in, uint32_t lo) {
  return lo - (uint32_t)(((uintptr_t)in + lo) & 3);
}

// Every window dword of the round is LOADED before any is stored: one
// load per window with its LDS store behind it serialized the round on
// global-memory latency (a wait per window: 32 / 24 round trips per round,
// most of the entropy launch — r5 trace).  Inactive windows load from
// `safe` (any valid global dword); dwords that reach past either end of
// the input take the guarded byte path afterwards (a stream's first /
// last window only).
template <uint32_t NWIN, uint32_t PER, class F>
HD void lp_windows(const uint32_t *safe, uint32_t t, F win) {
  uint32_t v[NWIN * PER];
  uint64_t slow = 0;
  static_assert(NWIN * PER <= 64, "window dwords per lane");
#pragma unroll
  for (uint32_t w = 0; w < NWIN; ++w) {
    const uint8_t *in;
    uint32_t len, lo;
    uint8_t *dst;
    const bool on = win(w, in, len, lo, dst);
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      const uint32_t p = lo + 4 * (t + k * NT);
      const bool fast = on && p < len && len - p >= 4;
      const ZG uint32_t *a = fast ? (const ZG uint32_t *)(zg(in) + p) : zg(safe);
      v[w * PER + k] = *a;
      if (on && !fast) slow |= 1ull << (w * PER + k);
    }
  }
  if (slow) {
#pragma unroll
    for (uint32_t w = 0; w < NWIN; ++w) {
      const uint8_t *in;
      uint32_t len, lo;
      uint8_t *dst;
      win(w, in, len, lo, dst);
#pragma unroll
      for (uint32_t k = 0; k < PER; ++k)
        if (slow >> (w * PER + k) & 1) v[w * PER + k] = lp_ld32(in, len, lo + 4 * (t + k * NT));
    }
  }
#pragma unroll
  for (uint32_t w = 0; w < NWIN; ++w) {
    const uint8_t *in;
    uint32_t len, lo;
    uint8_t *dst;
    if (!win(w, in, len, lo, dst)) continue;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) ((uint32_t *)dst)[t + k * NT] = v[w * PER + k];
  }
}

HD void lp_lit_windows(LpLWave &W, uint32_t t, const uint32_t *safe) {
  lp_windows<4 * LPLB, LP_LWIN / (4 * NT)>(safe, t, [&](uint32_t w, const uint8_t *&in,
                                                        uint32_t &len, uint32_t &lo, uint8_t *&dst) {
    LpL &s = W.b[w / 4];
    const uint32_t j = w % 4;
    in = s.in;
    len = s.len;
    lo = s.lwlo[j];
    dst = s.lwin[j];
    return (s.lact >> j & 1) != 0;
  });
}

HD void lp_seq_windows(LpSWave &W, uint32_t t, const uint32_t *safe) {
  lp_windows<LPSB, LP_SWIN / (4 * NT)>(safe, t, [&](uint32_t w, const uint8_t *&in, uint32_t &len,
                                                    uint32_t &lo, uint8_t *&dst) {
    LpS &s = W.b[w];
    in = s.in;
    len = s.len;
    lo = s.swlo;
    dst = s.swin;
    return s.act && !s.err && s.seq_done < s.nseq;
  });
}

// (1) up to LP_LSYM symbols of literal stream j, straight into the block's
// literal region (four per container check, as lit_chunk)
HD void lp_lit_chunk(LpL &s, uint32_t j) {
  const uint32_t left = s.lcnt[j];
  BR b = s.lbr[j];
  const Win w{(uint32_t)offsetof(LpL, lwin) + j * LP_LWIN, s.lwlo[j], LP_LWIN};
  const uint32_t n = left < LP_LSYM ? left : LP_LSYM, mb = s.hbits;
  ZG uint8_t *dst = zg(s.litp) + s.lout[j];
  const uint32_t nf = n & ~3u;
  for (uint32_t k = 0; k < nf; k += 4) {
    br_need(b, s, w, 4 * mb);
    uint32_t word = 0;
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const uint32_t lo = (uint32_t)(b.nbits - (int32_t)mb - b.cbase) & 63;
      const uint32_t x = ubfe((uint32_t)(b.cont >> lo), 0, mb);
      b.nbits -= (int32_t)s.hlen[x];
      word |= (uint32_t)s.hsym[x] << (8 * g);
    }
    ZG uint8_t *o = dst + k;
    if (((uintptr_t)o & 3) == 0) {
      *(ZG uint32_t *)o = word;
    } else {
      o[0] = (uint8_t)word;
      o[1] = (uint8_t)(word >> 8);
      o[2] = (uint8_t)(word >> 16);
      o[3] = (uint8_t)(word >> 24);
    }
  }
  if (nf < n) {
    br_need(b, s, w, 4 * mb);
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const uint32_t lo = (uint32_t)(b.nbits - (int32_t)mb - b.cbase) & 63;
      const uint32_t x = ubfe((uint32_t)(b.cont >> lo), 0, mb);
      if (nf + g < n) {
        b.nbits -= (int32_t)s.hlen[x];
        dst[nf + g] = s.hsym[x];
      }
    }
  }
  s.lout[j] += n;
  s.lcnt[j] = left - n;
  s.lbr[j] = b;
  if (left == n) {
    if (b.nbits != 0) s.err = ZF(kErrFormat);   // a stream ends exactly
    s.lact &= ~(1u << j);
  }
}

// the literal launch's wave: LPLB blocks' literal sections
template <class TM>
HD void lp_lit_group(TM &tm, LpLWave &W, LpBlock *blk, uint32_t k0, uint32_t nlist,
                     const uint8_t *src, uint8_t *dst, const strom_decomp_desc *desc) {
  tm.each([&](uint32_t t) {
    if (t % LPLL == 0) lp_lit_begin(W.b[t / LPLL], blk, k0 + t / LPLL, nlist, src, dst, desc);
  });
  tm.sync();
  for (;;) {
    const bool more = tm.any([&](uint32_t t) {
      LpL &s = W.b[t / LPLL];
      const uint32_t j = t % LPLL;
      if (j < 4 && s.err) s.lact = 0;
      return j < 4 && (s.lact >> j & 1);
    });
    if (!more) break;
    tm.each([&](uint32_t t) {
      LpL &s = W.b[t / LPLL];
      const uint32_t j = t % LPLL;
      if (j < 4 && (s.lact >> j & 1)) s.lwlo[j] = lp_align_lo(s.in, win_lo(s.lbr[j], LP_LWIN - 4));
    });
    tm.sync();
    tm.each([&](uint32_t t) { lp_lit_windows(W, t, (const uint32_t *)desc); });
    tm.sync();
    tm.each([&](uint32_t t) {
      LpL &s = W.b[t / LPLL];
      const uint32_t j = t % LPLL;
      if (j < 4 && (s.lact >> j & 1)) lp_lit_chunk(s, j);
    });
    tm.sync();
  }
  tm.each([&](uint32_t t) {
    if (t % LPLL == 0) lp_lit_end(W.b[t / LPLL], blk, k0 + t / LPLL, nlist);
  });
  tm.fence();
  tm.sync();
}

// (S0) block b's lane: the sequence section header (compact tables), from
// where the literal launch left it
HD void lp_seq_begin(LpS &s, const LpBlock *blk, uint32_t k, uint32_t nlist, const uint8_t *src,
                     const strom_decomp_desc *desc, uint8_t *pool) {
  s.act = 0;
  s.err = 0;
  if (k >= nlist) return;
  const LpBlock &r = blk[k];
  if (!r.active || r.err) return;
  const strom_decomp_desc dd = desc[r.stream];
  s.in = src + dd.src_off;
  s.len = dd.src_len;
  s.ent = (Ent *)(pool + r.ent_off);
  s.lit_n = r.lit_n;
  s.bend = r.bend;
  s.have_ll = r.d.have[kLL];
  s.have_of = r.d.have[kOF];
  s.have_ml = r.d.have[kML];
  for (uint32_t j = 0; j < 3; ++j) {
    s.tmode[j] = r.d.tmode[j];
    s.tpos[j] = r.d.tpos[j];
    s.tend[j] = r.d.tend[j];
    s.rep[j] = kSym | (j << 26);
  }
  s.act = 1;
  const Ctx c{s.in, nullptr, nullptr, s.len, 0};
  uint32_t p = r.sip;                         // after the literal section
  const uint32_t end = s.bend;
  s.seq_done = 0;
  s.lit = 0;
  s.out = 0;
  s.nent = 0;
  s.nseq = 0;
  if (p >= end) {
    s.err = ZF(kErrFormat);
    return;
  }
  const uint32_t b0 = gbyte(c, p);
  uint32_t n;
  if (b0 == 0) {
    if (p + 1 != end) s.err = ZF(kErrFormat);
    return;
  }
  if (b0 < 128) {
    n = b0;
    p += 1;
  } else if (b0 < 255) {
    n = ((b0 - 128) << 8) + gbyte(c, p + 1);
    p += 2;
  } else {
    n = gbyte(c, p + 1) + (gbyte(c, p + 2) << 8) + 0x7F00;
    p += 3;
  }
  s.nseq = n;
  if (p >= end || n > kMaxSeq) {
    s.err = ZF(kErrFormat);
    return;
  }
  const uint32_t modes = gbyte(c, p++);
  if ((modes & 3) || !seq_table4(s, c, modes >> 6, kLL, p, end, s.tll, s.al_ll, s.have_ll) ||
      !seq_table4(s, c, (modes >> 4) & 3, kOF, p, end, s.tof, s.al_of, s.have_of) ||
      !seq_table4(s, c, (modes >> 2) & 3, kML, p, end, s.tml, s.al_ml, s.have_ml) ||
      p >= end || !br_init(s.sbr, c, p, end - p)) {
    s.err = ZF(kErrFormat);
    return;
  }
  const Win w{0, 0, 0};
  s.st_ll = br_read(s.sbr, s, w, c, s.al_ll);
  s.st_of = br_read(s.sbr, s, w, c, s.al_of);
  s.st_ml = br_read(s.sbr, s, w, c, s.al_ml);
  if (s.sbr.nbits < 0) s.err = ZF(kErrFormat);
}

// (S) a block's lane: up to LP_SEQN sequences into its entries — seq_chunk
// with symbolic repeat offsets on one lane: the LL / ML baselines from the
// wave's code table, the repeat-offset update as selects
HD void lp_seq_chunk(LpS &s, const uint32_t *ctab) {
  const uint32_t left = s.nseq - s.seq_done;
  const uint32_t m = left < LP_SEQN ? left : LP_SEQN;
  BR b = s.sbr;
  const Win w{(uint32_t)offsetof(LpS, swin), s.swlo, LP_SWIN};
  uint32_t sll = s.st_ll, sof = s.st_of, sml = s.st_ml;
  uint32_t r0 = s.rep[0], r1 = s.rep[1], r2 = s.rep[2];
  uint32_t n = s.nent, out = s.out, lit = s.lit;
  bool bad = false;
  ZG Ent *ent = zg(s.ent);
  for (uint32_t i = 0; i < m; ++i) {
    const bool more = i + 1 < left;           // the block's last sequence reads no state bits
    const uint32_t eo = s.tof[sof], em = s.tml[sml], el = s.tll[sll];
    const uint32_t cm = ctab[36 + (em & 255)], cl = ctab[el & 255];
    const uint32_t oa = eo & 255, ob = 1u << oa;
    const uint32_t ma = cm >> 24, mb = cm & 0xFFFFFF, la = cl >> 24, lb = cl & 0xFFFFFF;
    br_need(b, s, w, 47);
    const uint64_t x1 = br_take(b, oa + ma);
    const uint32_t ml = mb + ubfe((uint32_t)x1, 0, ma);
    const uint32_t ofv = ob + ubfe((uint32_t)(x1 >> ma), 0, oa);
    const uint32_t onb = (eo >> 8) & 255, mnb = (em >> 8) & 255, lnb = (el >> 8) & 255;
    br_need(b, s, w, 42);
    const uint32_t nst = more ? lnb + mnb + onb : 0;
    const uint64_t x2 = br_take(b, la + nst);
    const uint32_t ll = lb + ubfe((uint32_t)(x2 >> nst), 0, la);
    const uint32_t y = (uint32_t)x2;
    sof = (eo >> 16) + ubfe(y, 0, onb);
    sml = (em >> 16) + ubfe(y, onb, mnb);
    sll = (el >> 16) + ubfe(y, onb + mnb, lnb);
    // repeat offsets (RFC 8878 3.1.2.5), as selects: "plain" is the first
    // repeat offset after literals (nothing changes); k = 1, 2 the second /
    // third, k = 3 the first minus one (symbolic: + 1 on the symbol's k)
    const bool isnew = ofv > 3;
    const bool plain = ofv == 1 && ll != 0;
    const uint32_t k = ofv - 1 + (ll == 0 ? 1u : 0u);
    const uint32_t r0m1 = is_sym(r0) ? r0 + 1 : r0 - 1;
    const uint32_t rep = k == 1 ? r1 : k == 2 ? r2 : r0m1;
    const uint32_t off = plain ? r0 : isnew ? ofv - 3 : rep;
    bad |= isnew && is_sym(off);
    const uint32_t n2 = plain ? r2 : (isnew || k >= 2) ? r1 : r2;
    const uint32_t n1 = plain ? r1 : r0;
    r2 = n2;
    r1 = n1;
    r0 = off;
    ZG Ent &e = ent[n++];
    e.ll = ll;
    e.off = off;
    e.lst = lit;
    e.ost = out;
    lit += ll;
    out += ll + ml;
  }
  int32_t err = 0;
  if (lit > s.lit_n || out > MAXB) err = ZF(kErrFormat);
  else if (bad) err = ZF(kErrDistance);
  s.seq_done += m;
  s.sbr = b;
  s.st_ll = sll;
  s.st_of = sof;
  s.st_ml = sml;
  s.rep[0] = r0;
  s.rep[1] = r1;
  s.rep[2] = r2;
  s.nent = n;
  s.out = out;
  s.lit = lit;
  if (err) s.err = err;
}

// (S) a block's lane: trailing literals, checks, the record's results
HD void lp_seq_end(LpS &s, LpBlock *blk, uint32_t k, uint32_t nlist) {
  if (k >= nlist) return;
  LpBlock &r = blk[k];
  if (!r.active) {
    r.err = 0;
    r.bout = r.bsize;
    r.nent = 0;
    r.nseq = 0;
    return;
  }
  if (r.err) return;                          // the literal launch's
  if (!s.err && s.nseq && s.sbr.nbits != 0) s.err = ZF(kErrFormat);
  if (!s.err) {
    const uint32_t rest = s.lit_n - s.lit;    // lit <= lit_n (lp_seq_chunk's check)
    if (rest) {
      Ent e;
      e.ll = rest;
      e.off = 0;
      e.lst = s.lit;
      e.ost = s.out;
      s.ent[s.nent++] = e;
      s.out += rest;
      s.lit += rest;
    }
    if (s.out > MAXB) s.err = ZF(kErrFormat);
  }
  r.err = s.err;
  r.nseq = s.nseq;
  r.nent = s.nent;
  r.bout = s.out;
  for (uint32_t j = 0; j < 3; ++j) r.rep[j] = s.rep[j];
}

// the sequence launch's wave: LPSB blocks' sequence sections
template <class TM>
HD void lp_seq_group(TM &tm, LpSWave &W, LpBlock *blk, uint32_t k0, uint32_t nlist,
                     const uint8_t *src, const strom_decomp_desc *desc, uint8_t *pool) {
  tm.each([&](uint32_t t) {
    for (uint32_t c = t; c < 36 + 53; c += tm.size()) {
      uint32_t base, add;
      code_base(c < 36 ? kLL : kML, c < 36 ? c : c - 36, base, add);
      W.ctab[c] = base | add << 24;
    }
    if (t < LPSB) lp_seq_begin(W.b[t], blk, k0 + t, nlist, src, desc, pool);
  });
  tm.sync();
  for (;;) {
    const bool more = tm.any([&](uint32_t t) {
      if (t >= LPSB) return false;
      const LpS &s = W.b[t];
      return s.act && !s.err && s.seq_done < s.nseq;
    });
    if (!more) break;
    tm.each([&](uint32_t t) {
      if (t >= LPSB) return;
      LpS &s = W.b[t];
      if (s.act && !s.err && s.seq_done < s.nseq)
        s.swlo = lp_align_lo(s.in, win_lo(s.sbr, LP_SWIN - 4));
    });
    tm.sync();
    tm.each([&](uint32_t t) { lp_seq_windows(W, t, (const uint32_t *)desc); });
    tm.sync();
    tm.each([&](uint32_t t) {
      if (t >= LPSB) return;
      LpS &s = W.b[t];
      if (s.act && !s.err && s.seq_done < s.nseq) lp_seq_chunk(s, W.ctab);
    });
    tm.sync();
  }
  tm.each([&](uint32_t t) {
    if (t < LPSB) lp_seq_end(W.b[t], blk, k0 + t, nlist);
  });
  tm.fence();
  tm.sync();
}

// (exec) One workgroup of LPX_T lanes per stream, blocks in order.  Its
// own LDS (25 KB, six workgroups per CU; the Smem-based exec_fp needs four
// Smem): a chunk of up to LPX_SEQ entries at a time, its output in batches
// of LPX_OB bytes — a source pointer per byte (literal index / stored
// output / earlier byte of the batch), pointer doubling, then every byte
// GATHERED before any is STORED: the block's literals sit in the output
// buffer's tail, never below the position they are copied to, but a batch
// may write where a later byte of the same batch reads.
constexpr uint32_t LPX_T = 256;
constexpr uint32_t LPX_EPT = 16;
constexpr uint32_t LPX_OB = LPX_T * LPX_EPT;    // output bytes per batch
constexpr uint32_t LPX_SEQ = 512;               // entries per chunk
HD constexpr uint32_t PX(uint32_t e) { return e + e / LPX_EPT; }   // bank skew, as PI

struct LpX {
  uint32_t ptr[PX(LPX_OB)];
  uint32_t sll[LPX_SEQ], soff[LPX_SEQ], lst[LPX_SEQ], ost[LPX_SEQ + 1];
  // frame: output position, repeat offsets; block: its record's fields
  uint32_t op, rep[3];
  uint32_t brep[3], btype, bstart, bsize, nseq, lit_kind, lit_n, lit_base, lit_rle;
  uint32_t m, end;                              // the chunk: entries, output bytes
  int32_t err;
};

HD uint32_t lpx_entry_of(const LpX &x, uint32_t pos) {   // ost strictly increases
  uint32_t lo = 0, hi = x.m;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (x.ost[mid] <= pos) lo = mid;
    else hi = mid;
  }
  return lo;
}

HD void lpx_fill(LpX &x, uint32_t t, uint32_t b0, uint32_t nb) {
  const uint32_t abs0 = x.op, e0 = t * LPX_EPT;
  if (e0 >= nb) return;
  uint32_t i = lpx_entry_of(x, b0 + e0);
  uint32_t start = x.ost[i], next = x.ost[i + 1];
  uint32_t ll = x.sll[i], off = x.soff[i], lst = x.lst[i];
  for (uint32_t k = 0; k < LPX_EPT; ++k) {
    const uint32_t e = e0 + k;
    if (e >= nb) break;
    const uint32_t pos = b0 + e;
    while (pos >= next) {
      ++i;
      start = next;
      next = x.ost[i + 1];
      ll = x.sll[i];
      off = x.soff[i];
      lst = x.lst[i];
    }
    const uint32_t r = pos - start;
    uint32_t v;
    if (r < ll) {
      v = kLit | (lst + r);
    } else {
      const uint32_t src = abs0 + pos - off;
      v = src < abs0 + b0 ? (kHist | src) : src - abs0 - b0;
    }
    x.ptr[PX(e)] = v;
  }
}

HD bool lpx_double(LpX &x, uint32_t t, uint32_t nb) {
  bool more = false;
  for (uint32_t k = 0; k < LPX_EPT; ++k) {
    const uint32_t e = k * LPX_T + t;
    if (e >= nb) break;
    const uint32_t v = x.ptr[PX(e)];
    if (v & kTag) continue;
    const uint32_t y = x.ptr[PX(v)];
    x.ptr[PX(e)] = y;
    more |= !(y & kTag);
  }
  return more;
}

HD void lpx_gather(LpX &x, const Ctx &c, const uint8_t *lit, uint32_t t, uint32_t nb) {
  for (uint32_t k = 0; k < LPX_EPT; ++k) {
    const uint32_t e = k * LPX_T + t;
    if (e >= nb) break;
    const uint32_t v = x.ptr[PX(e)], a = v & ~kTag;
    uint32_t y;
    if (v & kLit)
      y = x.lit_kind == kLitInput ? c.in[x.lit_base + a] : x.lit_kind == kLitRle ? x.lit_rle : lit[a];
    else
      y = c.out[a];
    x.ptr[PX(e)] = y;
  }
}

HD void lpx_store(const LpX &x, const Ctx &c, uint32_t t, uint32_t b0, uint32_t nb) {
  uint8_t *o = c.out + x.op + b0;
  for (uint32_t k = 0; k < LPX_EPT; ++k) {
    const uint32_t e = k * LPX_T + t;
    if (e >= nb) break;
    o[e] = (uint8_t)x.ptr[PX(e)];
  }
}

// one block of the stream at x.op (the frame state advances)
template <class TM>
HD void lpx_block(TM &tm, LpX &x, const Ctx &c, const LpBlock &b, const Ent *ent) {
  tm.one([&] {
    x.btype = b.btype;
    x.bstart = b.bstart;
    x.bsize = b.bsize;
    x.nseq = b.nseq;
    x.lit_kind = b.lit_kind;
    x.lit_n = b.lit_n;
    x.lit_base = b.lit_base;
    x.lit_rle = b.lit_rle;
    for (uint32_t j = 0; j < 3; ++j) x.brep[j] = b.rep[j];
    if ((uint64_t)x.op + b.bout > c.cap) x.err = kErrOverflow;
  });
  tm.sync();
  if (x.err) return;
  const uint32_t tn = tm.size(), nent = b.nent, bout = b.bout;
  if (x.btype != kComp) {
    tm.each([&](uint32_t t) {
      uint8_t *o = c.out + x.op;
      if (x.btype == kRle) {
        const uint8_t v = (uint8_t)gbyte(c, x.bstart);
        for (uint32_t i = t; i < x.bsize; i += tn) o[i] = v;
      } else {
        const uint8_t *in = c.in + x.bstart;
        for (uint32_t i = t; i < x.bsize; i += tn) o[i] = in[i];
      }
    });
  } else {
    const uint8_t *lit = c.out + b.lit_off;
    const uint32_t fpos = x.op;                  // one frame per LP stream: it starts at 0
    for (uint32_t i0 = 0; i0 < nent; i0 += LPX_SEQ) {
      const uint32_t m = nent - i0 < LPX_SEQ ? nent - i0 : LPX_SEQ;
      const uint32_t base = ent[i0].ost;
      const uint32_t end = (i0 + m < nent ? ent[i0 + m].ost : bout) - base;
      tm.each([&](uint32_t t) {
        const uint32_t rin[3] = {x.rep[0], x.rep[1], x.rep[2]};
        bool bad = false;
        for (uint32_t i = t; i < m; i += tn) {
          const Ent e = ent[i0 + i];
          const uint32_t off = sym_resolve(e.off, rin);
          // a match reaches back at most to the frame start; the trailing
          // literals entry has no match
          const bool has_match = (i0 + i + 1 < nent ? ent[i0 + i + 1].ost : bout) - e.ost > e.ll;
          bad |= has_match && off - 1 >= fpos + e.ost + e.ll;
          x.sll[i] = e.ll;
          x.soff[i] = off;
          x.lst[i] = e.lst;
          x.ost[i] = e.ost - base;
        }
        if (t == 0) {
          x.ost[m] = end;
          x.m = m;
        }
        if (bad) x.err = ZF(kErrDistance);
      });
      tm.sync();
      if (x.err) return;
      for (uint32_t b0 = 0; b0 < end; b0 += LPX_OB) {
        const uint32_t nb = end - b0 < LPX_OB ? end - b0 : LPX_OB;
        tm.each([&](uint32_t t) { lpx_fill(x, t, b0, nb); });
        tm.sync();
        while (tm.any([&](uint32_t t) { return lpx_double(x, t, nb); })) {
        }
        tm.each([&](uint32_t t) { lpx_gather(x, c, lit, t, nb); });
        tm.sync();
        tm.each([&](uint32_t t) { lpx_store(x, c, t, b0, nb); });
        tm.fence();
        tm.sync();
      }
      tm.one([&] { x.op += end; });
      tm.sync();
    }
  }
  tm.fence();
  tm.sync();
  tm.one([&] {
    if (x.btype != kComp) x.op += x.bsize;
    if (x.btype == kComp && x.nseq) {
      const uint32_t rin[3] = {x.rep[0], x.rep[1], x.rep[2]};
      for (uint32_t j = 0; j < 3; ++j) x.rep[j] = sym_resolve(x.brep[j], rin);
    }
  });
  tm.sync();
}

// (exec) one stream: its blocks in order, then the frame's checks.
// Returns the status, or kLpRedo when the serial decoder has to decode the
// stream (refused by the walk, or any LP error: it then reports the error
// the serial decoder finds).
constexpr int32_t kLpRedo = INT32_MIN;

template <class TM>
HD int32_t lp_exec_stream(TM &tm, LpX &x, const LpStream &st, const LpBlock *blk,
                          const uint8_t *pool, const Ctx &c) {
  if (st.mode != kLpDecode) return kLpRedo;
  for (uint32_t k = 0; k < st.nblk; ++k)
    if (blk[st.first + k].err) return kLpRedo;
  tm.one([&] {
    x.op = 0;
    x.rep[0] = 1;
    x.rep[1] = 4;
    x.rep[2] = 8;
    x.err = 0;
  });
  tm.sync();
  for (uint32_t k = 0; k < st.nblk && !x.err; ++k) {
    const LpBlock &b = blk[st.first + k];
    lpx_block(tm, x, c, b, (const Ent *)(pool + b.ent_off));
  }
  if (x.err || (st.fcs_set && x.op != st.fcs) || (st.expect >= 0 && (int64_t)x.op != st.expect))
    return kLpRedo;
  return (int32_t)x.op;
}

// frame-parallel scratch per workgroup: NW literal slots, then NW - 1
// entry buffers
HD constexpr size_t fp_scratch(uint32_t nw) {
  return (size_t)nw * (SLOT + kMaxEnt * sizeof(Ent));
}

#ifndef ZS_FPW
#define ZS_FPW 4
#endif
// frame-parallel up to this many of its resident rounds: at 1,024 val
// streams two FP rounds beat the wave decoder's one (26.4 vs 17.0 GB/s,
// profiles/r4/zstd/), at 2,048 the wave decoder's full round wins
#ifndef ZS_FP_ROUNDS
#define ZS_FP_ROUNDS 2
#endif
constexpr uint32_t FPW = ZS_FPW;                 // waves (blocks in flight) per stream
static_assert(FPW >= 2 && FPW <= NWMAX, "frame-parallel waves");

__global__ void __launch_bounds__(NT * FPW) __attribute__((amdgpu_waves_per_eu(2))) zstd_fp_kernel(int codec, const uint8_t *src,
                                                          uint8_t *dst,
                                                          const strom_decomp_desc *desc,
                                                          uint32_t n, int32_t *status,
                                                          uint8_t *scratch) {
  __shared__ Smem sm[FPW];
  __shared__ FpShared f;
  DevGroup g;
  uint8_t *base = scratch + (size_t)blockIdx.x * fp_scratch(FPW);
  for (uint32_t b = blockIdx.x; b < n; b += gridDim.x) {
    const strom_decomp_desc d = desc[b];
    const FpCtx x{Ctx{src + d.src_off, dst + d.dst_off, base, d.src_len, d.dst_len}, base, FPW};
    run_fp(g, sm, f, x, codec);
    if (threadIdx.x == 0) status[b] = sm[0].err ? sm[0].err : (int32_t)sm[0].op;
    __syncthreads();
  }
}

// 3 waves per SIMD (<= 168 VGPRs): with the phase-shared LDS, up to 12
// streams per CU
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(ZS_WPE))) zstd_kernel(int codec, const uint8_t *src, uint8_t *dst,
                                                   const strom_decomp_desc *desc, uint32_t n,
                                                   int32_t *status, uint8_t *scratch) {
  __shared__ Smem s;
  DevTeam tm;
  uint8_t *lit = scratch + (size_t)blockIdx.x * SLOT;
  for (uint32_t b = blockIdx.x; b < n; b += gridDim.x) {
    const strom_decomp_desc d = desc[b];
    const Ctx c{src + d.src_off, dst + d.dst_off, lit, d.src_len, d.dst_len};
    run(tm, s, c, codec);
    if (threadIdx.x == 0) status[b] = s.err ? s.err : (int32_t)s.op;
    __syncthreads();
  }
  tm.flush();
}

// ---- lane-parallel launches
// pool layout: LpHdr | LpStream[n] | LpBlock[blk_cap] | exec fallback slots | entries
struct LpLayout {
  size_t streams, blocks, slots, ents, total;
  uint32_t blk_cap, nslot;
  uint64_t ent_cap;
};

HD size_t lp_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

HD LpLayout lp_layout(uint32_t n, uint32_t blk_cap, uint32_t nslot, uint64_t ent_cap) {
  LpLayout l;
  l.blk_cap = blk_cap;
  l.nslot = nslot;
  l.ent_cap = ent_cap;
  l.streams = 256;
  l.blocks = lp_up(l.streams + (size_t)n * sizeof(LpStream), 256);
  l.slots = lp_up(l.blocks + (size_t)blk_cap * sizeof(LpBlock), 256);
  l.ents = lp_up(l.slots + (size_t)nslot * SLOT, 256);
  l.total = l.ents + (size_t)ent_cap;
  return l;
}

// one stream's walk: the stream record, its blocks listed and its entries
// allocated (two passes over its headers: count, then fill)
// A: atomics policy (device atomics, or plain adds on the CPU)
template <class A>
HD void lp_walk_stream(LpWalk &ws, const Ctx &c, int codec, uint32_t i, uint8_t *pool,
                       const LpLayout &l) {
  LpHdr &h = *(LpHdr *)pool;
  LpStream *st = (LpStream *)(pool + l.streams);
  LpBlock *blk = (LpBlock *)(pool + l.blocks);
  LpStream s{};
  s.mode = kLpSerial;
  s.expect = -1;
  uint32_t nblk, lits, nent;
  if (lp_walk(ws, c, codec, i, nullptr, 0, 0, nblk, lits, nent, s)) {
    const uint32_t first = A::add32(&h.nblk, nblk);
    const uint64_t need = (uint64_t)nent * sizeof(Ent);
    const uint64_t eoff = need ? A::add64(&h.ent_used, need) : 0;
    const bool fits = first < l.blk_cap && nblk <= l.blk_cap - first && eoff <= l.ent_cap &&
                      need <= l.ent_cap - eoff;
    uint32_t n2, l2, e2;
    if (fits && lp_walk(ws, c, codec, i, blk + first, c.cap - lits, eoff, n2, l2, e2, s) &&
        n2 == nblk && !s.cksum) {              // a content checksum: the serial decoder verifies it
      s.first = first;
      s.nblk = nblk;
      s.mode = kLpDecode;
    } else {
      // listed blocks of a stream the serial decoder takes: idle in the
      // entropy launch
      for (uint32_t k = first; k < l.blk_cap && k - first < nblk; ++k) {
        blk[k] = LpBlock{};
        blk[k].stream = i;
      }
      s.mode = kLpSerial;
    }
  }
  st[i] = s;
}

struct LpDevAtom {
  static __device__ uint32_t add32(uint32_t *p, uint32_t v) { return atomicAdd(p, v); }
  static __device__ uint64_t add64(uint64_t *p, uint64_t v) {
    return (uint64_t)atomicAdd((unsigned long long *)p, (unsigned long long)v);
  }
};

struct LpHostAtom {
  static uint32_t add32(uint32_t *p, uint32_t v) {
    const uint32_t o = *p;
    *p = o + v;
    return o;
  }
  static uint64_t add64(uint64_t *p, uint64_t v) {
    const uint64_t o = *p;
    *p = o + v;
    return o;
  }
};

constexpr uint32_t LP_WALK_T = 64;

__global__ void __launch_bounds__(LP_WALK_T) zstd_lp_walk(int codec, const uint8_t *src,
                                                          const strom_decomp_desc *desc, uint32_t n,
                                                          uint8_t *pool, LpLayout l) {
  __shared__ LpWalk ws[LP_WALK_T];
  const uint32_t i = blockIdx.x * LP_WALK_T + threadIdx.x;
  if (i >= n) return;
  const strom_decomp_desc d = desc[i];
  const Ctx c{src + d.src_off, nullptr, nullptr, d.src_len, d.dst_len};
  lp_walk_stream<LpDevAtom>(ws[threadIdx.x], c, codec, i, pool, l);
}

__global__ void __launch_bounds__(NT) zstd_lp_lit(const uint8_t *src, uint8_t *dst,
                                                  const strom_decomp_desc *desc, uint8_t *pool,
                                                  LpLayout l) {
  __shared__ LpLWave W;
  const uint32_t nb = *(const volatile uint32_t *)pool;
  const uint32_t nlist = nb < l.blk_cap ? nb : l.blk_cap;
  LpBlock *blk = (LpBlock *)(pool + l.blocks);
  DevTeam tm;
  for (uint32_t k0 = blockIdx.x * LPLB; k0 < nlist; k0 += gridDim.x * LPLB)
    lp_lit_group(tm, W, blk, k0, nlist, src, dst, desc);
}

__global__ void __launch_bounds__(NT) zstd_lp_seq(const uint8_t *src, const strom_decomp_desc *desc,
                                                  uint8_t *pool, LpLayout l) {
  __shared__ LpSWave W;
  const uint32_t nb = *(const volatile uint32_t *)pool;
  const uint32_t nlist = nb < l.blk_cap ? nb : l.blk_cap;
  LpBlock *blk = (LpBlock *)(pool + l.blocks);
  DevTeam tm;
  for (uint32_t k0 = blockIdx.x * LPSB; k0 < nlist; k0 += gridDim.x * LPSB)
    lp_seq_group(tm, W, blk, k0, nlist, src, desc, pool + l.ents);
}

__global__ void __launch_bounds__(LPX_T) zstd_lp_exec(const uint8_t *src, uint8_t *dst,
                                                      const strom_decomp_desc *desc, uint32_t n,
                                                      int32_t *status, uint8_t *pool, LpLayout l) {
  __shared__ LpX x;
  DevTeam tm;
  const LpStream *st = (const LpStream *)(pool + l.streams);
  const LpBlock *blk = (const LpBlock *)(pool + l.blocks);
  for (uint32_t b = blockIdx.x; b < n; b += gridDim.x) {
    const strom_decomp_desc d = desc[b];
    const Ctx c{src + d.src_off, dst + d.dst_off, nullptr, d.src_len, d.dst_len};
    const int32_t r = lp_exec_stream(tm, x, st[b], blk, pool + l.ents, c);
    if (threadIdx.x == 0) {
      status[b] = r;
      if (r != kLpRedo) atomicAdd(&((LpHdr *)pool)->lp_done, 1u);
    }
    __syncthreads();
  }
}

// the streams the LP path handed back (status kLpRedo): the serial decoder,
// one wave each, a literal slot per workgroup
__global__ void __launch_bounds__(NT) zstd_lp_serial(int codec, const uint8_t *src, uint8_t *dst,
                                                     const strom_decomp_desc *desc, uint32_t n,
                                                     int32_t *status, uint8_t *pool, LpLayout l) {
  __shared__ Smem s;
  DevTeam tm;
  uint8_t *lit = pool + l.slots + (size_t)blockIdx.x * SLOT;
  for (uint32_t b = blockIdx.x; b < n; b += gridDim.x) {
    if (status[b] != kLpRedo) continue;
    const strom_decomp_desc d = desc[b];
    const Ctx c{src + d.src_off, dst + d.dst_off, lit, d.src_len, d.dst_len};
    run(tm, s, c, codec);
    if (threadIdx.x == 0) status[b] = s.err ? s.err : (int32_t)s.op;
    __syncthreads();
  }
}

// LP launch geometry
uint32_t lp_lit_per_cu() {
  const uint32_t per = (160u << 10) / (uint32_t)sizeof(LpLWave);
  return per ? (per > 8 ? 8 : per) : 1;
}

uint32_t lp_seq_per_cu() {
  const uint32_t per = (160u << 10) / (uint32_t)sizeof(LpSWave);
  return per ? (per > 8 ? 8 : per) : 1;
}

uint32_t lp_exec_per_cu() {
  const uint32_t per = (160u << 10) / (uint32_t)sizeof(LpX);
  return per ? (per > 8 ? 8 : per) : 1;
}

double lp_ent_factor() {
  static double f = 0;
  if (f == 0) {
    const char *e = getenv("STROM_ZSTD_LP_ENT");
    f = e ? atof(e) : 0;
    if (!(f > 0)) f = 3.0;
  }
  return f;
}

// literal scratch per (device, stream): launches on one stream are ordered,
// concurrent launches on different streams never share a slot
std::mutex g_mu;
struct Scratch {
  uint8_t *p = nullptr;
  size_t bytes = 0;
  uint64_t used = 0;         // LRU stamp
};
// key: (device, stream, tag) — tag 0 the wave / frame-parallel decoders'
// literal slots, 1 the lane-parallel decoder's pool
struct ScratchKey {
  int dev;
  void *stream;
  int tag;
  bool operator<(const ScratchKey &o) const {
    return dev != o.dev ? dev < o.dev : stream != o.stream ? stream < o.stream : tag < o.tag;
  }
};
std::map<ScratchKey, Scratch> g_scratch;
uint64_t g_scratch_clock = 0;
constexpr size_t kScratchKeep = 8;   // streams with a cached buffer

// Caller holds g_mu until its launch is enqueued: an eviction (or
// strom_zstd_release) by another thread frees a buffer only with hipFree /
// hipStreamSynchronize, which wait for work already QUEUED — so the launch
// that uses the pointer must be queued before the lock drops.
uint8_t *scratch_for(void *stream, size_t bytes, int tag = 0) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  auto it = g_scratch.find(ScratchKey{dev, stream, tag});
  if (it == g_scratch.end()) {
    // bound the cache: a caller cycling through many streams would
    // otherwise keep up to ~290 MiB per stream; the least recently used
    // entry goes (hipFree waits for the device's outstanding work)
    if (g_scratch.size() >= kScratchKeep) {
      auto lru = g_scratch.begin();
      for (auto j = g_scratch.begin(); j != g_scratch.end(); ++j)
        if (j->second.used < lru->second.used) lru = j;
      if (lru->second.p) (void)hipFree(lru->second.p);
      g_scratch.erase(lru);
    }
    it = g_scratch.emplace(ScratchKey{dev, stream, tag}, Scratch{}).first;
  }
  Scratch &e = it->second;
  e.used = ++g_scratch_clock;
  if (e.bytes < bytes) {
    // a smaller buffer may still be in use by this stream's last launch
    if (e.p && hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return nullptr;
    if (e.p) (void)hipFree(e.p);
    e.p = nullptr;
    e.bytes = 0;
    void *q = nullptr;
    if (hipMalloc(&q, bytes) != hipSuccess) return nullptr;
    e.p = (uint8_t *)q;
    e.bytes = bytes;
  }
  return e.p;
}

uint32_t cu_count() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  static int cached[64] = {0};
  if (dev >= 0 && dev < 64 && cached[dev]) return (uint32_t)cached[dev];
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  if (dev >= 0 && dev < 64) cached[dev] = cus;
  return (uint32_t)cus;
}

uint32_t resident_groups() {
  uint32_t per_cu = (160u << 10) / (uint32_t)sizeof(Smem);   // LDS-bound residency
  if (per_cu > 12) per_cu = 12;                                // 3 waves per SIMD
  return cu_count() * (per_cu ? per_cu : 1);
}

// frame-parallel workgroups resident per CU (LDS-bound: FPW Smem each)
uint32_t fp_per_cu() {
  const uint32_t per = (160u << 10) / (uint32_t)(FPW * sizeof(Smem) + sizeof(FpShared));
  return per ? per : 1;
}

// Decoder choice: the frame-parallel kernel when the streams are too few to
// fill the wave-per-stream decoder's resident round — a stream then takes
// the time of its slowest block plus the executions, not of all its
// blocks — else one wave per stream (more streams in flight per CU).
// STROM_ZSTD_FP: 0 never, 1 always, unset/other: by the stream count.
std::atomic<int> g_fp_mode{-2};

int fp_mode() {
  int m = g_fp_mode.load(std::memory_order_relaxed);
  if (m == -2) {
    const char *e = getenv("STROM_ZSTD_FP");
    m = e && *e == '0' ? 0 : e && *e == '1' ? 1 : -1;
    g_fp_mode.store(m, std::memory_order_relaxed);
  }
  return m;
}

bool use_fp(uint32_t nstreams) {
  const int mode = fp_mode();
  if (mode >= 0) return mode == 1;
  return nstreams <= cu_count() * fp_per_cu() * ZS_FP_ROUNDS;
}

}  // namespace
}  // namespace zs

// Zstandard streams (STROM_CODEC_ZSTD: frames; STROM_CODEC_ARROW_ZSTD: an
// Arrow IPC buffer) — one wavefront per stream, persistent over the
// streams.  scratch: SLOT (128 KiB) per workgroup for decoded literals;
// NULL = a per-stream buffer kept by the library.
// mode: -1 the library's choice (strom_zstd_fp_mode / stream count), 0 one
// wave per stream, 1 frame-parallel — a caller that runs several decodes
// at once (the Arrow scan's slot streams) may want every one of them to
// take part of the chip rather than all of it.
extern "C" int strom_decompress_zstd_mode(int codec, const void *d_src, void *d_dst,
                                          const strom_decomp_desc *d_desc, uint32_t nstreams,
                                          int32_t *d_status, void *scratch,
                                          uint64_t scratch_bytes, void *stream, int mode) {
  using namespace zs;
  if (codec != STROM_CODEC_ZSTD && codec != STROM_CODEC_ARROW_ZSTD) return -22;
  if (mode < -1 || mode > 1) return -22;
  if (!nstreams) return 0;
  // a caller's scratch too small for one frame-parallel workgroup keeps
  // the wave-per-stream decoder
  const bool fp = (mode < 0 ? use_fp(nstreams) : mode == 1) &&
                  (!scratch || scratch_bytes >= fp_scratch(FPW));
  const size_t per_wg = fp ? fp_scratch(FPW) : SLOT;
  const uint32_t res = fp ? cu_count() * fp_per_cu() : resident_groups();
  uint32_t grid = nstreams < res ? nstreams : res;
  if (grid > 65535) grid = 65535;
  uint8_t *sc = (uint8_t *)scratch;
  std::unique_lock<std::mutex> g(g_mu, std::defer_lock);
  if (sc) {
    const uint64_t slots = scratch_bytes / per_wg;
    if (!slots) return -22;
    if (grid > slots) grid = (uint32_t)slots;
  } else {
    g.lock();                  // held through the launch (scratch_for)
    sc = scratch_for(stream, (size_t)grid * per_wg);
    if (!sc) return -12;
  }
  if (fp)
    hipLaunchKernelGGL(zstd_fp_kernel, dim3(grid), dim3(NT * FPW), 0, (hipStream_t)stream, codec,
                       (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nstreams, d_status, sc);
  else
    hipLaunchKernelGGL(zstd_kernel, dim3(grid), dim3(NT), 0, (hipStream_t)stream, codec,
                       (const uint8_t *)d_src, (uint8_t *)d_dst, d_desc, nstreams, d_status, sc);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int strom_decompress_zstd(int codec, const void *d_src, void *d_dst,
                                     const strom_decomp_desc *d_desc, uint32_t nstreams,
                                     int32_t *d_status, void *scratch, uint64_t scratch_bytes,
                                     void *stream) {
  return strom_decompress_zstd_mode(codec, d_src, d_dst, d_desc, nstreams, d_status, scratch,
                                    scratch_bytes, stream, -1);
}

extern "C" uint32_t strom_zstd_lds_bytes(void) { return (uint32_t)sizeof(zs::Smem); }

// (device, stream) buffers the library keeps (literal slots, LP entry
// pools): a caller decoding on more streams than this in turn evicts a
// pool per decode
extern "C" uint32_t strom_zstd_scratch_keep(void) { return (uint32_t)zs::kScratchKeep; }

// frame-parallel workgroups (streams) resident per CU
extern "C" uint32_t strom_zstd_fp_per_cu(void) { return zs::fp_per_cu(); }

// Decoder choice: -1 by the stream count (default), 0 wave per stream,
// 1 frame-parallel.  Returns the previous setting.
extern "C" int strom_zstd_fp_mode(int mode) {
  const int prev = zs::fp_mode();
  if (mode >= -1 && mode <= 1) zs::g_fp_mode.store(mode);
  return prev;
}

// scratch bytes per workgroup of each decoder (callers passing their own
// scratch size it for the grid): {wave-per-stream, frame-parallel}
extern "C" void strom_zstd_scratch_sizes(uint64_t *out) {
  out[0] = zs::SLOT;
  out[1] = zs::fp_scratch(zs::FPW);
}

// Free the literal scratch kept per (device, stream) (128 KiB per resident
// workgroup, up to ~290 MiB per stream, at most kScratchKeep streams):
// after the streams' last decodes.
extern "C" int strom_zstd_release(void) {
  std::lock_guard<std::mutex> g(zs::g_mu);
  int rc = 0;
  for (auto &kv : zs::g_scratch) {
    if (!kv.second.p) continue;
    if (hipStreamSynchronize((hipStream_t)kv.first.stream) != hipSuccess) rc = -5;
    if (hipFree(kv.second.p) != hipSuccess) rc = -5;
  }
  zs::g_scratch.clear();
  return rc;
}

#ifdef ZS_PROF
// read (and zero) the phase profile: out[kZpN] (cycles per phase, counts)
extern "C" int strom_zstd_prof(uint64_t *out) {
  unsigned long long h[zs::kZpN] = {0};
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(zs::g_zprof), sizeof h) != hipSuccess) return -5;
  unsigned long long z[zs::kZpN] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(zs::g_zprof), z, sizeof z);
  for (int i = 0; i < zs::kZpN; ++i) out[i] = h[i];
  return zs::kZpN;
}
#endif

// The same phases lane by lane on the CPU: the algorithm's reference
// (tests/test_codecs_cpu.py), no GPU involved.  Returns decoded bytes or a
// negative error as the kernel's status.
static thread_local uint32_t g_fp_host_stats[2];
// groups and blocks decoded ahead by the last strom_zstd_host_fp call
extern "C" void strom_zstd_host_fp_stats(uint32_t *out) {
  out[0] = g_fp_host_stats[0];
  out[1] = g_fp_host_stats[1];
}

// The frame-parallel decoder's phases on the CPU, waves one after another
// (nw blocks per group, 2..NWMAX).
extern "C" int strom_zstd_host_fp(int codec, const uint8_t *src, uint32_t src_len, uint8_t *dst,
                                  uint32_t cap, uint32_t nw) {
  using namespace zs;
  if (codec != STROM_CODEC_ZSTD && codec != STROM_CODEC_ARROW_ZSTD) return -22;
  if (nw < 2 || nw > NWMAX) return -22;
  std::unique_ptr<Smem[]> sm(new Smem[nw]());
  std::unique_ptr<FpShared> f(new FpShared());
  std::unique_ptr<uint8_t[]> sc(new uint8_t[fp_scratch(nw)]);
  const FpCtx x{Ctx{src, dst, sc.get(), src_len, cap}, sc.get(), nw};
  HostGroup g;
  g.nw = nw;
  run_fp(g, sm.get(), *f, x, codec);
  g_fp_host_stats[0] = g.groups;
  g_fp_host_stats[1] = g.blocks_par;
  return sm[0].err ? sm[0].err : (int32_t)sm[0].op;
}

extern "C" int strom_zstd_host(int codec, const uint8_t *src, uint32_t src_len, uint8_t *dst,
                               uint32_t cap) {
  using namespace zs;
  if (codec != STROM_CODEC_ZSTD && codec != STROM_CODEC_ARROW_ZSTD) return -22;
  std::unique_ptr<Smem> s(new Smem());
  std::unique_ptr<uint8_t[]> lit(new uint8_t[SLOT]);
  HostTeam tm;
  const Ctx c{src, dst, lit.get(), src_len, cap};
  run(tm, *s, c, codec);
  return s->err ? s->err : (int32_t)s->op;
}

// Lane-parallel zstd decode (see the "lane-parallel" section): walk, entropy
// and exec launches on `stream`.  dst_bytes: the decoded capacity of all
// streams together (sizes the entry pool: STROM_ZSTD_LP_ENT x dst_bytes;
// streams that do not fit are decoded by the serial decoder in the exec
// launch).  The pool is library-kept per (device, stream).
extern "C" int strom_decompress_zstd_lp(int codec, const void *d_src, void *d_dst,
                                        const strom_decomp_desc *d_desc, uint32_t nstreams,
                                        int32_t *d_status, uint64_t dst_bytes, void *stream) {
  using namespace zs;
  if (codec != STROM_CODEC_ZSTD && codec != STROM_CODEC_ARROW_ZSTD) return -22;
  if (!nstreams) return 0;
  const uint32_t cus = cu_count();
  uint32_t xgrid = cus * lp_exec_per_cu();
  if (xgrid > nstreams) xgrid = nstreams;
  // the serial fallback's workgroups (each a 128 KiB literal slot)
  uint32_t sgrid = cus * 2;
  if (sgrid > nstreams) sgrid = nstreams;
  const uint64_t bc = dst_bytes / 32768 + 4ull * nstreams + 64;
  const uint32_t blk_cap = bc > 0x7fffffffull ? 0x7fffffffu : (uint32_t)bc;
  const uint64_t ent_cap = lp_up((uint64_t)(lp_ent_factor() * (double)dst_bytes) + (1 << 20), 256);
  const LpLayout l = lp_layout(nstreams, blk_cap, sgrid, ent_cap);
  std::lock_guard<std::mutex> g(g_mu);          // held through the launches (scratch_for)
  uint8_t *pool = scratch_for(stream, l.total, 1);
  if (!pool) return -12;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(pool, 0, sizeof(LpHdr), s) != hipSuccess) return -5;
  hipLaunchKernelGGL(zstd_lp_walk, dim3((nstreams + LP_WALK_T - 1) / LP_WALK_T), dim3(LP_WALK_T), 0, s,
                     codec, (const uint8_t *)d_src, d_desc, nstreams, pool, l);
  // enough waves for every listed block in one or two resident rounds
  uint32_t lgrid = cus * lp_lit_per_cu(), sgrid2 = cus * lp_seq_per_cu();
  if (lgrid > (blk_cap + LPLB - 1) / LPLB) lgrid = (blk_cap + LPLB - 1) / LPLB;
  if (sgrid2 > (blk_cap + LPSB - 1) / LPSB) sgrid2 = (blk_cap + LPSB - 1) / LPSB;
  hipLaunchKernelGGL(zstd_lp_lit, dim3(lgrid), dim3(NT), 0, s, (const uint8_t *)d_src,
                     (uint8_t *)d_dst, d_desc, pool, l);
  hipLaunchKernelGGL(zstd_lp_seq, dim3(sgrid2), dim3(NT), 0, s, (const uint8_t *)d_src, d_desc,
                     pool, l);
  hipLaunchKernelGGL(zstd_lp_exec, dim3(xgrid), dim3(LPX_T), 0, s, (const uint8_t *)d_src,
                     (uint8_t *)d_dst, d_desc, nstreams, d_status, pool, l);
  hipLaunchKernelGGL(zstd_lp_serial, dim3(sgrid), dim3(NT), 0, s, codec, (const uint8_t *)d_src,
                     (uint8_t *)d_dst, d_desc, nstreams, d_status, pool, l);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// The last LP launch's counters on `stream` (synchronizes it): {blocks
// listed, streams the LP path decoded, entry bytes used, pool bytes}.
extern "C" int strom_zstd_lp_last(void *stream, uint64_t *out) {
  using namespace zs;
  std::lock_guard<std::mutex> g(g_mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -5;
  auto it = g_scratch.find(ScratchKey{dev, stream, 1});
  if (it == g_scratch.end() || !it->second.p) return -2;
  LpHdr h{};
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess ||
      hipMemcpy(&h, it->second.p, sizeof h, hipMemcpyDeviceToHost) != hipSuccess)
    return -5;
  out[0] = h.nblk;
  out[1] = h.lp_done;
  out[2] = h.ent_used;
  out[3] = it->second.bytes;
  return 0;
}

// LP geometry: {LDS bytes per sequence wave, its blocks, its waves per CU,
// exec workgroups per CU, LDS bytes per literal wave, its blocks, its waves
// per CU, 0}
extern "C" void strom_zstd_lp_info(uint32_t *out) {
  out[0] = (uint32_t)sizeof(zs::LpSWave);
  out[1] = zs::LPSB;
  out[2] = zs::lp_seq_per_cu();
  out[3] = zs::lp_exec_per_cu();
  out[4] = (uint32_t)sizeof(zs::LpLWave);
  out[5] = zs::LPLB;
  out[6] = zs::lp_lit_per_cu();
  out[7] = 0;
}

// The LP decoder's three phases on the CPU (host buffers): every stream
// walked, the block list's groups entropy-decoded lane by lane, every
// stream executed — the algorithm's reference for the kernels.  status[i]:
// decoded bytes or an error; returns the number of streams the LP path
// decoded (the rest went to the serial decoder: refused by the walk, or an
// LP error).
extern "C" int strom_zstd_host_lp(int codec, const uint8_t *src, const strom_decomp_desc *desc,
                                  uint32_t n, uint8_t *dst, int32_t *status, double ent_factor) {
  using namespace zs;
  if (codec != STROM_CODEC_ZSTD && codec != STROM_CODEC_ARROW_ZSTD) return -22;
  if (!n) return 0;
  uint64_t dst_bytes = 0;
  for (uint32_t i = 0; i < n; ++i) dst_bytes += desc[i].dst_len;
  const uint64_t bc = dst_bytes / 32768 + 4ull * n + 64;
  const uint64_t ent_cap = lp_up((uint64_t)((ent_factor > 0 ? ent_factor : 3.0) * (double)dst_bytes) + 4096, 256);
  const LpLayout l = lp_layout(n, (uint32_t)bc, 1, ent_cap);
  std::unique_ptr<uint8_t[]> pool(new uint8_t[l.total]());
  std::unique_ptr<LpWalk> ws(new LpWalk());
  for (uint32_t i = 0; i < n; ++i) {
    const Ctx c{src + desc[i].src_off, nullptr, nullptr, desc[i].src_len, desc[i].dst_len};
    lp_walk_stream<LpHostAtom>(*ws, c, codec, i, pool.get(), l);
  }
  const LpHdr &h = *(const LpHdr *)pool.get();
  const uint32_t nlist = h.nblk < l.blk_cap ? h.nblk : l.blk_cap;
  LpBlock *blk = (LpBlock *)(pool.get() + l.blocks);
  std::unique_ptr<LpLWave> WL(new LpLWave());
  std::unique_ptr<LpSWave> WS(new LpSWave());
  HostTeam tm;
  for (uint32_t k0 = 0; k0 < nlist; k0 += LPLB) lp_lit_group(tm, *WL, blk, k0, nlist, src, dst, desc);
  for (uint32_t k0 = 0; k0 < nlist; k0 += LPSB)
    lp_seq_group(tm, *WS, blk, k0, nlist, src, desc, pool.get() + l.ents);
  std::unique_ptr<LpX> x(new LpX());
  std::unique_ptr<Smem> sm(new Smem());
  HostTeam tx;
  tx.n = LPX_T;
  HostTeam t1;
  const LpStream *st = (const LpStream *)(pool.get() + l.streams);
  uint8_t *slot = pool.get() + l.slots;
  int taken = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const Ctx c{src + desc[i].src_off, dst + desc[i].dst_off, nullptr, desc[i].src_len,
                desc[i].dst_len};
    status[i] = lp_exec_stream(tx, *x, st[i], blk, pool.get() + l.ents, c);
    taken += status[i] != kLpRedo;
  }
  for (uint32_t i = 0; i < n; ++i) {
    if (status[i] != kLpRedo) continue;
    const Ctx c{src + desc[i].src_off, dst + desc[i].dst_off, slot, desc[i].src_len,
                desc[i].dst_len};
    run(t1, *sm, c, codec);
    status[i] = sm->err ? sm->err : (int32_t)sm->op;
  }
  return taken;
}
