// heapscan.hip — PostgreSQL heap pages scanned on the GPU.
//
// The reference's PostgreSQL CustomScan loads heap blocks into a DMA buffer
// and then walks line pointers on the CPU (pgsql/nvme_strom.c:1054-1092:
// nvmestrom_next_tuple), with visibility handled per tuple for blocks that
// came through the buffer manager (:896-940) and all-visible blocks taken as
// they are (:870-891).  On MI355X the loaded pages sit in HBM and one
// wavefront per page does all of it, from an LDS copy of the page:
//   0. the page is staged into LDS with coalesced 16-B loads (one 1 KiB
//      wave-instruction per 1 KiB of page); the NEXT page's loads are issued
//      before the current page is parsed, so HBM latency hides under the
//      parse (every later access — header, checksum columns, line pointers,
//      tuple headers, column values — is an LDS access);
//   1. page header sanity (pd_lower/pd_upper/pd_special bounds, flag bits,
//      page size) — PageIsVerified-style;
//   2. optional data checksum (pg_checksum_page: 32 interleaved FNV-1a
//      sums = 32 lanes, one column of uint32 words each, conflict-free
//      ds_read_b32 across the lanes of a row);
//   3. line pointers 64 at a time (one per lane): LP_NORMAL items, optional
//      visibility (PD_ALL_VISIBLE page: every tuple; else xmin known
//      committed — frozen xmin included — and xmax invalid or lock-only),
//      and an optional range predicate on a fixed-offset int4/int8 column;
//      the per-64 ballot masks are parked in LDS;
//   4. output reservation once per WORKGROUP (4 waves x 8 pages): the waves'
//      counts are summed in LDS and thread 0 does a single atomicAdd, then
//      each wave replays its masks to write (page << 16 | lineno) item ids.
//
// strom_heap_scan2 replaces the fixed-offset predicate of step 3 with what
// ExecScan does for the reference (pgsql/nvme_strom.c:1137-1143): every lane
// deforms its tuple in LDS with a tuple descriptor — null bitmap, attalign
// padding, fixed lengths, 1-byte / 4-byte / TOAST-pointer varlena headers,
// attcacheoff shortcuts for null-free tuples — and evaluates an AND-list of
// qualifiers (int / float ranges, IN lists, IS [NOT] NULL, text equality and
// prefix).  Quals are sorted by attribute, so one walk per tuple serves them
// all.  strom_heap_project gathers one attribute of the selected tuples with
// the same deformer, reading the pages in HBM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "strom/strom.h"

namespace {

// pg_checksum's per-lane FNV offsets (checksum_impl.h, checksumBaseOffsets)
__constant__ uint32_t g_pg_base[32] = {
    0x5B1F36E9, 0xB8525960, 0x02AB50AA, 0x1DE66D2A, 0x79FF467A, 0x9BB9F8A3, 0x217E7CD2,
    0x83E13D2C, 0xF8D4474F, 0xE39EB970, 0x42C6AE16, 0x993216FA, 0x7B093B5D, 0x98DAFF3C,
    0xF718902A, 0x0B1C9CDB, 0xE58F764B, 0x187636BC, 0x5D7B3BB1, 0xE73DE7DE, 0x92BEC979,
    0xCCA6C0B2, 0x304A0979, 0x85AA43D4, 0x783125BB, 0x6CA8EAA2, 0xE407EAC6, 0x4B5CFC3E,
    0x9FBF8C76, 0x15CA20BE, 0xF2CA9FFF, 0x3ED50F2B};

constexpr uint32_t kSizeOfPageHeader = 24;
constexpr uint32_t kLpNormal = 1;
constexpr uint32_t kHeapHasNull = 0x0001;
constexpr uint32_t kXmaxLockOnly = 0x0080;
constexpr uint32_t kXminCommitted = 0x0100;   // also set in a frozen xmin (0x0300)
constexpr uint32_t kXmaxInvalid = 0x0800;
constexpr uint32_t kPdAllVisible = 0x0004;
constexpr int kWaves = 4;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t fnv_mix(uint32_t s, uint32_t v) {
  uint32_t t = s ^ v;
  return t * 16777619u ^ (t >> 17);
}

// little-endian reads from the LDS page image.  Tuple offsets are MAXALIGNed
// but user columns need not be 4-aligned, so wide reads are assembled from
// the two aligned words around them.
__device__ __forceinline__ uint32_t lds_u32a(const uint8_t *pg, uint32_t off) {
  return *(const uint32_t *)(pg + off);  // off % 4 == 0
}
__device__ __forceinline__ uint32_t lds_u32(const uint8_t *pg, uint32_t off) {
  const uint32_t sh = (off & 3) * 8;
  const uint32_t lo = lds_u32a(pg, off & ~3u);
  if (!sh) return lo;
  const uint32_t hi = lds_u32a(pg, (off & ~3u) + 4);
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
}

struct PageHdr {
  uint32_t checksum, flags, lower, upper, special, psv;
};

__device__ __forceinline__ PageHdr read_hdr(const uint8_t *pg) {
  PageHdr h;
  const uint32_t w2 = lds_u32a(pg, 8), w3 = lds_u32a(pg, 12), w4 = lds_u32a(pg, 16);
  h.checksum = w2 & 0xffff;
  h.flags = w2 >> 16;
  h.lower = w3 & 0xffff;
  h.upper = w3 >> 16;
  h.special = w4 & 0xffff;
  h.psv = w4 >> 16;
  return h;
}

// page header check + optional checksum; returns STROM_PAGE_* bits
__device__ uint32_t page_status(const strom_heap_scan_args &a, const uint8_t *pg,
                                const PageHdr &h, uint32_t page_no, uint32_t lane) {
  if (h.upper == 0) return STROM_PAGE_EMPTY;
  if (h.lower < kSizeOfPageHeader || h.lower > h.upper || h.upper > h.special ||
      h.special > a.page_sz || (h.special & 7) || (h.flags & ~0x7u) ||
      (h.psv & 0xFF00u) != (a.page_sz & 0xFF00u))
    return STROM_PAGE_BAD_HEADER;
  if (!(a.flags & STROM_HEAP_VERIFY_CHECKSUM)) return 0;
  // lanes 0..31 own one FNV sum each (lanes 32..63 duplicate and are
  // ignored); lane j reads column j of each 128-B row: 32 consecutive words
  const uint32_t j = lane & 31;
  const uint32_t *w = (const uint32_t *)pg;
  uint32_t s = g_pg_base[j];
  const uint32_t rows = a.page_sz / 128;
  {
    uint32_t v = w[j];
    if (j == 2) v &= 0xffff0000u;  // pd_checksum reads as zero
    s = fnv_mix(s, v);
  }
  for (uint32_t r = 1; r < rows; ++r) s = fnv_mix(s, w[r * 32 + j]);
  s = fnv_mix(s, 0);
  s = fnv_mix(s, 0);
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) s ^= __shfl_xor(s, o, 64);
  const uint32_t blkno = a.blknos ? a.blknos[page_no] : a.blkno_base + page_no;
  const uint32_t c = ((s ^ blkno) % 65535u) + 1u;
  return (c & 0xffffu) != h.checksum ? STROM_PAGE_BAD_CHECKSUM : 0u;
}

// ---------------------------------------------------------------- deformer
__device__ __forceinline__ uint32_t align_up(uint32_t off, uint32_t al) {
  return (off + al - 1) & ~(al - 1);
}

// TOAST pointer payload size by vartag (postgres.h VARTAG_SIZE): indirect
// and expanded pointers are 8 bytes, an on-disk varatt_external 16
__device__ __forceinline__ uint32_t vartag_size(uint32_t tag) {
  return tag == 18 ? 16u : (tag >= 1 && tag <= 3) ? 8u : 0u;
}

// One tuple's attribute walk.  `t` points at the tuple (LDS page image or
// HBM), offsets are from the tuple start; attributes are visited in
// increasing order (quals are sorted by attno on the host).
struct Deform {
  const uint8_t *t;
  uint32_t tlen, hoff, natts;   // natts stored in this tuple (t_infomask2)
  bool hasnull, bad;
  uint32_t next, off;           // next attribute to pass, where its storage may start
};

struct Att {
  uint32_t off, len, hdr;       // datum offset, total bytes, varlena header bytes
  bool null, ext;               // ext: compressed or out-of-line varlena
};

__device__ __forceinline__ Deform deform_init(const uint8_t *t, uint32_t tlen) {
  Deform s;
  s.t = t;
  s.tlen = tlen;
  const uint32_t w16 = lds_u32(t, 16), w20 = lds_u32(t, 20);
  s.natts = (w16 >> 16) & 0x7ff;
  s.hasnull = (w20 & kHeapHasNull) != 0;
  s.hoff = (w20 >> 16) & 0xff;
  s.bad = s.hoff < 23 || s.hoff > tlen || (s.hasnull && 23 + ((s.natts + 7) >> 3) > s.hoff);
  s.next = 0;
  s.off = s.hoff;
  return s;
}

__device__ __forceinline__ Att deform_to(const strom_heap_tupdesc &d, Deform &s, uint32_t k) {
  Att a;
  a.off = a.len = a.hdr = 0;
  a.null = true;
  a.ext = false;
  if (s.bad) return a;
  if (k >= s.natts) {             // not stored (added later): NULL
    s.next = k + 1;
    return a;
  }
  if (!s.hasnull && d.cacheoff[k] >= 0 && d.attlen[k] > 0) {
    // attcacheoff: every earlier attribute is fixed-length and none is null
    a.off = s.hoff + (uint32_t)d.cacheoff[k];
    a.len = (uint32_t)d.attlen[k];
    a.null = false;
    if (a.off + a.len > s.tlen) s.bad = true;
    s.next = k + 1;
    s.off = a.off + a.len;
    return a;
  }
  for (uint32_t i = s.next; i <= k; ++i) {
    if (s.hasnull && !((s.t[23 + (i >> 3)] >> (i & 7)) & 1)) continue;  // NULL: no storage
    const int len = d.attlen[i];
    uint32_t o = s.off, L = 0, H = 0;
    bool E = false;
    if (len > 0) {
      o = align_up(o, d.attalign[i]);
      L = (uint32_t)len;
    } else if (len == -1) {
      if (o >= s.tlen) { s.bad = true; return a; }
      uint32_t b = s.t[o];
      if (b == 0) {               // a pad byte: the datum is an aligned 4-byte header
        o = align_up(o, d.attalign[i]);
        if (o >= s.tlen) { s.bad = true; return a; }
        b = s.t[o];
      }
      if ((b & 1) == 0) {         // 4-byte header; (b & 3) == 2: compressed inline
        if (o + 4 > s.tlen) { s.bad = true; return a; }
        L = (lds_u32(s.t, o) >> 2) & 0x3fffffffu;
        H = 4;
        E = (b & 3) == 2;
      } else if (b == 1) {        // 1-byte header 0x01: TOAST pointer, tag next
        if (o + 2 > s.tlen) { s.bad = true; return a; }
        const uint32_t ts = vartag_size(s.t[o + 1]);
        if (!ts) { s.bad = true; return a; }
        L = 2 + ts;
        H = 2;
        E = true;
      } else {                    // 1-byte header: short inline value
        L = b >> 1;
        H = 1;
      }
    } else {                      // cstring: bytes up to and including NUL
      uint32_t e = o;
      while (e < s.tlen && s.t[e]) ++e;
      L = e - o + 1;
    }
    if (L < H || o + L > s.tlen) { s.bad = true; return a; }
    s.off = o + L;
    if (i == k) {
      a.off = o;
      a.len = L;
      a.hdr = H;
      a.null = false;
      a.ext = E;
    }
  }
  s.next = k + 1;
  return a;
}

__device__ __forceinline__ int64_t att_int(const uint8_t *t, const Att &a) {
  switch (a.len) {
    case 1: return (int8_t)t[a.off];
    case 2: return (int16_t)(t[a.off] | (t[a.off + 1] << 8));
    case 4: return (int32_t)lds_u32(t, a.off);
    default: return (int64_t)((uint64_t)lds_u32(t, a.off) | ((uint64_t)lds_u32(t, a.off + 4) << 32));
  }
}

__device__ __forceinline__ double att_float(const uint8_t *t, const Att &a) {
  if (a.len == 4) return (double)__uint_as_float(lds_u32(t, a.off));
  return __longlong_as_double((long long)att_int(t, a));
}

// PostgreSQL float ordering: NaN equals NaN and sorts above every number
__device__ __forceinline__ bool pg_le(double x, double y) {
  if (isnan(y)) return true;
  if (isnan(x)) return false;
  return x <= y;
}

// 1 keep, 0 drop, 2 undecidable here (text qual on a compressed / TOAST value)
__device__ __forceinline__ int eval_quals(const strom_heap_scan2_args &g, const uint8_t *t,
                                          uint32_t tlen) {
  Deform s = deform_init(t, tlen);
  Att a;
  int last = -1;
  int verdict = 1;
  for (int qi = 0; qi < g.nquals; ++qi) {
    const strom_heap_qual &q = g.quals[qi];
    if (q.attno != last) {
      a = deform_to(g.desc, s, (uint32_t)q.attno);
      last = q.attno;
    }
    if (s.bad) return 0;
    if (q.kind == STROM_QUAL_IS_NULL) {
      if (!a.null) return 0;
      continue;
    }
    if (a.null) return 0;
    switch (q.kind) {
      case STROM_QUAL_NOT_NULL:
        break;
      case STROM_QUAL_INT_RANGE: {
        const int64_t v = att_int(t, a);
        if (v < q.lo || v > q.hi) return 0;
        break;
      }
      case STROM_QUAL_INT_IN: {
        const int64_t v = att_int(t, a);
        bool hit = false;
        for (uint32_t k = 0; k < q.nconst && k < 4; ++k) {
          int64_t c;
          __builtin_memcpy(&c, q.cbytes + 8 * k, 8);
          hit |= v == c;
        }
        if (!hit) return 0;
        break;
      }
      case STROM_QUAL_FLOAT_RANGE: {
        const double v = att_float(t, a);
        if (!pg_le(__longlong_as_double(q.lo), v) || !pg_le(v, __longlong_as_double(q.hi))) return 0;
        break;
      }
      case STROM_QUAL_TEXT_EQ:
      case STROM_QUAL_TEXT_PREFIX: {
        if (a.ext) {              // keep checking: a later qual may still reject it
          verdict = 2;
          break;
        }
        const uint32_t n = a.len - a.hdr;
        if (q.kind == STROM_QUAL_TEXT_EQ ? n != q.nconst : n < q.nconst) return 0;
        for (uint32_t k = 0; k < q.nconst; ++k)
          if (t[a.off + a.hdr + k] != q.cbytes[k]) return 0;
        break;
      }
      default:
        return 0;
    }
  }
  return verdict;
}

// ---- qualifier programs (strom_heap_qual2): CNF over any number of quals,
// constants in a device pool.  Three-valued like SQL's quals over values
// the GPU cannot read (compressed / TOAST varlena): a clause with no true
// qual and an undecidable one is undecidable; the tuple is dropped by a
// false clause, else undecidable (page flagged for a host recheck) if any
// clause is.
// The pool through the constant address space (never written while the
// kernel runs): wave-uniform dword reads are scalar loads.  Every constant
// starts 8-aligned and the pool is padded to 8 bytes (ops/heapscan.Program).
typedef const __attribute__((address_space(4))) uint8_t cu8;
typedef const __attribute__((address_space(4))) uint32_t cu32;
__device__ __forceinline__ uint32_t pool_u32(cu8 *p, uint32_t o) {   // o % 4 == 0
  return *(cu32 *)(p + o);
}
__device__ __forceinline__ uint32_t pool_u16(cu8 *p, uint32_t o) {   // o % 2 == 0
  return (pool_u32(p, o & ~3u) >> ((o & 2) * 8)) & 0xffff;
}

// A PostgreSQL numeric (numeric.c on-disk: NumericShort / NumericLong /
// special values) or a pool constant in the same normalized terms.
struct Num {
  uint32_t kind;     // 0 finite, 1 NaN, 2 +inf, 3 -inf
  uint32_t neg;
  int32_t weight;    // digits[0] x 10000^weight
  uint32_t nd;       // digits
  const uint8_t *dig;  // int16 little-endian base-10000 digits
};

__device__ __forceinline__ bool num_of_datum(const uint8_t *t, const Att &a, Num &n) {
  const uint32_t len = a.len - a.hdr;
  const uint8_t *d = t + a.off + a.hdr;
  if (len < 2) return false;
  const uint32_t h = (uint32_t)d[0] | ((uint32_t)d[1] << 8);
  n.kind = 0;
  n.neg = 0;
  if ((h & 0xC000) == 0xC000) {               // NUMERIC_SPECIAL
    const uint32_t sp = h & 0xF000;
    n.kind = sp == 0xC000 ? 1 : sp == 0xD000 ? 2 : sp == 0xF000 ? 3 : 9;
    n.nd = 0;
    return n.kind != 9;
  }
  if ((h & 0xC000) == 0x8000) {               // NUMERIC_SHORT
    n.neg = (h & 0x2000) != 0;
    n.weight = (h & 0x0040) ? (int32_t)(h | ~0x3Fu) : (int32_t)(h & 0x3F);
    n.nd = (len - 2) / 2;
    n.dig = d + 2;
    return ((len - 2) & 1) == 0;
  }
  if (len < 4) return false;                  // NumericLong
  n.neg = (h & 0xC000) == 0x4000;
  n.weight = (int16_t)((uint32_t)d[2] | ((uint32_t)d[3] << 8));
  n.nd = (len - 4) / 2;
  n.dig = d + 4;
  return ((len - 4) & 1) == 0;
}

__device__ __forceinline__ Num num_of_pool(cu8 *p, uint32_t o) {
  Num n;
  n.kind = pool_u16(p, o);
  n.neg = pool_u16(p, o + 2);
  n.weight = (int16_t)pool_u16(p, o + 4);
  n.nd = pool_u16(p, o + 6);
  n.dig = (const uint8_t *)(p + o + 8);
  return n;
}

__device__ __forceinline__ int32_t num_digit(const Num &n, uint32_t i) {
  return (int16_t)((uint32_t)n.dig[2 * i] | ((uint32_t)n.dig[2 * i + 1] << 8));
}

// cmp_abs_common (numeric.c): |a| vs |b|
__device__ __forceinline__ int num_cmp_abs(const Num &a, const Num &b) {
  uint32_t i1 = 0, i2 = 0;
  int32_t w1 = a.weight, w2 = b.weight;
  while (w1 > w2 && i1 < a.nd) {
    if (num_digit(a, i1++) != 0) return 1;
    --w1;
  }
  while (w2 > w1 && i2 < b.nd) {
    if (num_digit(b, i2++) != 0) return -1;
    --w2;
  }
  if (w1 == w2) {
    while (i1 < a.nd && i2 < b.nd) {
      const int32_t d = num_digit(a, i1++) - num_digit(b, i2++);
      if (d) return d > 0 ? 1 : -1;
    }
  }
  while (i1 < a.nd)
    if (num_digit(a, i1++) != 0) return 1;
  while (i2 < b.nd)
    if (num_digit(b, i2++) != 0) return -1;
  return 0;
}

__device__ __forceinline__ bool num_zero(const Num &n) {
  for (uint32_t i = 0; i < n.nd; ++i)
    if (num_digit(n, i)) return false;
  return true;
}

// cmp_numerics: NaN equals NaN and sorts above everything, +inf above every
// finite value, -inf below; finite values by sign, then magnitude
__device__ __forceinline__ int num_cmp(const Num &a, const Num &b) {
  auto rank = [](const Num &n) { return n.kind == 1 ? 3 : n.kind == 2 ? 2 : n.kind == 3 ? 0 : 1; };
  const int ra = rank(a), rb = rank(b);
  if (ra != rb) return ra < rb ? -1 : 1;
  if (ra != 1) return 0;
  const bool za = num_zero(a), zb = num_zero(b);
  if (za || zb) {
    if (za && zb) return 0;
    if (za) return b.neg ? 1 : -1;
    return a.neg ? -1 : 1;
  }
  if (a.neg != b.neg) return a.neg ? -1 : 1;
  const int m = num_cmp_abs(a, b);
  return a.neg ? -m : m;
}

// n bytes of a tuple vs a pool constant (8-aligned, read a dword at a time)
__device__ __forceinline__ bool bytes_eq(const uint8_t *x, cu8 *y, uint32_t n) {
  for (uint32_t k = 0; k < n; k += 4) {
    const uint32_t w = *(cu32 *)(y + k);
    const uint32_t m = n - k;
    for (uint32_t b = 0; b < 4 && b < m; ++b)
      if (x[k + b] != ((w >> (8 * b)) & 0xff)) return false;
  }
  return true;
}

// one qual of a program on attribute a: 1 true, 0 false, 2 undecidable
__device__ __forceinline__ int eval_qual2(const strom_heap_qual2 &q, cu8 *pool,
                                          const uint8_t *t, const Att &a) {
  if (q.flags & STROM_QUAL2_FALSE) return 0;
  if (q.kind == STROM_QUAL_IS_NULL) return a.null ? 1 : 0;
  if (a.null) return 0;
  switch (q.kind) {
    case STROM_QUAL_NOT_NULL:
      return 1;
    case STROM_QUAL_INT_RANGE: {
      const int64_t v = att_int(t, a);
      return v >= q.lo && v <= q.hi;
    }
    case STROM_QUAL_INT_IN: {
      const int64_t v = att_int(t, a);
      for (uint32_t k = 0; k < q.nconst; ++k) {
        const int64_t c = (int64_t)((uint64_t)pool_u32(pool, q.coff + 8 * k) |
                                    ((uint64_t)pool_u32(pool, q.coff + 8 * k + 4) << 32));
        if (v == c) return 1;
      }
      return 0;
    }
    case STROM_QUAL_FLOAT_RANGE: {
      const double v = att_float(t, a);
      return pg_le(__longlong_as_double(q.lo), v) && pg_le(v, __longlong_as_double(q.hi));
    }
    case STROM_QUAL_TEXT_EQ:
    case STROM_QUAL_TEXT_PREFIX:
    case STROM_QUAL_TEXT_IN: {
      if (a.ext) return 2;
      const uint32_t n = a.len - a.hdr;
      const uint8_t *v = t + a.off + a.hdr;
      if (q.kind == STROM_QUAL_TEXT_EQ) return n == q.nconst && bytes_eq(v, pool + q.coff, n);
      if (q.kind == STROM_QUAL_TEXT_PREFIX) return n >= q.nconst && bytes_eq(v, pool + q.coff, q.nconst);
      for (uint32_t k = 0; k < q.nconst; ++k) {
        const uint32_t co = pool_u32(pool, q.coff + 8 * k), cl = pool_u32(pool, q.coff + 8 * k + 4);
        if (n == cl && bytes_eq(v, pool + co, n)) return 1;
      }
      return 0;
    }
    case STROM_QUAL_NUMERIC_RANGE: {
      if (a.ext) return 2;
      Num v;
      if (!num_of_datum(t, a, v)) return 0;
      if (!(q.flags & 1)) {
        const int c = num_cmp(v, num_of_pool(pool, (uint32_t)q.lo));
        if (c < 0 || (c == 0 && (q.flags & 4))) return 0;
      }
      if (!(q.flags & 2)) {
        const int c = num_cmp(v, num_of_pool(pool, (uint32_t)q.hi));
        if (c > 0 || (c == 0 && (q.flags & 8))) return 0;
      }
      return 1;
    }
    default:
      return 0;
  }
}

// the program over one tuple: 1 keep, 0 drop, 2 undecidable.  The loop
// over quals stays uniform across the wave (a decided lane only stops
// evaluating; the wave leaves when every lane has decided), and the program
// is read through the constant address space, so its entries are scalar
// loads (profiles/r5/heap/prog_kbench.md)
__device__ __forceinline__ int eval_prog(const strom_heap_scan2_args &g, const uint8_t *t,
                                         uint32_t tlen) {
  Deform s = deform_init(t, tlen);
  Att a;
  a.off = a.len = a.hdr = 0;
  a.null = true;
  a.ext = false;
  int last = -1;
  int verdict = s.bad ? 0 : 1;
  bool live = verdict != 0;
  // the program through the constant address space: it is never written
  // while the kernel runs, so its wave-uniform reads become scalar loads
  // (a generic pointer next to the kernel's own stores gets per-lane vector
  // loads).  One 32-byte s_load per qual, the next one issued before the
  // current qual is evaluated.
  typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
  typedef const __attribute__((address_space(4))) u32x8 cq8;
  static_assert(sizeof(strom_heap_qual2) == 32, "one s_load_dwordx8 per qual");
  cq8 *prog = (cq8 *)g.prog;
  const uint32_t n = g.nprog;
  uint32_t qi = 0;
  u32x8 w = prog[0];                            // n >= 1 (program mode)
  while (qi < n) {
    const uint32_t cl = w[1];
    int cv = 0;                                 // the clause: 0 false, 1 true, 2 unknown
    do {
      strom_heap_qual2 q;
      q.attno = (int16_t)(w[0] & 0xffff);
      q.kind = (uint8_t)(w[0] >> 16);
      q.flags = (uint8_t)(w[0] >> 24);
      q.clause = cl;
      q.nconst = w[2];
      q.coff = w[3];
      q.lo = (int64_t)((uint64_t)w[4] | ((uint64_t)w[5] << 32));
      q.hi = (int64_t)((uint64_t)w[6] | ((uint64_t)w[7] << 32));
      if (++qi < n) w = prog[qi];
      if (!live || cv == 1) continue;           // decided: skip the clause's rest
      if (q.attno != last) {
        if ((uint32_t)q.attno < s.next) s = deform_init(t, tlen);   // walk again from the start
        a = deform_to(g.desc, s, (uint32_t)q.attno);
        last = q.attno;
      }
      if (s.bad) {
        live = false;
        verdict = 0;
        continue;
      }
      const int r = eval_qual2(q, (cu8 *)g.cpool, t, a);
      if (r == 1) cv = 1;
      else if (r == 2) cv = 2;
    } while (qi < n && w[1] == cl);
    if (live) {
      if (cv == 0) {
        live = false;
        verdict = 0;
      } else if (cv == 2) {
        verdict = 2;
      }
    }
    if (!__ballot(live)) break;                 // every lane decided
  }
  return verdict;
}

// ---- snapshot visibility: HeapTupleSatisfiesMVCC on the device.
// The reference hands every tuple of a block that is not all-visible to
// HeapTupleSatisfiesVisibility on the CPU (pgsql/nvme_strom.c:907-936);
// here each lane decides its own tuple from the header in the LDS page
// image, with the snapshot in the kernel arguments (scalar loads) and the
// SLRU windows — pg_xact, pg_subtrans, pg_multixact — in HBM, shared by
// every wave (L2-resident: a scan's tuples name few distinct xids).  The
// rules and their order are those of the host check (codecs.cc
// tuple_visible); the xid lists are sorted on upload and binary-searched.
// Three-valued like the qualifier programs: 1 visible, 0 not, -1 the inputs
// cannot decide (combo command id, an xid outside a window).
constexpr uint32_t kXmaxKeyshrLock = 0x0010, kComboCid = 0x0020, kXmaxExclLock = 0x0040,
                   kXminInvalid = 0x0200, kXmaxCommitted = 0x0400, kXmaxIsMulti = 0x1000;

struct MvccCtx {
  const strom_pg_mvcc &m;
  const uint32_t *run;        // running-xid bitmap from m.xmin (or null)
  uint32_t run_bits;
  bool und;
};

__device__ __forceinline__ bool mv_normal(uint32_t x) { return x >= 3; }
__device__ __forceinline__ bool mv_precedes(uint32_t a, uint32_t b) {   // TransactionIdPrecedes
  if (!mv_normal(a) || !mv_normal(b)) return a < b;
  return (int32_t)(a - b) < 0;
}

// membership in an ascending uint32 list (n may be 0)
__device__ __forceinline__ bool mv_has(const uint32_t *s, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint32_t v = s[mid];
    if (v == x) return true;
    if (v < x) lo = mid + 1;
    else hi = mid;
  }
  return false;
}

__device__ __forceinline__ int mv_clog(MvccCtx &c, uint32_t xid) {   // -1: outside the window
  const uint64_t k = (uint32_t)(xid - c.m.clog_base);
  if (!c.m.clog || k >= c.m.clog_n) return -1;
  return (c.m.clog[k >> 2] >> ((k & 3) * 2)) & 3;
}

__device__ __forceinline__ bool mv_parent(MvccCtx &c, uint32_t xid, uint32_t &p) {
  const uint32_t k = xid - c.m.subtrans_base;
  if (!c.m.subtrans || k >= c.m.subtrans_n) return false;
  p = c.m.subtrans[k];
  return true;
}

__device__ bool mv_did_commit(MvccCtx &c, uint32_t xid) {        // TransactionIdDidCommit
  for (int depth = 0; depth < 1024; ++depth) {
    if (!mv_normal(xid)) return xid == 1 || xid == 2;
    const int st = mv_clog(c, xid);
    if (st < 0) {
      c.und = true;
      return false;
    }
    if (st != 3) return st == 1;
    if (mv_precedes(xid, c.m.xmin)) return false;   // sub-committed, parent crashed
    uint32_t p;
    if (!mv_parent(c, xid, p)) {
      c.und = true;
      return false;
    }
    if (p == 0) return false;
    xid = p;
  }
  c.und = true;
  return false;
}

__device__ __forceinline__ bool mv_current(MvccCtx &c, uint32_t xid) {
  return mv_normal(xid) && mv_has(c.m.curxids, c.m.ncurxids, xid);
}

__device__ __forceinline__ bool mv_running_bit(const MvccCtx &c, uint32_t xid) {
  const uint32_t k = xid - c.m.xmin;                // xmin <= xid < xmax here
  return (c.run[k >> 5] >> (k & 31)) & 1;
}

__device__ bool mv_in_snapshot(MvccCtx &c, uint32_t xid) {       // XidInMVCCSnapshot
  if (mv_precedes(xid, c.m.xmin)) return false;
  if (!mv_precedes(xid, c.m.xmax)) return true;
  // the bitmap holds xip (+ subxip when not overflowed) over [xmin, xmax)
  if (c.run && !c.m.suboverflowed && xid - c.m.xmin < c.run_bits) return mv_running_bit(c, xid);
  if (!c.m.suboverflowed) {
    if (mv_has(c.m.subxip, c.m.nsubxip, xid)) return true;
  } else {
    uint32_t top = xid, p = xid;                    // SubTransGetTopmostTransaction
    for (int depth = 0; depth < 1024 && p; ++depth) {
      top = p;
      if (mv_precedes(p, c.m.xmin)) break;
      uint32_t q;
      if (!mv_parent(c, p, q) || (q && !mv_precedes(q, p))) {
        c.und = true;
        return true;
      }
      p = q;
    }
    xid = top;
    if (mv_precedes(xid, c.m.xmin)) return false;
    if (c.run && xid - c.m.xmin < c.run_bits) return mv_running_bit(c, xid);
  }
  return mv_has(c.m.xip, c.m.nxip, xid);
}

__device__ __forceinline__ bool mv_locked_only(uint32_t mask) {   // HEAP_XMAX_IS_LOCKED_ONLY
  return (mask & kXmaxLockOnly) ||
         (mask & (kXmaxIsMulti | kXmaxKeyshrLock | kXmaxExclLock)) == kXmaxExclLock;
}

// MultiXactIdGetUpdateXid over PostgreSQL's member page layout (409 groups
// of 4 status bytes + 4 xids per 8 KiB page); 0 when every member locks
__device__ uint32_t mv_update_xid(MvccCtx &c, uint32_t multi) {
  const uint32_t k = multi - c.m.mx_base;
  if (!c.m.mx_offsets || k >= c.m.mx_n || !c.m.mx_members) {
    c.und = true;
    return 0;
  }
  const uint32_t off = c.m.mx_offsets[k], n = c.m.mx_offsets[k + 1] - off;
  if (n > 65536) {
    c.und = true;
    return 0;
  }
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t mem = (uint32_t)(off + i - c.m.mxm_base);
    if (mem >= c.m.mxm_n) {
      c.und = true;
      return 0;
    }
    const uint64_t group = mem / 4, page = group / 409, within = mem % 4;
    const uint8_t *grp = c.m.mx_members + page * 8192 + (group % 409) * 20;
    if (grp[within] > 3) {                          // NoKeyUpdate / Update
      const uint8_t *x = grp + 4 + 4 * within;
      return (uint32_t)x[0] | ((uint32_t)x[1] << 8) | ((uint32_t)x[2] << 16) |
             ((uint32_t)x[3] << 24);
    }
  }
  return 0;
}

// the tuple at t (LDS page image), infomask already read
__device__ int mvcc_visible(const strom_heap_scan2_args &g, const uint8_t *t, uint32_t mask) {
  const strom_pg_mvcc &m = g.mvcc;
  MvccCtx c{m, g.mvcc_running, g.mvcc_running_bits, false};
  const uint32_t xmin = lds_u32(t, 0), xmax = lds_u32(t, 4);
  // the scanning transaction's own command id; a combo cid is backend-local
  auto own_cid = [&](uint32_t &cid) {
    if (mask & kComboCid) return false;
    cid = lds_u32(t, 8);
    return true;
  };
#define MV_UND(r) (c.und ? -1 : (r))
  if (!(mask & kXminCommitted)) {
    if (mask & kXminInvalid) return 0;
    if (mv_current(c, xmin)) {
      uint32_t cid;
      if (!own_cid(cid)) return -1;
      if (cid >= m.curcid) return 0;              // inserted after the scan started
      if ((mask & kXmaxInvalid) || mv_locked_only(mask)) return 1;
      if (mask & kXmaxIsMulti) {
        const uint32_t up = mv_update_xid(c, xmax);
        if (c.und) return -1;
        if (!mv_current(c, up)) return 1;          // the updating subxact aborted
        return cid >= m.curcid ? 1 : 0;
      }
      if (!mv_current(c, xmax)) return 1;          // the deleting subxact aborted
      return cid >= m.curcid ? 1 : 0;
    }
    if (mv_in_snapshot(c, xmin)) return MV_UND(0);
    if (!mv_did_commit(c, xmin)) return MV_UND(0);
  } else if ((mask & (kXminCommitted | kXminInvalid)) != (kXminCommitted | kXminInvalid) &&
             mv_in_snapshot(c, xmin)) {
    return MV_UND(0);                              // committed, not for this snapshot
  }
  if (c.und) return -1;
  if ((mask & kXmaxInvalid) || mv_locked_only(mask)) return 1;
  if (mask & kXmaxIsMulti) {
    const uint32_t up = mv_update_xid(c, xmax);
    if (c.und) return -1;
    if (!up) return 1;
    if (mv_current(c, up)) {
      uint32_t cid;
      if (!own_cid(cid)) return -1;
      return cid >= m.curcid ? 1 : 0;
    }
    if (mv_in_snapshot(c, up)) return MV_UND(1);
    return MV_UND(mv_did_commit(c, up) ? 0 : 1);
  }
  if (!(mask & kXmaxCommitted)) {
    if (mv_current(c, xmax)) {
      uint32_t cid;
      if (!own_cid(cid)) return -1;
      return cid >= m.curcid ? 1 : 0;
    }
    if (mv_in_snapshot(c, xmax)) return MV_UND(1);
    return MV_UND(mv_did_commit(c, xmax) ? 0 : 1);
  }
  return MV_UND(mv_in_snapshot(c, xmax) ? 1 : 0);
#undef MV_UND
}

// Bits: 1 keep, 2 undecidable here (a text qual met a compressed value, or
// the snapshot check could not decide: the page is flagged for a host
// recheck), 4 removed by the snapshot check.  3 = kept AND flagged: an
// undecided visibility keeps the tuple, as the host check does.
// GEN 0: the fixed int attribute of strom_heap_scan; 1: the fixed-size AND
// list (quals in the kernel arguments: scalar loads, early exit); 2: a
// program in device memory.  MV: the snapshot check on pages `check` marks.
// Separate instances: the program evaluator's and the snapshot check's
// registers and code stay out of the others.
template <int GEN, bool MV>
__device__ __forceinline__ int tuple_keep(const strom_heap_scan2_args &g, const uint8_t *pg,
                                          uint32_t lp, bool all_visible, bool check) {
  const strom_heap_scan_args &a = g.base;
  const uint32_t off = lp & 0x7fff, flags = (lp >> 15) & 3, len = lp >> 17;
  if (flags != kLpNormal || len < 23 || off < kSizeOfPageHeader || off + len > a.page_sz ||
      (off & 1))
    return 0;
  const uint32_t w20 = lds_u32(pg, off + 20);  // t_infomask (16) | t_hoff (8) | bits
  const uint32_t infomask = w20 & 0xffff, hoff = (w20 >> 16) & 0xff;
  if ((a.flags & STROM_HEAP_SKIP_INVISIBLE) && !all_visible) {
    // no clog here: only hint bits that prove visibility count
    if (!(infomask & kXminCommitted)) return 0;
    if (!(infomask & (kXmaxInvalid | kXmaxLockOnly))) return 0;
  }
  int und = 0;
  if (MV && check) {
    const int v = mvcc_visible(g, pg + off, infomask);
    if (v == 0) return 4;
    if (v < 0) und = 2;
  }
  if (GEN == 2) return eval_prog(g, pg + off, len) | und;
  if (GEN == 1) return (g.nquals ? eval_quals(g, pg + off, len) : 1) | und;
  if (a.attr_off < 0) return 1 | und;
  const uint32_t at = hoff + (uint32_t)a.attr_off;
  if ((infomask & kHeapHasNull) || at + (uint32_t)a.attr_width > len) return und;
  int64_t v;
  if (a.attr_width == 8) {
    const uint64_t lo = lds_u32(pg, off + at), hi = lds_u32(pg, off + at + 4);
    v = (int64_t)(lo | (hi << 32));
  } else {
    v = (int32_t)lds_u32(pg, off + at);
  }
  return (v >= a.lo && v <= a.hi ? 1 : 0) | und;
}

// PAGE = page size known at compile time (0: a.page_sz at run time).  Each
// lane moves NV 16-byte pieces of its wave's page per page.  A workgroup
// handles kWaves x kPerWave pages per output reservation: one same-address
// atomicAdd per 32 pages (round 1: per 4 pages, which capped scans where
// every page has qualifying rows at ~88 atomics/us, MI355X_MICROARCH.md
// row "dequeue" — 2.1 TB/s).
constexpr int kPerWave = 8;

template <int PAGE, int GEN, bool MV>
__global__ __launch_bounds__(256) void heap_scan_kernel(strom_heap_scan2_args g, uint32_t maxchunks,
                                                        uint32_t ppw) {
  const strom_heap_scan_args &a = g.base;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t page_sz = PAGE ? (uint32_t)PAGE : a.page_sz;
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint8_t *mypage = smem + (size_t)wid * page_sz;
  // masks[wid][j][chunk] for the wave's kPerWave pages
  uint64_t *masks =
      (uint64_t *)(smem + (size_t)kWaves * page_sz) + (size_t)wid * ppw * maxchunks;
  uint32_t *wcount =
      (uint32_t *)((uint64_t *)(smem + (size_t)kWaves * page_sz) + kWaves * ppw * maxchunks);
  uint32_t *wbase = wcount + kWaves;
  uint32_t *nch = wbase + kWaves + wid * ppw;        // chunks per page of this wave

  constexpr int NV = PAGE ? PAGE / (64 * 16) : 32;   // 32 = up to 32 KiB pages
  const uint32_t nv = page_sz / (64 * 16);
  v4u buf[NV];

#define STROM_HS_ISSUE(page_no)                                                           \
  do {                                                                                    \
    const v4u *src_ = (const v4u *)((const uint8_t *)a.pages + (uint64_t)(page_no) * page_sz); \
    _Pragma("unroll") for (int k = 0; k < NV; ++k)                                        \
      if (PAGE || (uint32_t)k < nv) buf[k] = __builtin_nontemporal_load(src_ + k * 64 + lane); \
  } while (0)

  const uint32_t kPerWg = kWaves * ppw;
  const uint32_t stride = gridDim.x * kPerWg;
  // wave wid owns pages [base + wid*ppw, +ppw) of each group
  uint32_t first = blockIdx.x * kPerWg + wid * ppw;
  if (first < a.npages) STROM_HS_ISSUE(first);
  // every wave of a workgroup runs the same trip counts (the output
  // reservation below has workgroup barriers)
  for (uint32_t base = blockIdx.x * kPerWg; base < a.npages; base += stride, first += stride) {
    uint32_t count = 0;
    for (uint32_t j = 0; j < ppw; ++j) {
      const uint32_t pg = first + j;
      const bool have = pg < a.npages;
      if (have) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
          if (PAGE || (uint32_t)k < nv) ((v4u *)mypage)[k * 64 + lane] = buf[k];
      }
      // the page image is this wave's alone: a wavefront-scope fence orders
      // its LDS stores before the reads below (a workgroup barrier here
      // held all four waves to the slowest page, twice per page)
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // the next page's loads are in flight while this one is parsed
      const uint32_t nxt = j + 1 < ppw ? pg + 1 : first + stride;
      if (nxt < a.npages && (j + 1 < ppw ? have : true)) STROM_HS_ISSUE(nxt);
      uint32_t nchunks = 0;
      if (have) {
        const PageHdr h = read_hdr(mypage);
        uint32_t status = page_status(a, mypage, h, pg, lane);
        if (status == 0) {
          const bool all_visible = (h.flags & kPdAllVisible) != 0;
          // the snapshot check: pages that are not PD_ALL_VISIBLE and that
          // the visibility map (mvcc_pages) did not route around it
          const bool check = MV && !all_visible && (!g.mvcc_pages || g.mvcc_pages[pg]);
          const uint32_t nitems = (h.lower - kSizeOfPageHeader) / 4;
          nchunks = (nitems + 63) / 64;
          uint32_t recheck = 0, removed = 0;
          for (uint32_t c = 0; c < nchunks; ++c) {
            const uint32_t i = c * 64 + lane;
            const int keep =
                i < nitems
                    ? tuple_keep<GEN, MV>(g, mypage, lds_u32a(mypage, kSizeOfPageHeader + 4 * i),
                                          all_visible, check)
                    : 0;
            const uint64_t m = __ballot(keep & 1);
            if (lane == 0) masks[j * maxchunks + c] = m;
            count += __popcll(m);
            if (GEN || MV) recheck += __popcll(__ballot(keep & 2));
            if (MV) removed += __popcll(__ballot(keep & 4));
          }
          if ((GEN || MV) && recheck) {
            status |= STROM_PAGE_RECHECK;
            if (lane == 0 && g.recheck_count) atomicAdd(g.recheck_count, recheck);
          }
          if (MV && removed && lane == 0 && g.mvcc_removed) atomicAdd(g.mvcc_removed, removed);
        }
        if (lane == 0 && a.page_status) a.page_status[pg] = status;
      }
      if (lane == 0) nch[j] = nchunks;
      // the wave's own page image is overwritten next
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) wcount[wid] = count;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t total = 0;
      for (int k = 0; k < kWaves; ++k) total += wcount[k];
      uint32_t start = total ? atomicAdd(a.out_count, total) : 0u;
      for (int k = 0; k < kWaves; ++k) {
        wbase[k] = start;
        start += wcount[k];
      }
    }
    __syncthreads();
    if (count && a.out_items) {
      uint32_t run = wbase[wid];
      const uint64_t below = (1ull << lane) - 1;
      for (uint32_t j = 0; j < ppw; ++j) {
        const uint32_t pg = first + j;
        for (uint32_t c = 0; c < nch[j]; ++c) {
          const uint64_t m = masks[j * maxchunks + c];
          if ((m >> lane) & 1) {
            const uint32_t slot = run + __popcll(m & below);
            if (slot < a.out_cap) a.out_items[slot] = (pg << 16) | (c * 64 + lane + 1);  // 1-based
          }
          run += __popcll(m);
        }
      }
    }
    __syncthreads();  // masks, counts and wcount are reused next iteration
  }
#undef STROM_HS_ISSUE
}

int heap_scan_launch(const strom_heap_scan2_args &g, int gen, void *stream) {
  const strom_heap_scan_args *a = &g.base;
  if (!a->pages || !a->out_count) return -22;
  if (a->page_sz < 1024 || (a->page_sz & 1023) || a->page_sz > 32768) return -22;
  if (a->attr_off >= 0 && a->attr_width != 4 && a->attr_width != 8) return -22;
  // (page << 16 | lineno) item ids address at most 65535 pages per call
  if (a->out_items && a->npages > 0xffffu) return -34;
  if (a->npages == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(a->out_count, 0, sizeof(uint32_t), st);
  const uint32_t maxchunks = ((a->page_sz - 24) / 4 + 63) / 64;
  // pages per wave per output reservation: kPerWave, fewer when the page
  // images leave too little LDS for the masks (32 KiB pages)
  const size_t budget = 160u * 1024u - (size_t)kWaves * a->page_sz - (3 * kWaves + kWaves * kPerWave) * 4;
  uint32_t ppw = (uint32_t)std::min<size_t>(kPerWave, budget / ((size_t)kWaves * maxchunks * 8));
  if (ppw < 1) return -22;
  const size_t lds = (size_t)kWaves * a->page_sz + (size_t)kWaves * ppw * maxchunks * 8 +
                     (2 * kWaves + kWaves * ppw) * 4;
  // enough workgroups to fill 256 CUs at the occupancy LDS allows, then stride
  const uint32_t per_cu = (uint32_t)(160u * 1024u / ((lds + 1023) & ~(size_t)1023));
  uint32_t grid = (a->npages + kWaves * ppw - 1) / (kWaves * ppw);
  const uint32_t cap = 256u * (per_cu ? per_cu : 1u) * 2u;
  if (grid > cap) grid = cap;
  auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, g, maxchunks, ppw); };
  const bool mv = g.mvcc_on != 0;
  if (a->page_sz == 8192) {
    if (mv) {
      if (gen == 2) launch(heap_scan_kernel<8192, 2, true>);
      else if (gen == 1) launch(heap_scan_kernel<8192, 1, true>);
      else launch(heap_scan_kernel<8192, 0, true>);
    } else {
      if (gen == 2) launch(heap_scan_kernel<8192, 2, false>);
      else if (gen == 1) launch(heap_scan_kernel<8192, 1, false>);
      else launch(heap_scan_kernel<8192, 0, false>);
    }
  } else {
    if (mv) {
      if (gen == 2) launch(heap_scan_kernel<0, 2, true>);
      else if (gen == 1) launch(heap_scan_kernel<0, 1, true>);
      else launch(heap_scan_kernel<0, 0, true>);
    } else {
      if (gen == 2) launch(heap_scan_kernel<0, 2, false>);
      else if (gen == 1) launch(heap_scan_kernel<0, 1, false>);
      else launch(heap_scan_kernel<0, 0, false>);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// the projected columns: ascending attribute numbers, each with its output
// column (values / valid are [ncol][cap]) and float flag
struct ProjSpec {
  uint32_t n;
  uint64_t fmask;                               // bit j: column j as float64
  uint8_t att[STROM_HEAP_MAX_ATTS], slot[STROM_HEAP_MAX_ATTS];
};

// one thread per selected item: deform its tuple once from the page in HBM,
// every projected attribute on the way
__global__ __launch_bounds__(256) void heap_project_kernel(const uint8_t *pages, uint32_t page_sz,
                                                           const uint32_t *items, const uint32_t *d_count,
                                                           uint32_t cap, strom_heap_tupdesc desc,
                                                           ProjSpec ps, uint64_t *values, uint8_t *valid) {
  const uint32_t n = min(*d_count, cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t it = items[i], pg = it >> 16, lineno = it & 0xffff;
    const uint8_t *page = pages + (uint64_t)pg * page_sz;
    const uint32_t lower = lds_u32a(page, 12) & 0xffff;
    bool tup = false;
    uint32_t off = 0, len = 0;
    if (lineno >= 1 && kSizeOfPageHeader + 4 * lineno <= lower) {
      const uint32_t lp = lds_u32a(page, kSizeOfPageHeader + 4 * (lineno - 1));
      off = lp & 0x7fff;
      len = lp >> 17;
      tup = len >= 23 && off >= kSizeOfPageHeader && off + len <= page_sz && !(off & 1);
    }
    Deform s = deform_init(page + off, tup ? len : 0);
    for (uint32_t j = 0; j < ps.n; ++j) {
      const uint32_t attno = ps.att[j], slot = ps.slot[j];
      uint64_t v = 0;
      uint8_t ok = 0;
      if (tup) {
        const Att a = deform_to(desc, s, attno);
        if (!s.bad && !a.null) {
          if (desc.attlen[attno] < 0) {   // varlena / cstring: where its bytes are
            v = ((uint64_t)((uint64_t)pg * page_sz + off + a.off + a.hdr) << 32) | (a.len - a.hdr);
            ok = a.ext ? 2 : 1;
          } else if ((ps.fmask >> slot) & 1) {
            v = (uint64_t)__double_as_longlong(att_float(page + off, a));
            ok = 1;
          } else {
            v = (uint64_t)att_int(page + off, a);
            ok = 1;
          }
        }
      }
      values[(size_t)slot * cap + i] = v;
      if (valid) valid[(size_t)slot * cap + i] = ok;
    }
  }
}

}  // namespace

extern "C" int strom_heap_scan(const strom_heap_scan_args *a, void *stream) {
  if (!a) return -22;
  strom_heap_scan2_args g;
  __builtin_memset(&g, 0, sizeof g);
  g.base = *a;
  return heap_scan_launch(g, 0, stream);
}

// the snapshot inputs' shape (their contents are device memory): windows
// within what the index arithmetic covers, lists present when counted
static int mvcc_check(const strom_pg_mvcc &m, uint32_t running_bits = 0) {
  if ((m.nxip && !m.xip) || (m.nsubxip && !m.subxip) || (m.ncurxids && !m.curxids)) return -22;
  if (running_bits > m.xmax - m.xmin) return -22;   // the bitmap covers [xmin, xmax) at most
  if (m.clog_n > (1ull << 32)) return -22;
  if (m.mx_n && (!m.mx_offsets || !m.mx_members)) return -22;
  return 0;
}

extern "C" int strom_heap_scan_mvcc(const strom_heap_scan_args *a, const strom_pg_mvcc *m,
                                    const uint8_t *mvcc_pages, uint32_t *mvcc_removed,
                                    uint32_t *recheck_count, const uint32_t *running,
                                    uint32_t running_bits, void *stream) {
  if (!a) return -22;
  strom_heap_scan2_args g;
  __builtin_memset(&g, 0, sizeof g);
  g.base = *a;
  g.recheck_count = recheck_count;
  if (m) {
    if (mvcc_check(*m, running ? running_bits : 0)) return -22;
    g.mvcc = *m;
    g.mvcc_on = 1;
    g.mvcc_pages = mvcc_pages;
    g.mvcc_removed = mvcc_removed;
    g.mvcc_running = running;
    g.mvcc_running_bits = running ? running_bits : 0;
  }
  return heap_scan_launch(g, 0, stream);
}

// host-side check of a program and its pool (copies in host memory, as
// uploaded): every qual's kind fits its attribute, clauses contiguous, every
// constant the device reads inside the pool — IN tables, text, numeric
// headers and their digits, the text entries an IN table names — and
// 8-aligned (the device reads the pool a dword at a time)
extern "C" int strom_heap_prog_check(const strom_heap_tupdesc *d, const strom_heap_qual2 *prog,
                                     uint32_t n, const uint8_t *pool, uint32_t pool_len) {
  if (!d || (n && !prog) || !pool || (pool_len & 7)) return -22;
  auto u32 = [&](uint64_t o) {
    return (uint32_t)pool[o] | ((uint32_t)pool[o + 1] << 8) | ((uint32_t)pool[o + 2] << 16) |
           ((uint32_t)pool[o + 3] << 24);
  };
  auto num_ok = [&](int64_t o) {              // header (kind, neg, weight, ndigits) + digits
    if (o < 0 || (o & 7) || (uint64_t)o + 8 > pool_len) return false;
    const uint32_t nd = (uint32_t)pool[o + 6] | ((uint32_t)pool[o + 7] << 8);
    return (uint64_t)o + 8 + 2ull * nd <= pool_len;
  };
  for (uint32_t i = 0; i < n; ++i) {
    const strom_heap_qual2 &x = prog[i];
    if (x.attno < 0 || x.attno >= d->natts) return -22;
    if (x.coff & 7) return -22;
    if (i && x.clause != prog[i - 1].clause) {
      for (uint32_t j = 0; j < i; ++j)       // a clause id may not come back
        if (prog[j].clause == x.clause) return -22;
    }
    const int len = d->attlen[x.attno];
    const uint64_t at = (uint64_t)x.coff;
    switch (x.kind) {
      case STROM_QUAL_INT_RANGE:
        if (len != 1 && len != 2 && len != 4 && len != 8) return -22;
        break;
      case STROM_QUAL_INT_IN:
        if (len != 1 && len != 2 && len != 4 && len != 8) return -22;
        if (at + 8ull * x.nconst > pool_len) return -22;
        break;
      case STROM_QUAL_FLOAT_RANGE:
        if (len != 4 && len != 8) return -22;
        break;
      case STROM_QUAL_TEXT_EQ:
      case STROM_QUAL_TEXT_PREFIX:
        if (len != -1 || at + x.nconst > pool_len) return -22;
        break;
      case STROM_QUAL_TEXT_IN:
        if (len != -1 || at + 8ull * x.nconst > pool_len) return -22;
        for (uint32_t k = 0; k < x.nconst; ++k) {
          const uint64_t co = u32(at + 8 * k), cl = u32(at + 8 * k + 4);
          if ((co & 7) || co + cl > pool_len) return -22;
        }
        break;
      case STROM_QUAL_NUMERIC_RANGE:
        if (len != -1) return -22;
        if (!(x.flags & 1) && !num_ok(x.lo)) return -22;
        if (!(x.flags & 2) && !num_ok(x.hi)) return -22;
        break;
      case STROM_QUAL_IS_NULL:
      case STROM_QUAL_NOT_NULL:
        break;
      default:
        return -22;
    }
  }
  return 0;
}

extern "C" int strom_heap_scan2(const strom_heap_scan2_args *g, void *stream) {
  if (!g || g->base.attr_off >= 0) return -22;
  if (g->mvcc_on && mvcc_check(g->mvcc, g->mvcc_running ? g->mvcc_running_bits : 0)) return -22;
  if (g->desc.natts < 1 || g->desc.natts > STROM_HEAP_MAX_ATTS) return -22;
  for (int i = 0; i < g->desc.natts; ++i) {
    const int al = g->desc.attalign[i], len = g->desc.attlen[i];
    if ((al != 1 && al != 2 && al != 4 && al != 8) || len == 0 || len < -2) return -22;
  }
  // a program was checked by the caller against its host copy
  // (strom_heap_prog_check); it lives in device memory here
  if (g->prog) {
    if (!g->nprog || !g->cpool || (g->cpool_len & 7)) return -22;   // the kernel reads prog[0]
    return heap_scan_launch(*g, 2, stream);
  }
  if (g->nquals < 0 || g->nquals > STROM_HEAP_MAX_QUALS) return -22;
  int last = -1;
  for (int q = 0; q < g->nquals; ++q) {
    const strom_heap_qual &x = g->quals[q];
    if (x.attno < last || x.attno >= g->desc.natts) return -22;  // sorted by attno
    last = x.attno;
    const int len = g->desc.attlen[x.attno];
    switch (x.kind) {
      case STROM_QUAL_INT_RANGE:
      case STROM_QUAL_INT_IN:
        if (len != 1 && len != 2 && len != 4 && len != 8) return -22;
        if (x.kind == STROM_QUAL_INT_IN && x.nconst > 4) return -22;
        break;
      case STROM_QUAL_FLOAT_RANGE:
        if (len != 4 && len != 8) return -22;
        break;
      case STROM_QUAL_TEXT_EQ:
      case STROM_QUAL_TEXT_PREFIX:
        if (len != -1 || x.nconst > 32) return -22;
        break;
      case STROM_QUAL_IS_NULL:
      case STROM_QUAL_NOT_NULL:
        break;
      default:
        return -22;
    }
  }
  return heap_scan_launch(*g, 1, stream);
}

extern "C" int strom_heap_project_n(const void *pages, uint32_t page_sz, const uint32_t *items,
                                    const uint32_t *d_count, uint32_t cap,
                                    const strom_heap_tupdesc *desc, const int32_t *attnos,
                                    uint32_t ncol, uint64_t float_mask, uint64_t *values,
                                    uint8_t *valid, void *stream) {
  if (!pages || !items || !d_count || !desc || !values || !attnos) return -22;
  if (desc->natts < 1 || desc->natts > STROM_HEAP_MAX_ATTS) return -22;
  if (ncol < 1 || ncol > STROM_HEAP_MAX_ATTS) return -22;
  if (page_sz < 1024 || (page_sz & 1023) || page_sz > 32768) return -22;
  ProjSpec ps;
  __builtin_memset(&ps, 0, sizeof ps);
  ps.n = ncol;
  ps.fmask = float_mask;
  for (uint32_t j = 0; j < ncol; ++j) {
    const int32_t k = attnos[j];
    if (k < 0 || k >= desc->natts) return -22;
    const int len = desc->attlen[k];
    if (((float_mask >> j) & 1) && len != 4 && len != 8) return -22;
    ps.att[j] = (uint8_t)k;
    ps.slot[j] = (uint8_t)j;
  }
  // ascending attributes: one forward deform walk per tuple
  for (uint32_t j = 1; j < ncol; ++j)
    for (uint32_t i = j; i > 0 && ps.att[i - 1] > ps.att[i]; --i) {
      std::swap(ps.att[i - 1], ps.att[i]);
      std::swap(ps.slot[i - 1], ps.slot[i]);
    }
  for (uint32_t j = 1; j < ncol; ++j)
    if (ps.att[j] == ps.att[j - 1]) return -22;
  if (cap == 0) return 0;
  const uint32_t grid = std::min<uint32_t>((cap + 255) / 256, 4096);
  hipLaunchKernelGGL(heap_project_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t *)pages, page_sz, items, d_count, cap, *desc, ps, values, valid);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int strom_heap_project(const void *pages, uint32_t page_sz, const uint32_t *items,
                                  const uint32_t *d_count, uint32_t cap,
                                  const strom_heap_tupdesc *desc, int attno, int as_float,
                                  uint64_t *values, uint8_t *valid, void *stream) {
  if (!desc) return -22;
  const int32_t k = attno;
  return strom_heap_project_n(pages, page_sz, items, d_count, cap, desc, &k, 1, as_float ? 1 : 0,
                              values, valid, stream);
}
