// codecs.cc — host-side reference codecs and checksums.
//
// These are the CPU references the GPU kernels are tested against, and the
// producers of compressed test data (no LZ4/snappy library is installed):
//   - CRC32C (Castagnoli, reflected 0x82F63B78), slicing-by-8;
//   - PostgreSQL's page checksum (FNV-1a variant over 32 interleaved sums,
//     pg_checksum_page semantics, BLCKSZ-generic);
//   - LZ4 raw block format: greedy single-probe compressor + safe decoder;
//   - snappy raw format: greedy compressor + safe decoder.
#include <errno.h>
#include <string.h>
#include <unistd.h>

#include <cstdint>
#include <vector>

#include "strom/strom.h"

namespace {

struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Crc32cTables &crc_tables() {
  static Crc32cTables t;
  return t;
}

const uint32_t kPgBase[32] = {
    0x5B1F36E9, 0xB8525960, 0x02AB50AA, 0x1DE66D2A, 0x79FF467A, 0x9BB9F8A3, 0x217E7CD2,
    0x83E13D2C, 0xF8D4474F, 0xE39EB970, 0x42C6AE16, 0x993216FA, 0x7B093B5D, 0x98DAFF3C,
    0xF718902A, 0x0B1C9CDB, 0xE58F764B, 0x187636BC, 0x5D7B3BB1, 0xE73DE7DE, 0x92BEC979,
    0xCCA6C0B2, 0x304A0979, 0x85AA43D4, 0x783125BB, 0x6CA8EAA2, 0xE407EAC6, 0x4B5CFC3E,
    0x9FBF8C76, 0x15CA20BE, 0xF2CA9FFF, 0x3ED50F2B};

inline uint32_t pg_mix(uint32_t sum, uint32_t v) {
  uint32_t t = sum ^ v;
  return t * 16777619u ^ (t >> 17);
}

inline uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

// ---------------------------------------------------------------- LZ4
constexpr int kMinMatch = 4;
constexpr int kLastLiterals = 5;
constexpr int kMfLimit = 12;

uint8_t *lz4_put_len(uint8_t *op, uint8_t *oend, size_t len) {
  while (len >= 255) {
    if (op >= oend) return nullptr;
    *op++ = 255;
    len -= 255;
  }
  if (op >= oend) return nullptr;
  *op++ = (uint8_t)len;
  return op;
}

}  // namespace

extern "C" {

uint32_t strom_crc32c_host(uint32_t crc, const void *buf, size_t len) {
  const Crc32cTables &T = crc_tables();
  const uint8_t *p = (const uint8_t *)buf;
  uint32_t c = ~crc;
  while (len >= 8) {
    uint32_t lo = rd32(p) ^ c, hi = rd32(p + 4);
    c = T.t[7][lo & 0xff] ^ T.t[6][(lo >> 8) & 0xff] ^ T.t[5][(lo >> 16) & 0xff] ^
        T.t[4][lo >> 24] ^ T.t[3][hi & 0xff] ^ T.t[2][(hi >> 8) & 0xff] ^
        T.t[1][(hi >> 16) & 0xff] ^ T.t[0][hi >> 24];
    p += 8;
    len -= 8;
  }
  while (len--) c = (c >> 8) ^ T.t[0][(c ^ *p++) & 0xff];
  return ~c;
}

uint16_t strom_pg_checksum_host(const void *page, uint32_t blkno, uint32_t page_sz) {
  const uint8_t *p = (const uint8_t *)page;
  uint32_t sums[32];
  memcpy(sums, kPgBase, sizeof sums);
  const uint32_t rows = page_sz / 4 / 32;
  for (uint32_t i = 0; i < rows; ++i)
    for (int j = 0; j < 32; ++j) {
      uint32_t off = (i * 32 + j) * 4;
      uint32_t v = rd32(p + off);
      if (off == 8) v &= 0xffff0000u;  // pd_checksum (bytes 8..9) reads as zero
      sums[j] = pg_mix(sums[j], v);
    }
  for (int r = 0; r < 2; ++r)
    for (int j = 0; j < 32; ++j) sums[j] = pg_mix(sums[j], 0);
  uint32_t x = 0;
  for (int j = 0; j < 32; ++j) x ^= sums[j];
  x ^= blkno;
  return (uint16_t)((x % 65535u) + 1);
}

// ---- MVCC visibility of heap tuples: HeapTupleSatisfiesMVCC
// (src/backend/access/heap/heapam_visibility.c), with the inputs it reads
// from shared memory and the SLRUs supplied by the caller (strom_pg_mvcc):
// hint bits, pg_xact, pg_subtrans (sub-committed xids follow their parent;
// XidInMVCCSnapshot maps to the topmost xid when the snapshot's subxip
// overflowed), pg_multixact (a locker-only xmax deletes nothing; otherwise
// the update member decides) and the scanning transaction's own xids with
// its command id.  Transaction ids compare modulo 2^32 (TransactionIdPrecedes).
// What it cannot decide — a combo command id (backend-local), a log window
// that does not cover an xid — is reported, never guessed.
namespace {
constexpr uint16_t kXmaxKeyshrLock = 0x0010, kComboCid = 0x0020, kXmaxExclLock = 0x0040,
                   kXmaxLockOnly = 0x0080, kXminCommitted = 0x0100, kXminInvalid = 0x0200,
                   kXmaxCommitted = 0x0400, kXmaxInvalid = 0x0800, kXmaxIsMulti = 0x1000;
constexpr uint16_t kLockMask = kXmaxKeyshrLock | kXmaxExclLock;

struct Vis {
  const strom_pg_mvcc &m;
  bool undecided = false;
};

bool xid_normal(uint32_t x) { return x >= 3; }
bool xid_precedes(uint32_t a, uint32_t b) {       // TransactionIdPrecedes
  if (!xid_normal(a) || !xid_normal(b)) return a < b;
  return (int32_t)(a - b) < 0;
}

int clog_status(Vis &v, uint32_t xid) {          // -1: outside the window
  const uint64_t k = (uint32_t)(xid - v.m.clog_base);
  if (!v.m.clog || k >= v.m.clog_n) return -1;
  return (v.m.clog[k >> 2] >> ((k & 3) * 2)) & 3;
}

bool subtrans_parent(Vis &v, uint32_t xid, uint32_t &parent) {
  const uint32_t k = xid - v.m.subtrans_base;
  if (!v.m.subtrans || k >= v.m.subtrans_n) return false;
  parent = v.m.subtrans[k];
  return true;
}

bool did_commit(Vis &v, uint32_t xid) {           // TransactionIdDidCommit
  for (int depth = 0; depth < 1024; ++depth) {
    if (!xid_normal(xid)) return xid == 1 || xid == 2;   // bootstrap / frozen; invalid never
    const int st = clog_status(v, xid);
    if (st < 0) {
      v.undecided = true;
      return false;
    }
    if (st != 3) return st == 1;
    // sub-committed: its parent decides; one older than every snapshot's
    // xmin whose parent never committed has crashed
    if (xid_precedes(xid, v.m.xmin)) return false;
    uint32_t p;
    if (!subtrans_parent(v, xid, p)) {
      v.undecided = true;
      return false;
    }
    if (p == 0) return false;
    xid = p;
  }
  v.undecided = true;
  return false;
}

bool in_list(const uint32_t *a, uint32_t n, uint32_t x) {
  for (uint32_t i = 0; i < n; ++i)
    if (a[i] == x) return true;
  return false;
}

bool is_current(Vis &v, uint32_t xid) {           // TransactionIdIsCurrentTransactionId
  return xid_normal(xid) && in_list(v.m.curxids, v.m.ncurxids, xid);
}

bool xid_in_snapshot(Vis &v, uint32_t xid) {     // XidInMVCCSnapshot: still running for us
  if (xid_precedes(xid, v.m.xmin)) return false;
  if (!xid_precedes(xid, v.m.xmax)) return true;
  if (!v.m.suboverflowed) {
    if (in_list(v.m.subxip, v.m.nsubxip, xid)) return true;
  } else {
    // SubTransGetTopmostTransaction
    uint32_t top = xid, p = xid;
    for (int depth = 0; depth < 1024 && p; ++depth) {
      top = p;
      if (xid_precedes(p, v.m.xmin)) break;
      uint32_t q;
      if (!subtrans_parent(v, p, q)) {
        v.undecided = true;
        return true;
      }
      if (q && !xid_precedes(q, p)) {                 // a corrupt entry
        v.undecided = true;
        return true;
      }
      p = q;
    }
    xid = top;
    if (xid_precedes(xid, v.m.xmin)) return false;
  }
  return in_list(v.m.xip, v.m.nxip, xid);
}

bool locked_only(uint16_t mask) {                 // HEAP_XMAX_IS_LOCKED_ONLY
  return (mask & kXmaxLockOnly) || (mask & (kXmaxIsMulti | kLockMask)) == kXmaxExclLock;
}

// MultiXactIdGetUpdateXid: the member whose status is an update (at most
// one); 0 when every member only locks
uint32_t multi_update_xid(Vis &v, uint32_t multi) {
  const uint32_t k = multi - v.m.mx_base;
  if (!v.m.mx_offsets || k >= v.m.mx_n || !v.m.mx_members) {
    v.undecided = true;
    return 0;
  }
  const uint32_t off = v.m.mx_offsets[k], n = v.m.mx_offsets[k + 1] - off;
  if (n > 65536) {
    v.undecided = true;
    return 0;
  }
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t mem = (uint32_t)(off + i - v.m.mxm_base);
    if (mem >= v.m.mxm_n) {
      v.undecided = true;
      return 0;
    }
    const uint64_t group = mem / 4, page = group / 409, within = mem % 4;
    const uint8_t *g = v.m.mx_members + page * 8192 + (group % 409) * 20;
    const uint32_t status = g[within];
    if (status > 3) return rd32(g + 4 + 4 * within);  // NoKeyUpdate / Update
  }
  return 0;
}

// a command id of the scanning transaction's own tuple; false: a combo
// command id (its mapping lives in that backend only)
bool own_cid(Vis &v, uint16_t mask, const uint8_t *tup, uint32_t &cid) {
  if (mask & kComboCid) {
    v.undecided = true;
    return false;
  }
  cid = rd32(tup + 8);
  return true;
}

int tuple_visible(Vis &v, const uint8_t *tup) {
  const uint32_t xmin = rd32(tup), xmax = rd32(tup + 4);
  const uint16_t mask = (uint16_t)(tup[20] | (tup[21] << 8));
#define UND(r) (v.undecided ? -1 : (r))
  if (!(mask & kXminCommitted)) {
    if (mask & kXminInvalid) return 0;
    if (is_current(v, xmin)) {
      uint32_t cid;
      if (!own_cid(v, mask, tup, cid)) return -1;
      if (cid >= v.m.curcid) return 0;             // inserted after the scan started
      if (mask & kXmaxInvalid) return 1;
      if (locked_only(mask)) return 1;
      if (mask & kXmaxIsMulti) {
        const uint32_t up = multi_update_xid(v, xmax);
        if (v.undecided) return -1;
        if (!is_current(v, up)) return 1;          // the updating subxact aborted
        return cid >= v.m.curcid ? 1 : 0;          // t_cid is the cmax here (no combo)
      }
      if (!is_current(v, xmax)) return 1;          // the deleting subxact aborted
      return cid >= v.m.curcid ? 1 : 0;
    }
    if (xid_in_snapshot(v, xmin)) return UND(0);
    if (!did_commit(v, xmin)) return UND(0);       // aborted or crashed
  } else if ((mask & (kXminCommitted | kXminInvalid)) != (kXminCommitted | kXminInvalid) &&
             xid_in_snapshot(v, xmin)) {
    return UND(0);                                 // committed, but not for this snapshot
  }
  if (v.undecided) return -1;
  // the inserting transaction is visible; now the deleter
  if (mask & kXmaxInvalid) return 1;
  if (locked_only(mask)) return 1;
  if (mask & kXmaxIsMulti) {
    const uint32_t up = multi_update_xid(v, xmax);
    if (v.undecided) return -1;
    if (!up) return 1;
    if (is_current(v, up)) {
      uint32_t cid;
      if (!own_cid(v, mask, tup, cid)) return -1;
      return cid >= v.m.curcid ? 1 : 0;
    }
    if (xid_in_snapshot(v, up)) return UND(1);
    return UND(did_commit(v, up) ? 0 : 1);
  }
  if (!(mask & kXmaxCommitted)) {
    if (is_current(v, xmax)) {
      uint32_t cid;
      if (!own_cid(v, mask, tup, cid)) return -1;
      return cid >= v.m.curcid ? 1 : 0;
    }
    if (xid_in_snapshot(v, xmax)) return UND(1);
    return UND(did_commit(v, xmax) ? 0 : 1);
  }
  return UND(xid_in_snapshot(v, xmax) ? 1 : 0);
#undef UND
}
}  // namespace

int strom_pg_tuple_visible(const void *tuple_header, const strom_pg_mvcc *m) {
  Vis v{*m};
  return tuple_visible(v, (const uint8_t *)tuple_header);
}

long strom_pg_apply_mvcc(void *page, uint32_t page_sz, const strom_pg_mvcc *m, uint16_t *recheck,
                         uint32_t cap, uint32_t *nrecheck) {
  uint8_t *p = (uint8_t *)page;
  if (nrecheck) *nrecheck = 0;
  const uint16_t lower = (uint16_t)(p[12] | (p[13] << 8)), flags = (uint16_t)(p[10] | (p[11] << 8));
  if (lower < 24 || lower > page_sz) return -22;
  if (flags & 0x0004) return 0;                      // PD_ALL_VISIBLE: nothing to check
  long removed = 0;
  uint32_t nr = 0;
  for (uint32_t i = 0; i < (uint32_t)(lower - 24) / 4; ++i) {
    uint8_t *lpp = p + 24 + 4 * i;
    uint32_t lp = rd32(lpp);
    const uint32_t off = lp & 0x7fff, fl = (lp >> 15) & 3, len = lp >> 17;
    if (fl != 1 || len < 23 || off < 24 || off + len > page_sz) continue;
    Vis v{*m};
    const int r = tuple_visible(v, p + off);
    if (r > 0) continue;
    if (r < 0) {                                     // kept for a recheck
      if (recheck && nr < cap) recheck[nr] = (uint16_t)(i + 1);
      ++nr;
      continue;
    }
    lp &= ~(3u << 15);                               // LP_UNUSED, as the reference marks them
    memcpy(lpp, &lp, 4);
    ++removed;
  }
  if (nrecheck) *nrecheck = nr;
  return removed;
}

// The buffer-manager leg of the reference's chunk loader
// (pgsql/nvme_strom.c:896-940: ReadBuffer, per-tuple visibility, copy into
// the chunk) for the blocks a scan checks on the host: one pread per run of
// consecutive blocks, the checksum ReadBuffer would verify, then the
// in-place LP_UNUSED marking.  A page that is not a heap page is left as
// read (the scan kernel reports its header).
long strom_pg_read_check_pages(int fd, const uint32_t *blocks, uint32_t n, uint32_t relseg_blocks,
                               uint32_t page_sz, void *stage, const strom_pg_mvcc *m,
                               int verify_checksum, uint8_t *recheck_flags) {
  if ((n && (!blocks || !stage)) || !m || page_sz < 1024 || (page_sz & 1023)) return -EINVAL;
  uint8_t *out = (uint8_t *)stage;
  long removed = 0;
  std::vector<uint16_t> rc(page_sz / 4);
  for (uint32_t i = 0; i < n;) {
    // a run of blocks consecutive in the file: one read
    uint32_t j = i + 1;
    const uint64_t b0 = relseg_blocks ? blocks[i] % relseg_blocks : blocks[i];
    while (j < n && blocks[j] == blocks[j - 1] + 1 &&
           (relseg_blocks ? blocks[j] % relseg_blocks : blocks[j]) == b0 + (j - i))
      ++j;
    const size_t want = (size_t)(j - i) * page_sz;
    size_t got = 0;
    while (got < want) {
      const ssize_t r = pread(fd, out + (size_t)i * page_sz + got, want - got,
                              (off_t)(b0 * page_sz + got));
      if (r < 0) {
        if (errno == EINTR) continue;
        return -errno;
      }
      if (r == 0) break;
      got += (size_t)r;
    }
    memset(out + (size_t)i * page_sz + got, 0, want - got);
    for (uint32_t k = i; k < j; ++k) {
      uint8_t *p = out + (size_t)k * page_sz;
      bool ck_ok = false;
      if (verify_checksum) {
        const uint16_t stored = (uint16_t)(p[8] | (p[9] << 8));
        ck_ok = strom_pg_checksum_host(p, blocks[k], page_sz) == stored;
      }
      uint32_t nr = 0;
      const long r = strom_pg_apply_mvcc(p, page_sz, m, rc.data(), (uint32_t)rc.size(), &nr);
      if (recheck_flags) recheck_flags[k] = r >= 0 && nr ? 1 : 0;
      if (r <= 0) continue;
      removed += r;
      if (ck_ok) {
        const uint16_t c = strom_pg_checksum_host(p, blocks[k], page_sz);
        p[8] = (uint8_t)c;
        p[9] = (uint8_t)(c >> 8);
      }
    }
    i = j;
  }
  return removed;
}

long strom_pg_apply_snapshot(void *page, uint32_t page_sz, uint32_t snap_xmin, uint32_t snap_xmax,
                             const uint32_t *xip, uint32_t nxip, const uint8_t *clog,
                             uint64_t clog_xids) {
  strom_pg_mvcc m{};
  m.xmin = snap_xmin;
  m.xmax = snap_xmax;
  m.xip = xip;
  m.nxip = nxip;
  m.clog = clog;
  m.clog_n = clog_xids;
  return strom_pg_apply_mvcc(page, page_sz, &m, nullptr, 0, nullptr);
}

uint64_t strom_atomic_fetch_add_u64(uint64_t *addr, uint64_t v) {
  return __atomic_fetch_add(addr, v, __ATOMIC_SEQ_CST);
}

int strom_atomic_cas_u64(uint64_t *addr, uint64_t expect, uint64_t desired) {
  return __atomic_compare_exchange_n(addr, &expect, desired, false, __ATOMIC_SEQ_CST,
                                     __ATOMIC_SEQ_CST) ? 1 : 0;
}

uint64_t strom_atomic_load_u64(const uint64_t *addr) {
  return __atomic_load_n(addr, __ATOMIC_SEQ_CST);
}

long strom_lz4_compress_host(const void *src, size_t n, void *dst, size_t cap) {
  const uint8_t *ip = (const uint8_t *)src, *base = ip, *iend = ip + n;
  const uint8_t *anchor = ip;
  uint8_t *op = (uint8_t *)dst, *oend = op + cap;
  std::vector<int32_t> table(1 << 16, -1);
  const uint8_t *mflimit = n > (size_t)kMfLimit ? iend - kMfLimit : base;
  const uint8_t *matchlimit = iend - kLastLiterals;
  if (n > (size_t)kMfLimit) {
    while (ip < mflimit) {
      uint32_t seq = rd32(ip);
      uint32_t h = (seq * 2654435761u) >> 16;
      int32_t cand = table[h];
      table[h] = (int32_t)(ip - base);
      if (cand < 0 || ip - (base + cand) > 65535 || rd32(base + cand) != seq) {
        ++ip;
        continue;
      }
      const uint8_t *match = base + cand;
      // extend backwards over pending literals
      while (ip > anchor && match > base && ip[-1] == match[-1]) {
        --ip;
        --match;
      }
      const uint8_t *mp = ip + kMinMatch, *mm = match + kMinMatch;
      while (mp < matchlimit && *mp == *mm) {
        ++mp;
        ++mm;
      }
      size_t lit = ip - anchor, mlen = mp - ip - kMinMatch;
      if (op + 1 + lit / 255 + lit + 2 + mlen / 255 + 2 > oend) return -ENOSPC;
      uint8_t *token = op++;
      *token = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
      if (lit >= 15) op = lz4_put_len(op, oend, lit - 15);
      memcpy(op, anchor, lit);
      op += lit;
      uint16_t off = (uint16_t)(ip - match);
      *op++ = (uint8_t)off;
      *op++ = (uint8_t)(off >> 8);
      *token |= (uint8_t)(mlen >= 15 ? 15 : mlen);
      if (mlen >= 15) op = lz4_put_len(op, oend, mlen - 15);
      if (!op) return -ENOSPC;
      ip = mp;
      anchor = ip;
      if (ip < mflimit) {
        // seed the table inside the match tail for better ratio
        table[(rd32(ip - 2) * 2654435761u) >> 16] = (int32_t)(ip - 2 - base);
      }
    }
  }
  size_t lit = iend - anchor;
  if (op + 1 + lit / 255 + 1 + lit > oend) return -ENOSPC;
  uint8_t *token = op++;
  *token = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
  if (lit >= 15) op = lz4_put_len(op, oend, lit - 15);
  memcpy(op, anchor, lit);
  op += lit;
  return op - (uint8_t *)dst;
}

long strom_lz4_decompress_host(const void *src, size_t n, void *dst, size_t cap) {
  const uint8_t *ip = (const uint8_t *)src, *iend = ip + n;
  uint8_t *op = (uint8_t *)dst, *ostart = op, *oend = op + cap;
  while (ip < iend) {
    uint8_t token = *ip++;
    size_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= iend) return -EINVAL;
        b = *ip++;
        lit += b;
      } while (b == 255);
    }
    if ((size_t)(iend - ip) < lit || (size_t)(oend - op) < lit) return -EINVAL;
    memcpy(op, ip, lit);
    op += lit;
    ip += lit;
    if (ip >= iend) break;  // last sequence: literals only
    if (iend - ip < 2) return -EINVAL;
    size_t off = ip[0] | (ip[1] << 8);
    ip += 2;
    if (off == 0 || off > (size_t)(op - ostart)) return -EINVAL;
    size_t mlen = token & 15;
    if (mlen == 15) {
      uint8_t b;
      do {
        if (ip >= iend) return -EINVAL;
        b = *ip++;
        mlen += b;
      } while (b == 255);
    }
    mlen += kMinMatch;
    if ((size_t)(oend - op) < mlen) return -EINVAL;
    const uint8_t *m = op - off;
    for (size_t i = 0; i < mlen; ++i) op[i] = m[i];  // overlap-safe forward copy
    op += mlen;
  }
  return op - ostart;
}

long strom_snappy_compress_host(const void *src, size_t n, void *dst, size_t cap) {
  const uint8_t *base = (const uint8_t *)src, *ip = base, *iend = base + n;
  uint8_t *op = (uint8_t *)dst, *oend = op + cap;
  // varint preamble
  size_t v = n;
  do {
    if (op >= oend) return -ENOSPC;
    uint8_t b = v & 0x7f;
    v >>= 7;
    *op++ = b | (v ? 0x80 : 0);
  } while (v);
  auto emit_literal = [&](const uint8_t *p, size_t len) -> bool {
    while (len) {
      size_t l = len;
      size_t m = l - 1;
      if (m < 60) {
        if (op + 1 + l > oend) return false;
        *op++ = (uint8_t)(m << 2);
      } else {
        int nb = m < 256 ? 1 : m < 65536 ? 2 : m < (1u << 24) ? 3 : 4;
        if (op + 1 + nb + l > oend) return false;
        *op++ = (uint8_t)((59 + nb) << 2);
        for (int i = 0; i < nb; ++i) *op++ = (uint8_t)(m >> (8 * i));
      }
      memcpy(op, p, l);
      op += l;
      p += l;
      len -= l;
    }
    return true;
  };
  auto emit_copy = [&](size_t off, size_t len) -> bool {
    while (len > 0) {
      size_t l = len > 64 ? 64 : len;
      if (len > 64 && len - 64 < 4) l = 60;  // keep the remainder >= 4
      if (l >= 4 && l <= 11 && off < 2048) {
        if (op + 2 > oend) return false;
        *op++ = (uint8_t)(1 | ((l - 4) << 2) | ((off >> 8) << 5));
        *op++ = (uint8_t)off;
      } else {
        if (op + 3 > oend) return false;
        *op++ = (uint8_t)(2 | ((l - 1) << 2));
        *op++ = (uint8_t)off;
        *op++ = (uint8_t)(off >> 8);
      }
      len -= l;
    }
    return true;
  };
  std::vector<int32_t> table(1 << 15, -1);
  const uint8_t *anchor = ip;
  if (n >= 8) {
    const uint8_t *limit = iend - 4;
    while (ip < limit) {
      uint32_t seq = rd32(ip);
      uint32_t h = (seq * 0x1e35a7bdu) >> 17;
      int32_t cand = table[h];
      table[h] = (int32_t)(ip - base);
      if (cand < 0 || ip - (base + cand) > 65535 || rd32(base + cand) != seq) {
        ++ip;
        continue;
      }
      const uint8_t *m = base + cand;
      size_t len = 4;
      while (ip + len < iend && ip[len] == m[len]) ++len;
      if (!emit_literal(anchor, ip - anchor)) return -ENOSPC;
      if (!emit_copy(ip - m, len)) return -ENOSPC;
      ip += len;
      anchor = ip;
    }
  }
  if (!emit_literal(anchor, iend - anchor)) return -ENOSPC;
  return op - (uint8_t *)dst;
}

long strom_snappy_decompress_host(const void *src, size_t n, void *dst, size_t cap) {
  const uint8_t *ip = (const uint8_t *)src, *iend = ip + n;
  uint64_t ulen = 0;
  int shift = 0;
  for (;;) {
    if (ip >= iend || shift > 35) return -EINVAL;
    uint8_t b = *ip++;
    ulen |= (uint64_t)(b & 0x7f) << shift;
    shift += 7;
    if (!(b & 0x80)) break;
  }
  if (ulen > cap) return -ENOSPC;
  uint8_t *op = (uint8_t *)dst, *ostart = op, *oend = op + ulen;
  while (ip < iend) {
    uint8_t tag = *ip++;
    size_t len, off;
    switch (tag & 3) {
      case 0: {
        len = (tag >> 2) + 1;
        if (len > 60) {
          int nb = (int)len - 60;
          if (iend - ip < nb) return -EINVAL;
          len = 0;
          for (int i = 0; i < nb; ++i) len |= (size_t)ip[i] << (8 * i);
          len += 1;
          ip += nb;
        }
        if ((size_t)(iend - ip) < len || (size_t)(oend - op) < len) return -EINVAL;
        memcpy(op, ip, len);
        op += len;
        ip += len;
        continue;
      }
      case 1:
        if (ip >= iend) return -EINVAL;
        len = 4 + ((tag >> 2) & 7);
        off = ((size_t)(tag >> 5) << 8) | *ip++;
        break;
      case 2:
        if (iend - ip < 2) return -EINVAL;
        len = (tag >> 2) + 1;
        off = ip[0] | (ip[1] << 8);
        ip += 2;
        break;
      default:
        if (iend - ip < 4) return -EINVAL;
        len = (tag >> 2) + 1;
        off = rd32(ip);
        ip += 4;
        break;
    }
    if (off == 0 || off > (size_t)(op - ostart) || (size_t)(oend - op) < len) return -EINVAL;
    const uint8_t *m = op - off;
    for (size_t i = 0; i < len; ++i) op[i] = m[i];
    op += len;
  }
  return op == oend ? (long)ulen : -EINVAL;
}

}  // extern "C"
