// heapscan.hip — PostgreSQL heap pages scanned on the GPU.
//
// The reference's PostgreSQL CustomScan loads heap blocks into a DMA buffer
// and then walks line pointers on the CPU (pgsql/nvme_strom.c:1054-1092:
// nvmestrom_next_tuple), with visibility handled per tuple for blocks that
// came through the buffer manager (:896-940).  On MI355X the loaded pages sit
// in HBM and one wavefront per page does all of it:
//   1. page header sanity (pd_lower/pd_upper/pd_special bounds, flag bits,
//      page size) — PageIsVerified-style;
//   2. optional data checksum (pg_checksum_page: 32 interleaved FNV-1a
//      sums = 32 lanes, one column of uint32 words each);
//   3. line pointers 64 at a time (one per lane): LP_NORMAL items, optional
//      hint-bit visibility (xmin committed, xmax invalid or lock-only), and
//      an optional range predicate on a fixed-offset int4/int8 column;
//   4. wave-level stream compaction (ballot + popcount + one atomicAdd per
//      64 items) into (page << 16 | lineno) item ids.
#include <hip/hip_runtime.h>

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
constexpr uint16_t kLpNormal = 1;
constexpr uint16_t kHeapHasNull = 0x0001;
constexpr uint16_t kXmaxLockOnly = 0x0080;
constexpr uint16_t kXminCommitted = 0x0100;
constexpr uint16_t kXminInvalid = 0x0200;
constexpr uint16_t kXmaxInvalid = 0x0800;

__device__ __forceinline__ uint32_t fnv_mix(uint32_t s, uint32_t v) {
  uint32_t t = s ^ v;
  return t * 16777619u ^ (t >> 17);
}

__device__ __forceinline__ uint16_t ld16(const uint8_t *p) {
  return (uint16_t)(p[0] | (p[1] << 8));
}

__device__ __forceinline__ uint32_t ld32u(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__global__ __launch_bounds__(256) void heap_scan_kernel(strom_heap_scan_args a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nwaves = gridDim.x * 4;
  for (uint32_t pg = blockIdx.x * 4 + (threadIdx.x >> 6); pg < a.npages; pg += nwaves) {
    const uint8_t *page = (const uint8_t *)a.pages + (uint64_t)pg * a.page_sz;
    const uint32_t *w = (const uint32_t *)page;
    // header (every lane reads the same 24 bytes: one broadcast line)
    const uint16_t pd_checksum = ld16(page + 8);
    const uint16_t pd_flags = ld16(page + 10);
    const uint16_t pd_lower = ld16(page + 12);
    const uint16_t pd_upper = ld16(page + 14);
    const uint16_t pd_special = ld16(page + 16);
    const uint16_t pd_psv = ld16(page + 18);
    uint32_t status = 0;
    const bool is_new = pd_upper == 0;
    if (is_new) {
      status |= STROM_PAGE_EMPTY;
    } else if (pd_lower < kSizeOfPageHeader || pd_lower > pd_upper || pd_upper > pd_special ||
               pd_special > a.page_sz || (pd_special & 7) || (pd_flags & ~0x7u) ||
               (pd_psv & 0xFF00u) != (a.page_sz & 0xFF00u)) {
      status |= STROM_PAGE_BAD_HEADER;
    }
    if ((a.flags & STROM_HEAP_VERIFY_CHECKSUM) && !is_new && !(status & STROM_PAGE_BAD_HEADER)) {
      // lanes 0..31 own one FNV sum each; lanes 32..63 duplicate (ignored)
      const uint32_t j = lane & 31;
      uint32_t s = g_pg_base[j];
      const uint32_t rows = a.page_sz / 128;
      for (uint32_t r = 0; r < rows; ++r) {
        uint32_t v = w[r * 32 + j];
        if (r == 0 && j == 2) v &= 0xffff0000u;  // pd_checksum reads as zero
        s = fnv_mix(s, v);
      }
      s = fnv_mix(s, 0);
      s = fnv_mix(s, 0);
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) s ^= __shfl_xor(s, o, 64);
      const uint32_t blkno = a.blknos ? a.blknos[pg] : a.blkno_base + pg;
      uint32_t c = ((s ^ blkno) % 65535u) + 1u;
      if ((uint16_t)c != pd_checksum) status |= STROM_PAGE_BAD_CHECKSUM;
    }
    if (lane == 0 && a.page_status) a.page_status[pg] = status;
    if (status & (STROM_PAGE_BAD_HEADER | STROM_PAGE_EMPTY)) continue;
    if ((status & STROM_PAGE_BAD_CHECKSUM)) continue;

    const uint32_t nitems = (pd_lower - kSizeOfPageHeader) / 4;
    for (uint32_t base = 0; base < nitems; base += 64) {
      const uint32_t i = base + lane;
      bool keep = false;
      if (i < nitems) {
        uint32_t lp = w[6 + i];
        uint32_t off = lp & 0x7fff, flags = (lp >> 15) & 3, len = lp >> 17;
        if (flags == kLpNormal && len >= 23 && off >= kSizeOfPageHeader && off + len <= a.page_sz) {
          const uint8_t *tup = page + off;
          uint16_t infomask = ld16(tup + 20);
          uint8_t hoff = tup[22];
          keep = true;
          if (a.flags & STROM_HEAP_SKIP_INVISIBLE) {
            bool xmin_ok = (infomask & kXminCommitted) && !(infomask & kXminInvalid);
            bool xmax_ok = (infomask & kXmaxInvalid) || (infomask & kXmaxLockOnly);
            keep = xmin_ok && xmax_ok;
          }
          if (keep && a.attr_off >= 0) {
            uint32_t at = hoff + (uint32_t)a.attr_off;
            if ((infomask & kHeapHasNull) || at + (uint32_t)a.attr_width > len) {
              keep = false;
            } else {
              int64_t v;
              if (a.attr_width == 8) {
                uint64_t lo = ld32u(tup + at), hi = ld32u(tup + at + 4);
                v = (int64_t)(lo | (hi << 32));
              } else {
                v = (int32_t)ld32u(tup + at);
              }
              keep = v >= a.lo && v <= a.hi;
            }
          }
        }
      }
      uint64_t mask = __ballot(keep);
      if (!mask) continue;
      uint32_t cnt = __popcll(mask);
      uint32_t start = 0;
      if (lane == 0) start = atomicAdd(a.out_count, cnt);
      start = __shfl(start, 0, 64);
      if (keep) {
        uint32_t rank = __popcll(mask & ((1ull << lane) - 1));
        uint32_t slot = start + rank;
        if (slot < a.out_cap) a.out_items[slot] = (pg << 16) | (i + 1);  // lineno is 1-based
      }
    }
  }
}

}  // namespace

extern "C" int strom_heap_scan(const strom_heap_scan_args *a, void *stream) {
  if (!a || !a->pages || !a->out_count) return -22;
  if (a->page_sz < 1024 || (a->page_sz & 127) || a->page_sz > 32768) return -22;
  if (a->attr_off >= 0 && a->attr_width != 4 && a->attr_width != 8) return -22;
  // (page << 16 | lineno) item ids address at most 65535 pages per call
  if (a->out_items && a->npages > 0xffffu) return -34;
  if (a->npages == 0) return 0;
  (void)hipMemsetAsync(a->out_count, 0, sizeof(uint32_t), (hipStream_t)stream);
  uint32_t grid = (a->npages + 3) / 4;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(heap_scan_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, *a);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
