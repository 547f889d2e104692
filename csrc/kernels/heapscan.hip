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

__device__ __forceinline__ bool tuple_keep(const strom_heap_scan_args &a, const uint8_t *pg,
                                           uint32_t lp, bool all_visible) {
  const uint32_t off = lp & 0x7fff, flags = (lp >> 15) & 3, len = lp >> 17;
  if (flags != kLpNormal || len < 23 || off < kSizeOfPageHeader || off + len > a.page_sz ||
      (off & 1))
    return false;
  const uint32_t w20 = lds_u32(pg, off + 20);  // t_infomask (16) | t_hoff (8) | bits
  const uint32_t infomask = w20 & 0xffff, hoff = (w20 >> 16) & 0xff;
  if ((a.flags & STROM_HEAP_SKIP_INVISIBLE) && !all_visible) {
    // no clog here: only hint bits that prove visibility count
    if (!(infomask & kXminCommitted)) return false;
    if (!(infomask & (kXmaxInvalid | kXmaxLockOnly))) return false;
  }
  if (a.attr_off < 0) return true;
  const uint32_t at = hoff + (uint32_t)a.attr_off;
  if ((infomask & kHeapHasNull) || at + (uint32_t)a.attr_width > len) return false;
  int64_t v;
  if (a.attr_width == 8) {
    const uint64_t lo = lds_u32(pg, off + at), hi = lds_u32(pg, off + at + 4);
    v = (int64_t)(lo | (hi << 32));
  } else {
    v = (int32_t)lds_u32(pg, off + at);
  }
  return v >= a.lo && v <= a.hi;
}

// PAGE = page size known at compile time (0: a.page_sz at run time).  Each
// lane moves NV 16-byte pieces of its wave's page per page.  A workgroup
// handles kWaves x kPerWave pages per output reservation: one same-address
// atomicAdd per 32 pages (round 1: per 4 pages, which capped scans where
// every page has qualifying rows at ~88 atomics/us, MI355X_MICROARCH.md
// row "dequeue" — 2.1 TB/s).
constexpr int kPerWave = 8;

template <int PAGE>
__global__ __launch_bounds__(256) void heap_scan_kernel(strom_heap_scan_args a, uint32_t maxchunks,
                                                        uint32_t ppw) {
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
        const uint32_t status = page_status(a, mypage, h, pg, lane);
        if (lane == 0 && a.page_status) a.page_status[pg] = status;
        if (status == 0) {
          const bool all_visible = (h.flags & kPdAllVisible) != 0;
          const uint32_t nitems = (h.lower - kSizeOfPageHeader) / 4;
          nchunks = (nitems + 63) / 64;
          for (uint32_t c = 0; c < nchunks; ++c) {
            const uint32_t i = c * 64 + lane;
            const bool keep =
                i < nitems && tuple_keep(a, mypage, lds_u32a(mypage, kSizeOfPageHeader + 4 * i),
                                         all_visible);
            const uint64_t m = __ballot(keep);
            if (lane == 0) masks[j * maxchunks + c] = m;
            count += __popcll(m);
          }
        }
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

}  // namespace

extern "C" int strom_heap_scan(const strom_heap_scan_args *a, void *stream) {
  if (!a || !a->pages || !a->out_count) return -22;
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
  if (a->page_sz == 8192)
    hipLaunchKernelGGL(heap_scan_kernel<8192>, dim3(grid), dim3(256), lds, st, *a, maxchunks, ppw);
  else
    hipLaunchKernelGGL(heap_scan_kernel<0>, dim3(grid), dim3(256), lds, st, *a, maxchunks, ppw);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
