// ingest.hip — the device side of the HBM ingest engine (csrc/engine/ingest.cc).
//
// The reference never copied anything on the GPU: its NVMe READs wrote
// straight into BAR pages (kmod/nvme_strom.c:1408-1482).  An unprivileged
// process reads into pinned host staging instead, and every staged request
// then has to reach HBM.  Round 1 issued one hipMemcpyAsync + hipEventRecord
// per (coalesced) request: 14-23 us of host CPU per call (profiles/r1s), which
// capped 4-128 KiB streams at 65-75% of the storage rate.  Here the copy is
// PULLED by the GPU: a small persistent grid polls a descriptor ring in
// fine-grained host memory, copies each staged range over PCIe with 16-byte
// loads (16 KiB in flight per wave), and publishes completion into a
// host-memory done[] word.  Posting a request costs the host one 32-byte
// store sequence; no HIP API call, no syscall.
//
// Protocol (host side: ingest.cc):
//   ring[s % nslots] = {src, dst, len, seq = s + 1}   host stores seq last
//   done[s % nslots] = s + 1                          device, after the bytes
//                                                     are written through to HBM
//   *stop != 0                                        every waiting wave exits
// A wave claims the next sequence number from a device counter, waits for
// the host to post it (or for stop), copies, and publishes.  Payload stores
// are write-through (sc1: the line leaves this XCD's L2), the wave drains
// its stores (s_waitcnt vmcnt(0)), then its lane 0 stores done[] at system
// scope: the valid hand-off form of
// MI355X_MICROARCH.md §visibility without an L2 write-back of the whole XCD
// (other kernels' dirty lines are not ours to flush).
//
// Termination: the host sets *stop whenever the engine goes idle (no request
// outstanding) and before it exits; every spin in here re-reads *stop, so the
// grid always drains.
//
// Consumer contract (what the visibility argument above covers): done[] is
// read by the HOST (ingest.cc), which then completes the task; the bytes
// are consumed by work ordered after that completion — a kernel launched
// afterwards (launch = acquire at agent scope, so every XCD's L2 sees the
// written-through lines), hipMemcpy/SDMA, or an RCCL collective issued
// afterwards (tests: test_pread_gpu_visible_to_next_kernel,
// test_pread_gpu_visible_to_sdma_readback).  An ALREADY-RUNNING kernel
// polling done[] on another XCD is NOT a supported consumer: it would need
// a system-scope acquire on done[] and an L2 invalidate of its own XCD
// (buffer_inv sc1) before reading the payload, and nothing in the engine
// does that — a fused ingest-then-decode pipeline would have to add both and
// its own test first.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u gv4u;   // global, not flat

struct IngestDesc {          // 32 bytes, ingest.cc writes the same layout
  uint64_t src;              // pinned host VA (fine-grained, GPU-mapped)
  uint64_t dst;              // device VA
  uint64_t len_tag;          // low 32 bits: byte count (multiple of 16)
  uint64_t seq;              // s + 1 once posted
};

constexpr int kThreads = 256;  // 4 waves, each an independent copier
constexpr int kUnroll = 16;    // 16-B loads in flight per lane (16 KiB per wave)
constexpr int kAuxSc1 = 16;    // buffer store cache policy: sc1 (write-through)

__device__ __forceinline__ uint64_t ld_sys(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// readfirstlane returns int: both halves go through uint32_t, or the low
// word's bit 31 would sign-extend over the high word
__device__ __forceinline__ uint64_t bcast64(uint64_t v) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
  return ((uint64_t)hi << 32) | lo;
}

// Every WAVE claims, copies and publishes descriptors on its own: a 4 KiB
// request is one 16-B load per lane of one wave, so the grid keeps 4x as
// many small descriptors in flight as a workgroup-wide claim did (round 4:
// 2.3 M descriptors/s from 8 workers queued behind 16 one-at-a-time
// workgroups, profiles/r4/engine).  Large descriptors move 16 KiB per wave
// per round trip.
__global__ __launch_bounds__(kThreads) void ingest_kernel(const IngestDesc *ring, uint64_t *done,
                                                          const uint64_t *stop, uint32_t *next,
                                                          uint32_t nslots, uint64_t base) {
  const uint32_t lane = threadIdx.x & 63;
  for (;;) {
    uint64_t s = 0, src = 0, dst = 0, len = 0;
    int ok = 0;
    if (lane == 0) {
      s = base + atomicAdd(next, 1u);
      const IngestDesc *d = ring + (s % nslots);
      for (uint32_t spin = 0;; ++spin) {
        if (ld_sys(&d->seq) == s + 1) {
          ok = 1;
          break;
        }
        if (ld_sys(stop)) break;
        if (spin < 256) __builtin_amdgcn_s_sleep(1);
        else __builtin_amdgcn_s_sleep(16);
      }
      // the field loads below are issued after the seq load returned
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (ok) {
        src = ld_sys(&d->src);
        dst = ld_sys(&d->dst);
        len = ld_sys(&d->len_tag);
      }
    }
    ok = __builtin_amdgcn_readfirstlane(ok);
    if (!ok) return;  // wave-uniform: stop requested
    s = bcast64(s);
    src = bcast64(src);
    dst = bcast64(dst);
    const uint32_t nbytes = __builtin_amdgcn_readfirstlane((uint32_t)len);
    gv4u *sp = (gv4u *)src;
    const uint32_t n16 = nbytes >> 4;
    // wave-uniform descriptor for the destination (SGPRs: no waterfall loop)
    __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)dst, (short)0, (int)nbytes, 0x00020000);
    for (uint32_t i = lane; i < n16; i += 64 * kUnroll) {
      v4u r[kUnroll];
#pragma unroll
      for (int k = 0; k < kUnroll; ++k) {
        const uint32_t idx = i + k * 64;
        if (idx < n16) r[k] = __builtin_nontemporal_load(sp + idx);
      }
#pragma unroll
      for (int k = 0; k < kUnroll; ++k) {
        const uint32_t idx = i + k * 64;
        if (idx < n16) __builtin_amdgcn_raw_buffer_store_b128(r[k], rsrc, (int)(idx * 16), 0, kAuxSc1);
      }
    }
    // the wave drains its own write-through stores, then one lane publishes
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(done + (s % nslots), s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace

// Launch `grid` workgroups of the ingest grid on `stream`.  `next` is a
// device u32 the caller zeroed on the same stream; sequence numbers handed out
// start at `base`.  Returns 0 or -EIO.
extern "C" int strom_ingest_kernel_launch(const void *ring, void *done, const void *stop,
                                          void *next, uint32_t nslots, uint64_t base,
                                          uint32_t grid, void *stream) {
  if (!ring || !done || !stop || !next || nslots == 0 || grid == 0 || grid > 1024) return -22;
  hipLaunchKernelGGL(ingest_kernel, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream,
                     (const IngestDesc *)ring, (uint64_t *)done, (const uint64_t *)stop,
                     (uint32_t *)next, nslots, base);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
