// ingest.cc — host side of the HBM ingest engine (device side: csrc/kernels/ingest.hip).
//
// Staged storage reads reach HBM by a GPU-side pull instead of one
// hipMemcpyAsync + event per request (round 1: 14-23 us of host CPU per call,
// profiles/r1s/copy_coalesce.txt).  One Ingest per device owns:
//   ring_   nslots x 32-B descriptors in fine-grained host memory
//   done_   nslots x u64 completion words (written by the GPU, system scope)
//   stop_   one u64 the grid polls between descriptors
//   next_   a device u32 the grid's workgroups claim sequence numbers from
// Posting is lock-free: a batch reserves its sequence numbers with one
// fetch_add and stores each descriptor (fields, then seq with release order);
// completion is a plain load of done_[s % nslots].
//
// Lifecycle: the grid is launched on the first post after an idle period and
// stopped by the first worker that goes to sleep with nothing outstanding
// (IoEngine::Worker::run), so a device-wide synchronize (torch.cuda.synchronize,
// hipDeviceSynchronize) never waits on an idle persistent grid for longer than
// the workers' idle spin.  A relaunch first waits for the previous grid to exit
// (its end event), then restarts the device counter at the host's sequence
// number.  atexit stops every grid before the HIP runtime tears down.
#include <hip/hip_runtime_api.h>  // host API only: builds with g++ (sanitizers)
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <x86intrin.h>

#include "engine.h"

// Device-side launcher (csrc/kernels/ingest.hip).  Weak so that host-only
// builds (the sanitizer self-tests) link without device code: there the
// engine keeps the SDMA path.
extern "C" __attribute__((weak)) int strom_ingest_kernel_launch(const void *, void *, const void *,
                                                                void *, uint32_t, uint64_t,
                                                                uint32_t, void *) {
  return -ENOSYS;
}

namespace strom {

namespace {
struct IngestDesc {
  uint64_t src;
  uint64_t dst;
  uint64_t len_tag;
  volatile uint64_t seq;
};
static_assert(sizeof(IngestDesc) == 32, "ingest descriptor layout (ingest.hip)");

std::mutex g_ing_mu;
std::map<int, Ingest *> g_ing;
bool g_ing_atexit = false;

void stop_all_at_exit() {
  std::lock_guard<std::mutex> g(g_ing_mu);
  for (auto &kv : g_ing)
    if (kv.second) kv.second->shutdown();
}
}  // namespace

Ingest *Ingest::get(int device) {
  if (device < 0 || !config().ingest || !hip::available()) return nullptr;
  std::lock_guard<std::mutex> g(g_ing_mu);
  auto it = g_ing.find(device);
  if (it != g_ing.end()) return it->second;
  Ingest *ing = new Ingest(device);
  if (!ing->init()) {
    STROM_LOG(0, "device %d: ingest grid unavailable, staged copies use SDMA", device);
    delete ing;
    ing = nullptr;
  } else if (!g_ing_atexit) {
    g_ing_atexit = true;
    atexit(stop_all_at_exit);  // registered after HIP's own handlers: runs before them
  }
  g_ing[device] = ing;
  return ing;
}

Ingest::Ingest(int device) : device_(device) {}

bool Ingest::init() {
  nslots_ = 4096;
  grid_ = (uint32_t)std::max(1, std::min(256, config().ingest_grid));
  if (hipSetDevice(device_) != hipSuccess) return false;
  const size_t bytes = nslots_ * sizeof(IngestDesc) + nslots_ * sizeof(uint64_t) + 64;
  void *h = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  memset(h, 0, bytes);
  host_ = h;
  ring_ = h;
  done_ = (volatile uint64_t *)((char *)h + nslots_ * sizeof(IngestDesc));
  stop_ = (volatile uint64_t *)((char *)done_ + nslots_ * sizeof(uint64_t));
  int prio_least = 0, prio_greatest = 0;
  if (config().ingest_prio && hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess)
    prio_greatest = 0;
  if (hipMalloc(&next_, 64) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  // The grid needs a hardware queue of its own: a kernel queued behind it
  // on a shared queue waits until the grid goes idle, and a grid relaunch
  // waits behind that kernel (round 5 trace: Arrow ZSTD decodes on the
  // grid's queue ran only between reads, profiles/r5/zstd_arrow).  HIP
  // hands normal-priority streams GPU_MAX_HW_QUEUES (4) queues round-robin,
  // so a process with more streams aliases them; a CU-masked stream always
  // gets a new queue (tools/probe/hwq_probe.py), so the grid's stream is one
  // with every CU in its mask.  ingest_prio=1 (default): a greatest-priority
  // non-blocking stream instead — the first one of its priority also gets a
  // queue of its own, and unlike the CU-masked stream (created blocking:
  // there is no flags argument) it is not ordered with the NULL stream by
  // HIP's rules.  (Round 5 A/B: once the Arrow scan stopped ordering its
  // decode streams after the default stream, both kinds overlap its decodes
  // with the reads, profiles/r5/zstd_arrow/grid_stream_ab.)
  bool made = false;
  if (!config().ingest_prio) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_) == hipSuccess &&
        cus > 0 && cus <= 1024) {
      uint32_t mask[32] = {0};
      for (int i = 0; i < cus; ++i) mask[i / 32] |= 1u << (i % 32);
      made = hipExtStreamCreateWithCUMask((hipStream_t *)&stream_, (uint32_t)((cus + 31) / 32),
                                          mask) == hipSuccess;
      if (!made) (void)hipGetLastError();
    }
  }
  if (!made && hipStreamCreateWithPriority((hipStream_t *)&stream_, hipStreamNonBlocking,
                                           config().ingest_prio ? prio_greatest : 0) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (hipEventCreateWithFlags((hipEvent_t *)&end_ev_, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  // probe: one launch that is told to stop at once must come back
  *stop_ = 1;
  if (launch_grid() != 0) return false;
  if (hipEventSynchronize((hipEvent_t)end_ev_) != hipSuccess) return false;
  launched_ = false;
  return true;
}

int Ingest::launch_grid() {
  (void)hipSetDevice(device_);
  if (hipMemsetAsync(next_, 0, sizeof(uint32_t), (hipStream_t)stream_) != hipSuccess) return -EIO;
  int rc = strom_ingest_kernel_launch(ring_, (void *)done_, (const void *)stop_, next_, nslots_,
                                      post_seq_.load(), grid_, stream_);
  if (rc) return rc;
  if (hipEventRecord((hipEvent_t)end_ev_, (hipStream_t)stream_) != hipSuccess) return -EIO;
  launched_ = true;
  return 0;
}

// under mu_, with the running bit clear: no descriptor is reserved until
// the bit is set again, so post_seq_ is the first number the grid serves
int Ingest::start_locked() {
  if (state_.load() & 1) return 0;
  if (launched_) {
    // the previous grid was told to stop: it must be gone before the
    // device counter restarts
    (void)hipSetDevice(device_);
    if (hipEventSynchronize((hipEvent_t)end_ev_) != hipSuccess) return -EIO;
    launched_ = false;
  }
  __atomic_store_n(stop_, 0, __ATOMIC_SEQ_CST);
  int rc = launch_grid();
  if (rc) return rc;
  state_.fetch_or(1);
  nr_launch_++;
  return 0;
}

bool Ingest::post(const void *src, uint64_t dst, uint32_t len, uint64_t *seq) {
  uint32_t n = 0;
  return post_many(src, dst, len, len, seq, &n);
}

bool Ingest::post_many(const void *src, uint64_t dst, uint32_t len, uint32_t piece,
                       uint64_t *first, uint32_t *n) {
  Run r{src, dst, len, false, 0, 0};
  post_runs(&r, 1, piece);
  *first = r.first;
  *n = r.n;
  return r.ok;
}

// Lock-free posting: one RMW on state_ and one on post_seq_ for the whole
// batch; the mutex is taken only when the grid has to be (re)started.
void Ingest::post_runs(Run *runs, size_t nruns, uint32_t piece) {
  piece = std::max<uint32_t>(16, piece & ~15u);
  uint64_t total = 0;
  for (size_t i = 0; i < nruns; ++i) {
    Run &r = runs[i];
    r.n = 0;
    r.ok = r.len != 0 && !(r.len & 15) && !(((uint64_t)r.src | r.dst) & 15);
    if (r.ok) total += (r.len + piece - 1) / piece;
  }
  auto fail_all = [&] {
    for (size_t i = 0; i < nruns; ++i) runs[i].ok = false;
  };
  if (total == 0) return;
  if (dead_.load(std::memory_order_relaxed)) return fail_all();
  const uint64_t old = state_.fetch_add(2 * total);
  if (!(old & 1)) {
    std::lock_guard<std::mutex> g(mu_);
    if (dead_.load() || start_locked() != 0) {
      dead_.store(true);
      state_.fetch_sub(2 * total);
      return fail_all();
    }
  }
  uint64_t s = post_seq_.fetch_add(total);
  for (size_t i = 0; i < nruns; ++i) {
    Run &r = runs[i];
    if (!r.ok) continue;
    r.first = s + 1;
    for (uint32_t off = 0; off < r.len; off += piece, ++s, ++r.n)
      if (!write_desc(s, (const char *)r.src + off, r.dst + off, std::min(piece, r.len - off))) {
        // the grid is gone (shutdown): this and the later runs take the
        // caller's SDMA fallback; their reservations are never served
        for (size_t j = i; j < nruns; ++j) runs[j].ok = false;
        return;
      }
  }
}

bool Ingest::write_desc(uint64_t s, const void *src, uint64_t dst, uint32_t len) {
  const uint32_t k = (uint32_t)(s % nslots_);
  // the slot's previous occupant (s - nslots) must be done: in-flight
  // requests are bounded by the workers' staging, far below nslots.  A
  // poster that reserved before shutdown() and finds the grid gone would
  // spin here forever: gone_ ends the wait.
  if (s >= nslots_)
    while (__atomic_load_n(&done_[k], __ATOMIC_ACQUIRE) < s - nslots_ + 1) {
      if (gone_.load(std::memory_order_acquire)) return false;
      _mm_pause();
    }
  IngestDesc *d = (IngestDesc *)ring_ + k;
  d->src = (uint64_t)src;
  d->dst = dst;
  d->len_tag = len;
  __atomic_store_n(&d->seq, s + 1, __ATOMIC_RELEASE);
  return true;
}

bool Ingest::is_done(uint64_t seq) const {
  return __atomic_load_n(&done_[(seq - 1) % nslots_], __ATOMIC_ACQUIRE) >= seq;
}

void Ingest::info(uint64_t *out) {
  out[0] = dead_.load() ? 0 : 1;
  {
    std::lock_guard<std::mutex> g(mu_);
    out[1] = nr_launch_;
  }
  out[2] = post_seq_.load();
  out[3] = state_.load() >> 1;
}

void Ingest::retired(uint32_t n) { state_.fetch_sub(2ull * n); }

void Ingest::idle() {
  if (state_.load(std::memory_order_relaxed) != 1) return;  // stopped, or work outstanding
  std::lock_guard<std::mutex> g(mu_);
  uint64_t running_idle = 1;
  if (state_.compare_exchange_strong(running_idle, 0)) __atomic_store_n(stop_, 1, __ATOMIC_SEQ_CST);
}

void Ingest::shutdown() {
  {
    std::lock_guard<std::mutex> g(mu_);
    dead_.store(true);                 // no new reservations from here on
  }
  // a poster that passed the dead_ check and reserved while the grid was
  // running gets its descriptors served before the grid is told to stop
  // (bounded: at exit a reservation may never be retired)
  const uint64_t drain_end = mono_ns() + 200000000ull;
  while ((state_.load() >> 1) != 0 && (state_.load() & 1) && mono_ns() < drain_end) _mm_pause();
  std::lock_guard<std::mutex> g(mu_);
  state_.fetch_and(~1ull);
  __atomic_store_n(stop_, 1, __ATOMIC_SEQ_CST);
  if (launched_) {
    // bounded: every waiting wave re-reads stop within microseconds
    const uint64_t end = mono_ns() + 2000000000ull;
    while (hipEventQuery((hipEvent_t)end_ev_) == hipErrorNotReady && mono_ns() < end)
      _mm_pause();
    launched_ = false;
  }
  gone_.store(true, std::memory_order_release);
}

}  // namespace strom

// Ingest grid counters of a device: out = {available, grid launches,
// descriptors posted, descriptors outstanding}.  -ENODEV when the grid
// cannot run there (disabled, host-only build, launch failure).
extern "C" int strom_ingest_info(int device, uint64_t *out) {
  strom::Ingest *ing = strom::Ingest::get(device);
  if (!ing) return -ENODEV;
  ing->info(out);
  return 0;
}
