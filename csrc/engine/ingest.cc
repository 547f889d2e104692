// ingest.cc — host side of the HBM ingest engine (device side: csrc/kernels/ingest.hip).
//
// Staged storage reads reach HBM by a GPU-side pull instead of one
// hipMemcpyAsync + event per request (round 1: 14-23 us of host CPU per call,
// profiles/r1s/copy_coalesce.txt).  One Ingest per device owns:
//   ring_   nslots x 32-B descriptors in fine-grained host memory
//   done_   nslots x u64 completion words (written by the GPU, system scope)
//   stop_   one u64 the grid polls between descriptors
//   next_   a device u32 the grid's workgroups claim sequence numbers from
// Posting is a mutex-protected store sequence (fields, then seq with release
// order); completion is a plain load of done_[s % nslots].
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
  if (hipMalloc(&next_, 64) != hipSuccess ||
      hipStreamCreateWithFlags((hipStream_t *)&stream_, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags((hipEvent_t *)&end_ev_, hipEventDisableTiming) != hipSuccess) {
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
                                      post_seq_, grid_, stream_);
  if (rc) return rc;
  if (hipEventRecord((hipEvent_t)end_ev_, (hipStream_t)stream_) != hipSuccess) return -EIO;
  launched_ = true;
  return 0;
}

int Ingest::start_locked() {
  if (running_) return 0;
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
  running_ = true;
  nr_launch_++;
  return 0;
}

void Ingest::stop_locked() {
  if (!running_) return;
  __atomic_store_n(stop_, 1, __ATOMIC_SEQ_CST);
  running_ = false;
}

bool Ingest::post(const void *src, uint64_t dst, uint32_t len, uint64_t *seq) {
  uint32_t n = 0;
  return post_many(src, dst, len, len, seq, &n);
}

bool Ingest::post_many(const void *src, uint64_t dst, uint32_t len, uint32_t piece,
                       uint64_t *first, uint32_t *n) {
  if (len == 0 || (len & 15) || (((uint64_t)src | dst) & 15)) return false;
  piece = std::max<uint32_t>(16, piece & ~15u);
  std::lock_guard<std::mutex> g(mu_);
  if (dead_) return false;
  if (start_locked() != 0) {
    dead_ = true;
    return false;
  }
  *n = 0;
  for (uint32_t off = 0; off < len; off += piece) {
    uint64_t s;
    post_locked((const char *)src + off, dst + off, std::min(piece, len - off), &s);
    if (*n == 0) *first = s;
    ++*n;
  }
  return true;
}

bool Ingest::post_locked(const void *src, uint64_t dst, uint32_t len, uint64_t *seq) {
  const uint64_t s = post_seq_++;
  const uint32_t k = (uint32_t)(s % nslots_);
  // the slot's previous occupant (s - nslots) must be done: in-flight
  // requests are bounded by the workers' staging, far below nslots
  if (s >= nslots_)
    while (done_[k] < s - nslots_ + 1) _mm_pause();
  IngestDesc *d = (IngestDesc *)ring_ + k;
  d->src = (uint64_t)src;
  d->dst = dst;
  d->len_tag = len;
  __atomic_store_n(&d->seq, s + 1, __ATOMIC_RELEASE);
  outstanding_.fetch_add(1, std::memory_order_relaxed);
  *seq = s + 1;
  return true;
}

bool Ingest::is_done(uint64_t seq) const {
  return __atomic_load_n(&done_[(seq - 1) % nslots_], __ATOMIC_ACQUIRE) >= seq;
}

void Ingest::info(uint64_t *out) {
  std::lock_guard<std::mutex> g(mu_);
  out[0] = dead_ ? 0 : 1;
  out[1] = nr_launch_;
  out[2] = post_seq_;
  out[3] = (uint64_t)outstanding_.load();
}

void Ingest::retired(uint32_t n) { outstanding_.fetch_sub(n, std::memory_order_relaxed); }

void Ingest::idle() {
  if (outstanding_.load(std::memory_order_relaxed) != 0) return;
  std::lock_guard<std::mutex> g(mu_);
  if (outstanding_.load() == 0) stop_locked();
}

void Ingest::shutdown() {
  std::lock_guard<std::mutex> g(mu_);
  stop_locked();
  if (launched_) {
    // bounded: every waiting workgroup re-reads stop within microseconds
    const uint64_t end = mono_ns() + 2000000000ull;
    while (hipEventQuery((hipEvent_t)end_ev_) == hipErrorNotReady && mono_ns() < end)
      _mm_pause();
    launched_ = false;
  }
  dead_ = true;
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
