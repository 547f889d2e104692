// io.cc — request execution: io_uring / pread workers with HBM staging.
//
// Replaces the reference's PRP-list pool + blk-mq async submit/complete
// (kmod/nvme_strom.c:822-1120) for an unprivileged process on MI355X:
//
//   caller thread ── submit() ──► per-worker queue (batched, one lock)
//   worker k:  io_uring READs (O_DIRECT) up to queue_depth in flight
//              ├─ host destination (SSD2RAM): done on CQE
//              └─ HBM destination: CQE ► descriptor(s) posted to the device's
//                 ingest grid (ingest.cc: the GPU pulls the staged bytes into
//                 HBM; no HIP call on this thread); the worker polls the
//                 done words, returns the pinned slot and puts the task.
//                 Without the grid (ingest=0, host-only builds): small
//                 requests are CPU-stored through the large BAR, larger ones
//                 go out as coalesced hipMemcpyAsync SDMA copies + events.
//
// Each worker owns its ring, its staging slots and its stream, so the hot
// path takes no shared lock.  Workers are pinned to the CPUs of the GPU's
// NUMA node and allocate staging there (PAR5 in SURVEY §2.3).
#include <hip/hip_runtime_api.h>  // host API only: builds with g++ (sanitizers)
#include <errno.h>
#include <fcntl.h>
#include <linux/io_uring.h>
#include <sched.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <unistd.h>
#include <x86intrin.h>

#include <algorithm>
#include <functional>
#include <fstream>

#include "engine.h"

#ifndef MPOL_PREFERRED
#define MPOL_PREFERRED 1
#endif

namespace strom {

// ------------------------------------------------------------ raw io_uring
class Uring {
 public:
  ~Uring() { close_ring(); }
  int init(unsigned entries) {
    io_uring_params p;
    memset(&p, 0, sizeof p);
    fd_ = (int)syscall(__NR_io_uring_setup, entries, &p);
    if (fd_ < 0) return -errno;
    sq_sz_ = p.sq_off.array + p.sq_entries * sizeof(unsigned);
    cq_sz_ = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
    bool single = p.features & IORING_FEAT_SINGLE_MMAP;
    if (single) sq_sz_ = cq_sz_ = std::max(sq_sz_, cq_sz_);
    sq_ptr_ = mmap(nullptr, sq_sz_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_,
                   IORING_OFF_SQ_RING);
    if (sq_ptr_ == MAP_FAILED) return fail();
    cq_ptr_ = single ? sq_ptr_
                     : mmap(nullptr, cq_sz_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE,
                            fd_, IORING_OFF_CQ_RING);
    if (cq_ptr_ == MAP_FAILED) return fail();
    sqe_sz_ = p.sq_entries * sizeof(io_uring_sqe);
    sqes_ = (io_uring_sqe *)mmap(nullptr, sqe_sz_, PROT_READ | PROT_WRITE,
                                 MAP_SHARED | MAP_POPULATE, fd_, IORING_OFF_SQES);
    if (sqes_ == MAP_FAILED) return fail();
    char *sq = (char *)sq_ptr_, *cq = (char *)cq_ptr_;
    sq_head_ = (unsigned *)(sq + p.sq_off.head);
    sq_tail_ = (unsigned *)(sq + p.sq_off.tail);
    sq_mask_ = *(unsigned *)(sq + p.sq_off.ring_mask);
    sq_array_ = (unsigned *)(sq + p.sq_off.array);
    cq_head_ = (unsigned *)(cq + p.cq_off.head);
    cq_tail_ = (unsigned *)(cq + p.cq_off.tail);
    cq_mask_ = *(unsigned *)(cq + p.cq_off.ring_mask);
    cqes_ = (io_uring_cqe *)(cq + p.cq_off.cqes);
    entries_ = p.sq_entries;
    return 0;
  }
  io_uring_sqe *next_sqe() {
    unsigned tail = *sq_tail_;
    unsigned head = __atomic_load_n(sq_head_, __ATOMIC_ACQUIRE);
    if (tail - head >= entries_) return nullptr;
    unsigned idx = tail & sq_mask_;
    io_uring_sqe *s = &sqes_[idx];
    memset(s, 0, sizeof *s);
    sq_array_[idx] = idx;
    __atomic_store_n(sq_tail_, tail + 1, __ATOMIC_RELEASE);
    ++pending_;
    return s;
  }
  int enter(unsigned min_complete) {
    unsigned flags = min_complete ? IORING_ENTER_GETEVENTS : 0;
    int r = (int)syscall(__NR_io_uring_enter, fd_, pending_, min_complete, flags, nullptr, 0);
    if (r < 0) return -errno;
    pending_ -= (unsigned)r <= pending_ ? (unsigned)r : pending_;
    return r;
  }
  bool peek(io_uring_cqe *out) {
    unsigned head = *cq_head_;
    if (head == __atomic_load_n(cq_tail_, __ATOMIC_ACQUIRE)) return false;
    *out = cqes_[head & cq_mask_];
    __atomic_store_n(cq_head_, head + 1, __ATOMIC_RELEASE);
    return true;
  }
  unsigned pending() const { return pending_; }
  bool ok() const { return fd_ >= 0; }
  void unregister_buffers() {
    (void)syscall(__NR_io_uring_register, fd_, IORING_UNREGISTER_BUFFERS, nullptr, 0u);
  }
  // one fixed buffer (index 0) covering [p, p+len); -errno when refused
  int register_buffer(void *p, size_t len) {
    iovec iov{p, len};
    int r = (int)syscall(__NR_io_uring_register, fd_, IORING_REGISTER_BUFFERS, &iov, 1u);
    return r < 0 ? -errno : 0;
  }

 private:
  int fail() {
    int e = errno;
    close_ring();
    return -e;
  }
  void close_ring() {
    if (sqes_ && sqes_ != MAP_FAILED) munmap(sqes_, sqe_sz_);
    if (cq_ptr_ && cq_ptr_ != MAP_FAILED && cq_ptr_ != sq_ptr_) munmap(cq_ptr_, cq_sz_);
    if (sq_ptr_ && sq_ptr_ != MAP_FAILED) munmap(sq_ptr_, sq_sz_);
    if (fd_ >= 0) close(fd_);
    fd_ = -1;
    sqes_ = nullptr;
    sq_ptr_ = cq_ptr_ = nullptr;
  }
  int fd_ = -1;
  void *sq_ptr_ = nullptr, *cq_ptr_ = nullptr;
  size_t sq_sz_ = 0, cq_sz_ = 0, sqe_sz_ = 0;
  io_uring_sqe *sqes_ = nullptr;
  io_uring_cqe *cqes_ = nullptr;
  unsigned *sq_head_ = nullptr, *sq_tail_ = nullptr, *sq_array_ = nullptr;
  unsigned *cq_head_ = nullptr, *cq_tail_ = nullptr;
  unsigned sq_mask_ = 0, cq_mask_ = 0, entries_ = 0, pending_ = 0;
};

// worker-level I/O facts for tools (strom_io_info)
static std::atomic<uint64_t> g_fixed_workers{0}, g_fixed_refused{0}, g_fixed_errno{0};

// ------------------------------------------------------------- completion
void finish_request(IoReq &r, long status) {
  Stats &st = stats();
  st.nr_ssd2gpu.fetch_add(1, std::memory_order_relaxed);
  st.clk_ssd2gpu.fetch_add(tsc_now() - r.t_submit_tsc, std::memory_order_relaxed);
  st.inflight_dec();
  if (r.gmap) {
    if (r.gmap->inflight.fetch_sub(1) == 1 && r.gmap->draining.load()) {
      std::lock_guard<std::mutex> g(r.gmap->mu);
      r.gmap->cv.notify_all();
    }
  }
  if (r.task) tasks().put(r.task, status);
  else if (r.status_out) *r.status_out = status;
}

// read [off, off+len) fully; returns bytes read or -errno.
static long pread_full(int fd, uint8_t *buf, uint32_t len, uint64_t off) {
  uint32_t done = 0;
  while (done < len) {
    ssize_t n = pread(fd, buf + done, len - done, (off_t)(off + done));
    if (n < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (n == 0) break;
    done += (uint32_t)n;
  }
  return done;
}

// Post-process a storage read of `len` bytes into dst that returned `got`
// (bytes or -errno): O_DIRECT refusal falls back to a buffered read, a read
// shorter than the bytes before EOF is an error, the tail past EOF is
// zero-filled.  Returns 0 or -errno.
static long finalize_read(const IoReq &r, uint8_t *dst, uint32_t len, long got) {
  if (got == -EINVAL && r.fd_buffered >= 0 && r.fd_buffered != r.fd)
    got = pread_full(r.fd_buffered, dst, len, r.off);
  if (got < 0) return got;
  if ((uint32_t)got < r.valid) return -EIO;
  if ((uint32_t)got < r.len) memset(dst + got, 0, r.len - (uint32_t)got);
  return 0;
}

// ------------------------------------------------------------------ worker
// Phase attribution of a worker's loop (config io_prof): every TSC cycle of
// the loop is charged to exactly one phase ("lap" timer), so the phases sum
// to the worker's wall time.
enum ProfPhase {
  PF_IDLE,     // idle spin + sleeping for work
  PF_TAKE,     // taking the queue (lock + swap)
  PF_START,    // preparing reads (SQEs, staging slots)
  PF_SUBMIT,   // io_uring_enter to submit (page-cache reads copy in here)
  PF_REAP,     // CQE handling, read finalisation
  PF_BAR,      // CPU stores through the large BAR
  PF_POST,     // ingest descriptors (lock + stores)
  PF_HDP,      // sfence + HDP flush, once per batch and mapping
  PF_FINISH,   // publishing a batch: stats, mapping counts, task puts
  PF_RETIRE,   // polling ingest done words / SDMA events
  PF_WAIT,     // blocked on a read or an HBM copy
};
static_assert(PF_WAIT + 1 == IoEngine::kProfPhases, "phase count");
enum ProfCount { PC_REQ, PC_BATCH, PC_ENTER, PC_SLEEP, PC_DESC };
static_assert(PC_DESC + 1 == IoEngine::kProfCounts, "count count");

// pin the calling thread to NUMA node `node`'s CPUs (within its allowed
// set) and prefer that node's memory; no-op for node < 0
static void bind_to_node(int node) {
  if (node < 0) return;
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!(f >> list)) return;
  cpu_set_t want, allowed, use;
  CPU_ZERO(&want);
  size_t pos = 0;
  while (pos < list.size()) {
    size_t comma = list.find(',', pos);
    std::string part = list.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
    int a = 0, b = 0;
    if (sscanf(part.c_str(), "%d-%d", &a, &b) == 2) {
      for (int c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(c, &want);
    } else if (sscanf(part.c_str(), "%d", &a) == 1 && a < CPU_SETSIZE) {
      CPU_SET(a, &want);
    }
    if (comma == std::string::npos) break;
    pos = comma + 1;
  }
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
  CPU_AND(&use, &want, &allowed);
  if (CPU_COUNT(&use) > 0) sched_setaffinity(0, sizeof use, &use);
  unsigned long mask[16] = {0};
  if (node < 1024) {
    mask[node / 64] = 1ul << (node % 64);
    syscall(SYS_set_mempolicy, MPOL_PREFERRED, mask, 1024ul);
  }
}

struct IoEngine::Worker {
  struct Slot {
    uint8_t *buf = nullptr;
    hipEvent_t ev = nullptr;
    int ev_dev = -1;
    IoReq req;
    uint64_t t_copy_ns = 0;
    int ev_slot = -1;    // slot whose event covers this slot's copy
    Ingest *ing = nullptr;   // ingest descriptors seq_first .. + nseq - 1
    uint64_t seq_first = 0;
    uint32_t nseq = 0;
    uint32_t nret = 0;   // descriptors this slot reports retired (run head)
    uint32_t held = 0;   // bytes of the in-flight byte budget its request holds
  };
  struct Ctx {           // one in-flight storage read
    IoReq req;
    int slot = -1;       // staging slot (HBM destination) or -1
    uint8_t *dst = nullptr;
    uint32_t len = 0;
    uint64_t t0 = 0;
    long got = 0;        // fake backend: the read's result, delivered later
    uint64_t seq = 0;    // fake backend: submission order
  };

  // Fake namespace (backend=fake, CPU tests): reads are served from the
  // file at submission, but their completions are held in a device queue
  // and delivered in a seeded random order once the queue is full or the
  // worker runs dry — what an NVMe controller may do, and what the task
  // refcounts, landing order and staging-slot recycling must survive.
  std::vector<Ctx> fake_cq;
  uint64_t fake_rng = 0, fake_seq = 0, fake_next = 0;

  uint64_t fake_rand() {
    fake_rng ^= fake_rng << 13;
    fake_rng ^= fake_rng >> 7;
    fake_rng ^= fake_rng << 17;
    return fake_rng;
  }

  void reap_fake() {
    now_ns = mono_ns();
    while (!fake_cq.empty()) {
      const size_t i = (size_t)(fake_rand() % fake_cq.size());
      Ctx c = fake_cq[i];
      fake_cq[i] = fake_cq.back();
      fake_cq.pop_back();
      --reads_inflight;
      faults().fake_completions.fetch_add(1, std::memory_order_relaxed);
      if (c.seq != fake_next) faults().fake_reordered.fetch_add(1, std::memory_order_relaxed);
      fake_next = c.seq + 1;
      on_read_done(c, c.got);
    }
    post_ingest();
    flush_staged();
  }

  int idx = 0;
  Config cfg;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<IoReq> q;             // handed over in slices (one copy, no
                                    // per-request allocation)
  bool stop = false;
  bool sleeping = false;            // in cv.wait (guarded by mu)
  std::atomic<int> pending{0};      // q non-empty hint for the idle spin
  std::vector<Slot> slots;
  uint8_t *staging = nullptr;     // one registered region, cut into slots
  size_t staging_bytes = 0;
  bool staging_thp = false;
  bool fixed = false;             // staging registered with the ring (READ_FIXED)
  std::deque<int> free_slots;     // FIFO: consecutive requests get adjacent slots
  size_t stage_inflight = 0;      // bytes of requests holding a slot (stage_budget)
  std::deque<int> copying;        // FIFO of slots with copies in flight
  std::vector<int> staged;        // reads done, HBM copy not yet issued
  std::vector<int> ing_staged;    // reads done, ingest descriptor not yet posted
  std::vector<int> ingesting;     // slots whose bytes the ingest grid is pulling
  std::vector<std::pair<int, Ingest *>> ings;  // device -> ingest grid (or null)
  std::vector<Ingest::Run> runs;  // post_ingest scratch: ranges and their
  std::vector<std::pair<size_t, size_t>> span;  // [lo, hi) in ing_staged
  std::vector<hipStream_t> streams;
  int cur_dev = -2;
  Uring ring;
  std::vector<Ctx> ctx;
  std::vector<int> free_ctx;
  int reads_inflight = 0;
  int numa_node = -1;
  uint64_t now_ns = 0;            // one clock read per batch of completions

  // ---- completion batching.  Requests finished in one pass of the loop are
  // published together by flush_done(): one RMW per task, per mapping and per
  // counter for the batch, and one sfence + HDP flush per mapping for all its
  // BAR stores.  Per request these were ~8 RMWs on lines shared with the
  // submitter and the other workers.
  struct Fin {
    Task *task;
    GpuMapping *gmap;
    long status;
    long *status_out;
  };
  std::vector<Fin> fin;
  uint64_t fin_clk = 0;           // sum of (completion - submission) TSC cycles
  std::vector<std::pair<GpuMapping *, const uint8_t *>> bar_dirty;
  uint32_t nbar = 0;              // BAR-stored requests in this batch
  uint64_t ndesc = 0;             // HBM copies / ingest descriptors issued
  uint64_t copy_clk = 0;
  uint32_t lh_io[STROM_HIST_BUCKETS] = {}, lh_copy[STROM_HIST_BUCKETS] = {};
  uint64_t lh_io_mask = 0, lh_copy_mask = 0;

  // ---- attribution (config io_prof).  Single writer (this worker):
  // relaxed load + store, no RMW on the hot path; IoEngine::prof reads them
  // concurrently and "resets" by moving its own baseline (prof_base_*,
  // guarded by IoEngine::prof_mu_), never by writing the worker's counters.
  bool prof_on = false;
  uint64_t prof_t = 0;
  std::atomic<uint64_t> prof_cyc[kProfPhases] = {};
  std::atomic<uint64_t> prof_cnt[kProfCounts] = {};
  uint64_t prof_base_cyc[kProfPhases] = {};
  uint64_t prof_base_cnt[kProfCounts] = {};
  static void bump(std::atomic<uint64_t> &c, uint64_t d) {
    c.store(c.load(std::memory_order_relaxed) + d, std::memory_order_relaxed);
  }
  void lap(int k) {
    if (__builtin_expect(prof_on, 0)) {
      const uint64_t t = tsc_now();
      bump(prof_cyc[k], t - prof_t);
      prof_t = t;
    }
  }

  void hist_io(uint64_t ns) {
    const int b = Hist::bucket(ns);
    ++lh_io[b];
    lh_io_mask |= 1ull << b;
  }
  void hist_copy(uint64_t ns, uint32_t n = 1) {
    const int b = Hist::bucket(ns);
    lh_copy[b] += n;
    lh_copy_mask |= 1ull << b;
  }

  void complete(const IoReq &r, long status) {
    fin.push_back(Fin{r.task, r.gmap, status, r.status_out});
    fin_clk += tsc_now() - r.t_submit_tsc;
  }

  void flush_done() {
    if (fin.empty()) return;
    for (auto &b : bar_dirty) b.first->bar_flush(b.second, true);
    bar_dirty.clear();
    if (nbar) {
      hist_copy(mono_ns() - now_ns, nbar);
      nbar = 0;
    }
    lap(PF_HDP);
    Stats &st = stats();
    const uint64_t n = fin.size();
    st.nr_ssd2gpu.fetch_add(n, std::memory_order_relaxed);
    st.clk_ssd2gpu.fetch_add(fin_clk, std::memory_order_relaxed);
    st.inflight_dec(n);
    fin_clk = 0;
    if (ndesc) {
      st.nr_debug[0].fetch_add(ndesc, std::memory_order_relaxed);
      st.clk_debug[0].fetch_add(copy_clk, std::memory_order_relaxed);
      ndesc = copy_clk = 0;
    }
    for (uint64_t m = lh_io_mask; m; m &= m - 1) {
      const int b = __builtin_ctzll(m);
      st.io_ns.b[b].fetch_add(lh_io[b], std::memory_order_relaxed);
      lh_io[b] = 0;
    }
    for (uint64_t m = lh_copy_mask; m; m &= m - 1) {
      const int b = __builtin_ctzll(m);
      st.copy_ns.b[b].fetch_add(lh_copy[b], std::memory_order_relaxed);
      lh_copy[b] = 0;
    }
    lh_io_mask = lh_copy_mask = 0;
    // mappings first: a task's last put may drop the mapping's last owner
    for (size_t i = 0; i < fin.size();) {
      GpuMapping *g = fin[i].gmap;
      size_t j = i + 1;
      while (j < fin.size() && fin[j].gmap == g) ++j;
      if (g) {
        const int k = (int)(j - i);
        if (g->inflight.fetch_sub(k) == k && g->draining.load()) {
          std::lock_guard<std::mutex> lk(g->mu);
          g->cv.notify_all();
        }
      }
      i = j;
    }
    for (size_t i = 0; i < fin.size();) {
      Task *t = fin[i].task;
      long status = fin[i].status;
      size_t j = i + 1;
      if (t) {
        while (j < fin.size() && fin[j].task == t) {
          if (!status) status = fin[j].status;
          ++j;
        }
        tasks().put_n(t, (int)(j - i), status);
      } else if (fin[i].status_out) {
        *fin[i].status_out = status;
      }
      i = j;
    }
    bump(prof_cnt[PC_REQ], n);
    bump(prof_cnt[PC_BATCH], 1);
    fin.clear();
    lap(PF_FINISH);
  }

  void bind_numa() {
    if (cfg.numa_bind) bind_to_node(numa_node);
  }

  // staging slots (each max_request bytes): at least staging_slots; small
  // requests get up to 4 x queue_depth slots within the same in-flight byte
  // budget (staging_slots x 1 MiB), so reads keep the queue as deep as the
  // raw ceiling's while earlier slots are still on their way to HBM (round 2
  // sweep: 4 slots capped 64 KiB reads at 0.72 of raw); staging_bytes opts
  // into more
  // ... and, config stage_by_bytes, at least queue_depth slots: requests
  // shorter than max_request (an Arrow column's buffers, 200-500 KiB) are
  // held to the same in-flight BYTES as full ones (stage_budget), not to the
  // same count.  Only with slot_lifo: 8 slots handed out FIFO put twice the
  // staging under 1 MiB reads and cost the bench 12 % (profiles/r6/SUMMARY.md)
  int nslots() const {
    const size_t budget = (size_t)cfg.staging_slots << 20;
    const size_t small = std::min<size_t>((size_t)cfg.queue_depth * 4, budget / cfg.max_request);
    const size_t by_bytes = std::min<size_t>(cfg.staging_bytes / cfg.max_request, 256);
    return (int)std::min<size_t>(256, std::max<size_t>({(size_t)cfg.staging_slots, small, by_bytes,
                                                        cfg.stage_by_bytes ? (size_t)cfg.queue_depth : 0}));
  }
  // the staging bytes requests may hold at once: the slots' bytes up to the
  // default budget (staging_slots x 1 MiB), or the staging_bytes opt-in
  size_t stage_budget() const {
    const size_t budget = std::max<size_t>((size_t)cfg.staging_slots << 20, cfg.staging_bytes);
    return std::min<size_t>(budget, (size_t)nslots() * cfg.max_request);
  }
  void release_slot(int si) {
    stage_inflight -= slots[si].held;
    slots[si].held = 0;
    free_slots.push_back(si);
  }

  bool ensure_slots() {
    if (!slots.empty()) return true;
    const int ns = nslots();
    size_t bytes = (size_t)ns * cfg.max_request;
    staging = (uint8_t *)hip::host_alloc_thp(bytes, cfg.ingest);
    staging_thp = staging != nullptr;
    if (!staging) staging = (uint8_t *)hip::host_alloc(bytes, cfg.ingest);
    if (!staging) {
      STROM_LOG(0, "worker %d: pinned staging allocation failed", idx);
      return false;
    }
    staging_bytes = bytes;
    slots.resize(ns);
    for (int i = 0; i < ns; ++i) {
      slots[i].buf = staging + (size_t)i * cfg.max_request;
      free_slots.push_back(i);          // (held = 0: the budget starts empty)
    }
    // the staging is pinned already (hipHostMalloc); registering it lets
    // READ_FIXED skip the per-I/O get_user_pages of the O_DIRECT path
    fixed = false;
    if (cfg.fixed_bufs && ring.ok()) {
      int rc = ring.register_buffer(staging, bytes);
      fixed = rc == 0;
      if (rc) {
        STROM_LOG(1, "worker %d: io_uring buffer registration refused (%d)", idx, rc);
        g_fixed_refused.fetch_add(1);
        g_fixed_errno.store((uint64_t)-rc);
      } else {
        g_fixed_workers.fetch_add(1);
      }
    }
    return true;
  }

  void free_staging() {
    if (!staging) return;
    if (fixed) {
      ring.unregister_buffers();
      g_fixed_workers.fetch_sub(1);
    }
    fixed = false;
    if (staging_thp) hip::host_free_thp(staging, staging_bytes);
    else hip::host_free(staging);
    staging = nullptr;
  }

  hipStream_t stream_for(int dev) {
    if (dev != cur_dev) {
      (void)hipSetDevice(dev);
      cur_dev = dev;
    }
    if ((int)streams.size() <= dev) streams.resize(dev + 1, nullptr);
    if (!streams[dev]) (void)hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking);
    return streams[dev];
  }

  Ingest *ingest_for(int dev) {
    for (auto &p : ings)
      if (p.first == dev) return p.second;
    Ingest *ing = cfg.ingest ? Ingest::get(dev) : nullptr;
    ings.emplace_back(dev, ing);
    return ing;
  }

  // retire slots whose ingest descriptors are all done
  bool retire_ingest() {
    bool any = false;
    uint64_t now = 0;
    for (size_t i = 0; i < ingesting.size();) {
      const int si = ingesting[i];
      Slot &s = slots[si];
      bool all = true;
      for (uint32_t k = 0; k < s.nseq && all; ++k) all = s.ing->is_done(s.seq_first + k);
      if (!all) {
        ++i;
        continue;
      }
      if (!now) now = mono_ns();
      const uint64_t dt = now - s.t_copy_ns;
      hist_copy(dt);
      copy_clk += dt;
      if (s.nret) s.ing->retired(s.nret);
      ingesting[i] = ingesting.back();
      ingesting.pop_back();
      release_slot(si);
      complete(s.req, 0);
      any = true;
    }
    return any;
  }

  // storage read finished for ctx c with `got` bytes or -errno
  void on_read_done(Ctx &c, long got) {
    IoReq &r = c.req;
    hist_io(now_ns - c.t0);
    long status = finalize_read(r, c.dst, c.len, got);
    if (c.slot < 0) {
      complete(r, status);
      return;
    }
    Slot &s = slots[c.slot];
    if (status != 0) {
      release_slot(c.slot);
      complete(r, status);
      return;
    }
    s.req = r;
    s.t_copy_ns = now_ns;
    if (r.gmap && r.len >= cfg.ingest_min && ingest_for(r.device)) {
      ing_staged.push_back(c.slot);  // posted per batch (post_ingest)
      return;
    }
    to_hbm(c.slot);
  }

  // the slot's bytes reach HBM without the ingest grid: CPU stores through
  // the BAR (small requests) or a staged SDMA copy (flush_staged)
  void to_hbm(int si) {
    Slot &s = slots[si];
    const IoReq &r = s.req;
    // worker requests take the BAR only up to 64 KiB: past that the workers'
    // CPU stores fall behind SDMA (256 KiB: 14.2 vs 17.8 GiB/s, 512 KiB: 23.7
    // vs 26.5, profiles/r1j/sweep_barmax_*); synchronous reads keep bar_max
    constexpr uint32_t kWorkerBarMax = 64u << 10;
    if (r.len <= std::min(cfg.bar_max, kWorkerBarMax) && r.gmap) {
      lap(PF_REAP);
      const bool ok = r.gmap->bar_write(r.gpu_dst, s.buf, r.len, false);
      lap(PF_BAR);
      if (ok) {
        // small request: CPU stores through the large BAR beat an SDMA round
        // trip; the sfence + HDP flush is paid once per batch (flush_done)
        const uint8_t *last = r.gmap->bar + (r.gpu_dst - r.gmap->bar_va) + ((r.len - 1) & ~3u);
        if (!bar_dirty.empty() && bar_dirty.back().first == r.gmap) bar_dirty.back().second = last;
        else bar_dirty.emplace_back(r.gmap, last);
        ++nbar;
        ++ndesc;
        release_slot(si);
        complete(r, 0);
        return;
      }
    }
    staged.push_back(si);
  }

  // Post the ingest descriptors of the reads that finished in this batch:
  // adjacent staging slots whose destinations are adjacent in HBM go out as
  // one range (split into ingest_piece descriptors), and the whole batch
  // takes the grid's lock once.
  void post_ingest() {
    if (ing_staged.empty()) return;
    lap(PF_REAP);
    std::sort(ing_staged.begin(), ing_staged.end());
    size_t i = 0;
    while (i < ing_staged.size()) {
      // one device per post_runs call
      const int dev = slots[ing_staged[i]].req.device;
      Ingest *ing = ingest_for(dev);
      runs.clear();
      span.clear();
      size_t k = i;
      while (k < ing_staged.size() && slots[ing_staged[k]].req.device == dev) {
        size_t j = k + 1;
        uint64_t bytes = slots[ing_staged[k]].req.len;
        while (cfg.coalesce && j < ing_staged.size()) {
          const Slot &p = slots[ing_staged[j - 1]], &q2 = slots[ing_staged[j]];
          if (ing_staged[j] != ing_staged[j - 1] + 1 || p.req.len != cfg.max_request ||
              q2.req.device != dev || q2.req.gpu_dst != p.req.gpu_dst + p.req.len ||
              bytes + q2.req.len > (64u << 20))
            break;
          bytes += q2.req.len;
          ++j;
        }
        const Slot &h = slots[ing_staged[k]];
        runs.push_back(Ingest::Run{h.buf, h.req.gpu_dst, (uint32_t)bytes, false, 0, 0});
        span.emplace_back(k, j);
        k = j;
      }
      ing->post_runs(runs.data(), runs.size(), cfg.ingest_piece);
      for (size_t r = 0; r < runs.size(); ++r) {
        const Ingest::Run &run = runs[r];
        for (size_t m = span[r].first; m < span[r].second; ++m) {
          const int si = ing_staged[m];
          if (!run.ok) {
            to_hbm(si);
            continue;
          }
          Slot &s = slots[si];
          s.ing = ing;
          s.seq_first = run.first;
          s.nseq = run.n;
          s.nret = m == span[r].first ? run.n : 0;
          ingesting.push_back(si);
        }
        if (run.ok) {
          ndesc += run.n;
          bump(prof_cnt[PC_DESC], run.n);
        }
      }
      i = k;
    }
    ing_staged.clear();
    lap(PF_POST);
  }

  // Issue the HBM copies of the reads that finished in this batch.  Reads of
  // adjacent staging slots whose destinations are adjacent in HBM go out as
  // one SDMA copy with one event: a host-side hipMemcpyAsync costs ~11 us
  // and a 128 KiB copy ~8 us (profiles/r1p), so per-request copies capped
  // 64-256 KiB streams at about 60% of the storage rate.
  void flush_staged() {
    if (staged.empty()) return;
    std::sort(staged.begin(), staged.end());
    size_t i = 0;
    while (i < staged.size()) {
      size_t j = i + 1;
      uint64_t bytes = slots[staged[i]].req.len;
      while (cfg.coalesce && j < staged.size()) {
        const Slot &p = slots[staged[j - 1]], &q = slots[staged[j]];
        if (staged[j] != staged[j - 1] + 1 || p.req.len != cfg.max_request ||
            q.req.device != p.req.device || q.req.gpu_dst != p.req.gpu_dst + p.req.len)
          break;
        bytes += q.req.len;
        ++j;
      }
      Slot &head = slots[staged[i]];
      const int last = staged[j - 1];
      Slot &tail = slots[last];
      const int dev = head.req.device;
      hipStream_t st = stream_for(dev);
      if (!tail.ev || tail.ev_dev != dev) {
        if (tail.ev) (void)hipEventDestroy(tail.ev);
        (void)hipEventCreateWithFlags(&tail.ev, hipEventDisableTiming);
        tail.ev_dev = dev;
      }
      hipError_t e = hipMemcpyAsync((void *)head.req.gpu_dst, head.buf, bytes,
                                    hipMemcpyHostToDevice, st);
      if (e == hipSuccess) e = hipEventRecord(tail.ev, st);
      for (size_t k = i; k < j; ++k) {
        const int si = staged[k];
        if (e != hipSuccess) {
          release_slot(si);
          complete(slots[si].req, -EIO);
          continue;
        }
        slots[si].ev_slot = last;
        copying.push_back(si);
      }
      if (e != hipSuccess) STROM_LOG(0, "hipMemcpyAsync failed: %s", hipGetErrorString(e));
      else ++ndesc;
      i = j;
    }
    staged.clear();
  }

  // retire finished HBM copies; block on the oldest when `block`
  void retire(bool block) {
    while (!copying.empty()) {
      Slot &s = slots[copying.front()];
      hipEvent_t ev = slots[s.ev_slot].ev;
      hipError_t e = block ? hipEventSynchronize(ev) : hipEventQuery(ev);
      if (e == hipErrorNotReady) return;
      uint64_t dt = mono_ns() - s.t_copy_ns;
      hist_copy(dt);
      copy_clk += dt;
      int si = copying.front();
      copying.pop_front();
      release_slot(si);
      complete(s.req, e == hipSuccess ? 0 : -EIO);
      block = false;
    }
  }

  // start one request; false when it has to wait for a staging slot
  bool start(IoReq &r, bool use_ring) {
    int slot = -1;
    uint8_t *dst = r.host_dst;
    if (!dst) {
      if (!ensure_slots()) {
        complete(r, -ENOMEM);
        return true;
      }
      if (free_slots.empty()) return false;
      // the byte budget (a request alone may always start)
      if (cfg.stage_by_bytes && stage_inflight && stage_inflight + r.len > stage_budget()) return false;
      if (cfg.coalesce && !cfg.slot_lifo) {
        slot = free_slots.front();
        free_slots.pop_front();
      } else {
        slot = free_slots.back();
        free_slots.pop_back();
      }
      dst = slots[slot].buf;
      slots[slot].held = r.len;
      stage_inflight += r.len;
    }
    uint32_t len = r.len;
    int frc = faults().on_request(&len);
    Ctx c;
    c.req = r;
    c.slot = slot;
    c.dst = dst;
    c.len = len;
    c.t0 = now_ns;
    if (frc && cfg.backend != BackendKind::kFake) {
      on_read_done(c, frc);
      post_ingest();
      flush_staged();
      return true;
    }
    if (cfg.backend == BackendKind::kFake) {
      c.got = frc ? frc : pread_full(r.fd, dst, len, r.off);
      c.seq = fake_seq++;
      fake_cq.push_back(c);
      ++reads_inflight;
      return true;
    }
    if (use_ring) {
      int ci;
      if (free_ctx.empty()) {
        ci = (int)ctx.size();
        ctx.push_back(c);
      } else {
        ci = free_ctx.back();
        free_ctx.pop_back();
        ctx[ci] = c;
      }
      io_uring_sqe *sqe = ring.next_sqe();
      if (!sqe) {  // ring full: flush and retry synchronously
        ring.enter(0);
        sqe = ring.next_sqe();
      }
      if (fixed && slot >= 0) {
        sqe->opcode = IORING_OP_READ_FIXED;
        sqe->buf_index = 0;
      } else {
        sqe->opcode = IORING_OP_READ;
      }
      sqe->fd = read_fd(r);
      sqe->addr = (uint64_t)dst;
      sqe->len = len;
      sqe->off = r.off;
      sqe->user_data = (uint64_t)ci;
      ++reads_inflight;
      return true;
    }
    long got = pread_full(read_fd(r), dst, len, r.off);
    now_ns = mono_ns();
    on_read_done(c, got);
    post_ingest();
    flush_staged();
    return true;
  }
  int read_fd(const IoReq &r) const {
    return cfg.backend == BackendKind::kCache && r.fd_buffered >= 0 ? r.fd_buffered : r.fd;
  }

  void reap() {
    io_uring_cqe cqe;
    bool first = true;
    while (ring.peek(&cqe)) {
      if (first) {
        now_ns = mono_ns();
        first = false;
      }
      int ci = (int)cqe.user_data;
      Ctx c = ctx[ci];
      free_ctx.push_back(ci);
      --reads_inflight;
      long got = cqe.res;
      if (got >= 0 && (uint32_t)got < c.len) {
        // partial completion: finish the remainder synchronously
        long more = pread_full(read_fd(c.req), c.dst + got, c.len - (uint32_t)got, c.req.off + got);
        got = more < 0 ? more : got + more;
      }
      on_read_done(c, got);
    }
    post_ingest();
    flush_staged();
    lap(PF_REAP);
  }

  void run() {
    bind_numa();
    const bool fake = cfg.backend == BackendKind::kFake;
    bool use_ring = cfg.backend == BackendKind::kUring || cfg.backend == BackendKind::kCache;
    // reads in flight: queue_depth, or the staging_bytes opt-in's slot count
    const int qd_cfg = (int)std::max<size_t>(
        {(size_t)cfg.queue_depth, (size_t)cfg.staging_slots,
         std::min<size_t>(cfg.staging_bytes / cfg.max_request, 256)});
    if (use_ring && ring.init((unsigned)std::max(8, qd_cfg * 2)) != 0) use_ring = false;
    int qd = use_ring || fake ? qd_cfg : 1;
    fake_rng = faults().fake_seed.load() * 2654435761u + (uint64_t)idx * 0x9E3779B97F4A7C15ull + 1;
    const uint64_t spin_ns = (uint64_t)cfg.spin_us * 1000;
    prof_on = cfg.io_prof;
    prof_t = tsc_now();
    std::vector<IoReq> local;
    size_t lpos = 0;                // next request of `local` to start
    for (;;) {
      flush_done();
      if (lpos == local.size()) {
        const bool quiet = reads_inflight == 0 && copying.empty() && ingesting.empty();
        if (spin_ns && quiet && !pending.load(std::memory_order_acquire)) {
          // idle: poll briefly before sleeping, so back-to-back work skips
          // the futex wake-up (bounded, so stop is still seen promptly)
          const uint64_t end = mono_ns() + spin_ns;
          while (!pending.load(std::memory_order_acquire) && mono_ns() < end)
            for (int i = 0; i < 32; ++i) _mm_pause();
        }
        if (quiet && !pending.load(std::memory_order_acquire)) {
          // about to sleep: let the ingest grids stop if nobody has work
          // in them (a device-wide synchronize must not wait on them)
          for (auto &p : ings)
            if (p.second) p.second->idle();
        }
        lap(PF_IDLE);
        std::unique_lock<std::mutex> g(mu);
        if (q.empty() && quiet) {
          if (stop) break;
          sleeping = true;
          bump(prof_cnt[PC_SLEEP], 1);
          cv.wait(g, [&] { return stop || !q.empty(); });
          sleeping = false;
          lap(PF_IDLE);
        }
        local.clear();
        lpos = 0;
        local.swap(q);
        pending.store(0, std::memory_order_relaxed);
        g.unlock();
        lap(PF_TAKE);
      }
      // issue as much as the queue depth and staging allow
      bool blocked = false;
      now_ns = mono_ns();
      while (lpos < local.size() && reads_inflight < qd) {
        if (!start(local[lpos], use_ring)) {
          blocked = true;
          break;
        }
        ++lpos;
      }
      lap(PF_START);
      if (use_ring && ring.pending()) {
        ring.enter(0);
        bump(prof_cnt[PC_ENTER], 1);
        lap(PF_SUBMIT);
      }
      const bool drained = lpos == local.size();
      if (fake && (drained || blocked || reads_inflight >= qd)) reap_fake();
      retire(false);
      retire_ingest();
      lap(PF_RETIRE);
      if (use_ring) reap();
      flush_done();
      if (lpos < local.size() && !blocked && reads_inflight < qd) continue;
      // nothing more can start: wait for a read, a copy, or new work
      const bool hbm_busy = !copying.empty() || !ingesting.empty();
      if (reads_inflight > 0 && !hbm_busy) {
        if (fake) {
          reap_fake();
        } else {
          ring.enter(1);
          bump(prof_cnt[PC_ENTER], 1);
          lap(PF_WAIT);
          reap();
        }
      } else if (reads_inflight == 0 && hbm_busy) {
        if (lpos == local.size()) {
          std::lock_guard<std::mutex> g(mu);
          if (!q.empty()) continue;
        }
        if (!ingesting.empty()) {
          // the grid's completions land in host memory within microseconds:
          // poll them (and any SDMA events) instead of sleeping
          const uint64_t end = mono_ns() + 200000;
          while (!retire_ingest() && mono_ns() < end) {
            for (int i = 0; i < 16; ++i) _mm_pause();
            if (pending.load(std::memory_order_acquire)) break;
          }
          retire(false);
          lap(PF_WAIT);
        } else {
          retire(true);
          lap(PF_WAIT);
        }
      } else if (reads_inflight > 0) {
        if (!retire_ingest()) sched_yield();  // both pipes busy
        lap(PF_WAIT);
      }
    }
    for (auto &s : slots)
      if (s.ev) (void)hipEventDestroy(s.ev);
    free_staging();
    for (auto st : streams)
      if (st) (void)hipStreamDestroy(st);
  }
};

int IoEngine::prof(uint64_t *out, int nout, bool reset) {
  const int need = 2 + kProfPhases + kProfCounts + 4;
  if (nout < need) return -EINVAL;
  memset(out, 0, sizeof(uint64_t) * need);
  out[0] = workers_.size();
  out[1] = tsc_khz();
  std::lock_guard<std::mutex> lk(prof_mu_);
  for (auto &w : workers_) {
    for (int k = 0; k < kProfPhases; ++k) {
      const uint64_t v = w->prof_cyc[k].load(std::memory_order_relaxed);
      out[2 + k] += v - w->prof_base_cyc[k];
      if (reset) w->prof_base_cyc[k] = v;
    }
    for (int k = 0; k < kProfCounts; ++k) {
      const uint64_t v = w->prof_cnt[k].load(std::memory_order_relaxed);
      out[2 + kProfPhases + k] += v - w->prof_base_cnt[k];
      if (reset) w->prof_base_cnt[k] = v;
    }
  }
  CallerProf &cp = caller_prof();
  std::atomic<uint64_t> *c[4] = {&cp.calls, &cp.plan, &cp.build, &cp.submit};
  for (int k = 0; k < 4; ++k) out[2 + kProfPhases + kProfCounts + k] = reset ? c[k]->exchange(0) : c[k]->load();
  return need;
}

IoEngine::IoEngine(const Config &cfg) {
  int node = -1;
  if (cfg.numa_bind && hip::available()) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    node = hip::numa_node_of_device(dev);
  }
  for (int i = 0; i < cfg.workers; ++i) {
    auto w = std::make_unique<Worker>();
    w->idx = i;
    w->cfg = cfg;
    w->numa_node = node;
    Worker *wp = w.get();
    w->th = std::thread([wp] { wp->run(); });
    workers_.push_back(std::move(w));
  }
}

IoEngine::~IoEngine() {
  for (auto &w : workers_) {
    std::lock_guard<std::mutex> g(w->mu);
    w->stop = true;
    w->cv.notify_all();
  }
  for (auto &w : workers_) w->th.join();
}

// Per-thread resources of the inline path.  Never freed: the HIP runtime
// may already be gone when a thread-local destructor would run at exit.
struct InlineCtx {
  uint8_t *buf = nullptr;
  size_t cap = 0;
  uint8_t *plain = nullptr;      // config inline_plain: unpinned bounce for BAR stores
  size_t plain_cap = 0;
  int dev = -1;
  hipStream_t st = nullptr;
  hipEvent_t ev = nullptr;
};
static thread_local InlineCtx tl_inline;

void IoEngine::run_inline(IoReq &r) {
  InlineCtx &c = tl_inline;
  uint32_t len = r.len;
  int frc = faults().on_request(&len);
  uint64_t t0 = mono_ns();
  if (r.host_dst) {
    long got = frc ? frc : pread_full(r.fd, r.host_dst, len, r.off);
    stats().io_ns.add(mono_ns() - t0);
    phase_mark(3);
    finish_request(r, finalize_read(r, r.host_dst, len, got));
    phase_mark(6);
    return;
  }
  const bool ing_ok = config().ingest;
  if (c.cap < r.len) {
    size_t cap = std::max<size_t>(r.len, 64u << 10);
    uint8_t *b = (uint8_t *)hip::host_alloc_thp(cap, ing_ok);
    if (!b) b = (uint8_t *)hip::host_alloc(cap, ing_ok);
    if (!b) {
      finish_request(r, -ENOMEM);
      return;
    }
    c.buf = b;  // the old buffer (if any) is leaked on purpose: it is small
    c.cap = cap;
  }
  const int rfd = config().backend == BackendKind::kCache && r.fd_buffered >= 0 ? r.fd_buffered : r.fd;
  // a read the CPU will store through the BAR needs no pinned bounce
  const bool to_bar = r.len <= config().bar_max && r.gmap && r.gmap->bar;
  uint8_t *rb = c.buf;
  if (to_bar && config().inline_plain) {
    if (c.plain_cap < r.len) {
      free(c.plain);
      c.plain_cap = 0;
      const size_t cap = std::max<size_t>(r.len, 64u << 10);
      c.plain = posix_memalign((void **)&c.plain, 4096, cap) == 0 ? c.plain : nullptr;
      if (c.plain) c.plain_cap = cap;
    }
    if (c.plain) rb = c.plain;
  }
  long got = frc ? frc : pread_full(rfd, rb, len, r.off);
  uint64_t t1 = mono_ns();
  if (tl_phase) tl_phase[3] = t1;
  stats().io_ns.add(t1 - t0);
  long status = finalize_read(r, rb, len, got);
  Ingest *ing = nullptr;
  uint64_t first = 0;
  uint32_t nseq = 0;
  const bool bar_ok = status == 0 && to_bar && r.gmap->bar_write(r.gpu_dst, rb, r.len);
  // the other paths below read the pinned bounce
  if (!bar_ok && status == 0 && rb != c.buf) memcpy(c.buf, rb, r.len);
  if (bar_ok) {
    stats().copy_ns.add(mono_ns() - t1);
    stats().nr_debug[0].fetch_add(1, std::memory_order_relaxed);
  } else if (status == 0 && ing_ok && r.gmap && (ing = Ingest::get(r.device)) &&
             ing->post_many(c.buf, r.gpu_dst, r.len, config().ingest_piece, &first, &nseq)) {
    // past the BAR cut: the ingest grid pulls the bytes (no HIP call here)
    for (uint32_t k = 0; k < nseq; ++k)
      while (!ing->is_done(first + k)) _mm_pause();
    ing->retired(nseq);
    // no worker may go idle after this (the task never reached one): stop
    // the grid here if nothing else is outstanding, or a device-wide
    // synchronize would wait on it forever
    ing->idle();
    phase_mark(4);
    stats().copy_ns.add(mono_ns() - t1);
    stats().nr_debug[0].fetch_add(nseq, std::memory_order_relaxed);
  } else if (status == 0) {
    if (c.dev != r.device) {
      (void)hipSetDevice(r.device);
      (void)hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking);
      (void)hipEventCreateWithFlags(&c.ev, hipEventDisableTiming);
      c.dev = r.device;
    }
    hipError_t e = hipMemcpyAsync((void *)r.gpu_dst, c.buf, r.len, hipMemcpyHostToDevice, c.st);
    if (e == hipSuccess) e = hipStreamSynchronize(c.st);
    phase_mark(4);
    if (e != hipSuccess) status = -EIO;
    stats().copy_ns.add(mono_ns() - t1);
    stats().nr_debug[0].fetch_add(1, std::memory_order_relaxed);
  }
  finish_request(r, status);
  phase_mark(6);
}

void IoEngine::submit(std::vector<IoReq> &reqs) {
  const size_t n = workers_.size();
  if (reqs.empty()) return;
  uint32_t start = rr_.fetch_add((uint32_t)reqs.size());
  // contiguous runs per worker keep each ring's reads sequential
  size_t per = (reqs.size() + n - 1) / n;
  for (size_t k = 0; k < n; ++k) {
    size_t lo = k * per, hi = std::min(reqs.size(), lo + per);
    if (lo >= hi) break;
    Worker &w = *workers_[(start + k) % n];
    bool wake;
    {
      std::lock_guard<std::mutex> g(w.mu);
      w.q.insert(w.q.end(), reqs.begin() + lo, reqs.begin() + hi);
      w.pending.store(1, std::memory_order_release);
      wake = w.sleeping;
    }
    if (wake) w.cv.notify_one();
  }
}

}  // namespace strom

// per-worker phase attribution (IoEngine::prof); -ENODEV before the engine
// exists, else the number of u64 written
extern "C" int strom_io_prof(uint64_t *out, int nout, int reset) {
  return strom::engine().io().prof(out, nout, reset != 0);
}

// workers whose staging is registered (READ_FIXED), refusals, last errno
extern "C" int strom_io_info(uint64_t *out) {
  out[0] = strom::g_fixed_workers.load();
  out[1] = strom::g_fixed_refused.load();
  out[2] = strom::g_fixed_errno.load();
  return 0;
}

// ----------------------------------------------------- raw storage ceiling
namespace {
// One ring per thread kept `qd` deep with O_DIRECT (or buffered, mode bit 1)
// reads into host memory (2 MiB pages registered with the ring for
// READ_FIXED with mode bit 2); next(tid, k, &off, &len) names thread tid's
// k-th read (false: the thread is done).  Returns the first error; *bytes
// the bytes read, *sec the wall time.
int raw_reads(int fd, int mode, uint32_t threads, uint32_t qd, uint64_t slot,
              const std::function<bool(uint32_t, uint32_t, uint64_t *, uint32_t *)> &next,
              uint64_t *bytes_out, double *sec_out) {
  using namespace strom;
  const bool fixed = (mode & 4) != 0;
  if (slot * qd > (4ull << 30)) return -E2BIG;   // per ring: qd reads of the largest request
  // rings on the CPUs the engine's workers use (config numa_bind: the
  // current GPU's NUMA node), so the comparison is like for like
  int node = -1;
  if (config().numa_bind && hip::available()) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    node = hip::numa_node_of_device(dev);
  }
  char path[64];
  snprintf(path, sizeof path, "/proc/self/fd/%d", fd);
  int d = open(path, O_RDONLY | ((mode & 2) ? 0 : O_DIRECT) | O_CLOEXEC);
  if (d < 0) return -errno;
  std::atomic<int> err{0};
  std::atomic<uint64_t> total{0};
  auto body = [&](uint32_t tid) {
    bind_to_node(node);
    Uring ring;
    int rc = ring.init(qd);
    void *buf = nullptr;
    const size_t bytes = (size_t)slot * qd, huge = (bytes + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    bool mapped = false, reg = false;
    if (rc == 0 && fixed) {
      // 2 MiB aligned inside a larger anonymous map, huge pages advised
      void *m = mmap(nullptr, huge + (2u << 20), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (m != MAP_FAILED) {
        uint8_t *a = (uint8_t *)(((uintptr_t)m + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1));
        if (a > (uint8_t *)m) munmap(m, (size_t)(a - (uint8_t *)m));
        const size_t tail = (size_t)((uint8_t *)m + huge + (2u << 20) - (a + huge));
        if (tail) munmap(a + huge, tail);
        (void)madvise(a, huge, MADV_HUGEPAGE);
        memset(a, 0, huge);
        buf = a;
        mapped = true;
        reg = ring.register_buffer(buf, bytes) == 0;
      }
    }
    if (rc == 0 && !buf && posix_memalign(&buf, 4096, bytes) != 0) rc = -ENOMEM;
    uint32_t inflight = 0, k = 0;
    uint64_t got_bytes = 0;
    bool more = true;
    std::vector<uint32_t> freeslot;
    for (uint32_t s = 0; s < qd; ++s) freeslot.push_back(s);
    bool init_ok = rc == 0;
    while (init_ok) {
      while (rc == 0 && more && !freeslot.empty()) {
        uint64_t off = 0;
        uint32_t len = 0;
        if (!(more = next(tid, k, &off, &len))) break;
        ++k;
        uint32_t s = freeslot.back();
        freeslot.pop_back();
        io_uring_sqe *q = ring.next_sqe();
        q->opcode = reg ? IORING_OP_READ_FIXED : IORING_OP_READ;
        q->buf_index = 0;
        q->fd = d;
        q->addr = (uint64_t)buf + (uint64_t)s * slot;
        q->len = len;
        q->off = off;
        q->user_data = s;
        ++inflight;
      }
      if (inflight == 0) break;
      // submit, then look at the completion queue for a while before
      // sleeping in the kernel — as the engine's workers reap (spin_us): a
      // sleep + wake-up per completion batch made this "ceiling" slower
      // than the engine at 4-32 KiB on RAM-class storage
      int r = ring.pending() ? ring.enter(0) : 0;
      if (r < 0 && r != -EINTR && rc == 0) rc = r;
      io_uring_cqe c;
      uint32_t got = 0;
      auto reap = [&] {
        while (ring.peek(&c)) {
          if (c.res < 0 && rc == 0) rc = c.res;
          if (c.res > 0) got_bytes += (uint64_t)c.res;
          freeslot.push_back((uint32_t)c.user_data);
          --inflight;
          ++got;
        }
      };
      for (uint64_t t0 = mono_ns(); !got && mono_ns() - t0 < 20000;) {
        reap();
        if (!got) _mm_pause();
      }
      if (!got) {
        r = ring.enter(1);  // in-flight reads drain even after an error
        if (r < 0 && r != -EINTR && rc == 0) rc = r;
        reap();
      }
    }
    if (rc) err.store(rc);
    total.fetch_add(got_bytes);
    if (reg) ring.unregister_buffers();
    if (mapped) munmap(buf, huge);
    else free(buf);
  };
  const uint64_t t0 = mono_ns();
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < threads; ++t) th.emplace_back(body, t);
  for (auto &t : th) t.join();
  *sec_out = (mono_ns() - t0) * 1e-9;
  *bytes_out = total.load();
  close(d);
  return err.load();
}
}  // namespace

// The device's own limit for a block size, with no engine in the way:
// `threads` threads, each with its own io_uring kept `qd` deep with O_DIRECT
// reads of `block` bytes at random aligned offsets into host memory (or,
// with `sequential`, each ring its own run of the file in order: the order
// the engine's workers stream a window in).  The sweep prints it next to the engine's
// SSD→HBM numbers.  `mode` bit 0: sequential; bit 1: buffered reads (the
// page-cache ceiling the engine-only sweep compares against); bit 2: reads
// into 2 MiB-page memory registered with the ring (READ_FIXED), as the
// engine's pinned staging does.
extern "C" int strom_raw_read_rate(int fd, uint64_t block, uint32_t nreq, uint32_t threads,
                                   uint32_t qd, int mode, double *iops, double *gibps) {
  const bool sequential = mode & 1;
  if (block == 0 || (block & 4095) || block > (1ull << 30) || nreq == 0 || threads == 0 || qd == 0 ||
      qd > 256)
    return -EINVAL;
  struct stat st;
  if (fstat(fd, &st) != 0) return -errno;
  const uint64_t nblk = (uint64_t)st.st_size / block;
  if (nblk == 0) return -ERANGE;
  // Every ring owns its share of the requests and, sequential, a disjoint
  // run of the file read in order — as the engine's workers read theirs.
  // No cursor is shared between rings: a common atomic cursor costs a
  // contended cache line per request and interleaves the rings' reads,
  // which made this "ceiling" slower than the engine at 4-16 KiB
  // (VERDICT r4 weak #5).
  const uint64_t run = std::max<uint64_t>(1, nblk / threads);
  std::vector<uint64_t> x(threads);
  for (uint32_t t = 0; t < threads; ++t) x[t] = 0x9e3779b97f4a7c15ull * (t + 1);
  auto next = [&](uint32_t tid, uint32_t k, uint64_t *off, uint32_t *len) {
    const uint32_t mine = nreq / threads + (tid < nreq % threads ? 1 : 0);
    if (k >= mine) return false;
    uint64_t &r = x[tid];
    r ^= r << 13, r ^= r >> 7, r ^= r << 17;
    *off = (sequential ? ((uint64_t)tid * run + k % run) % nblk : r % nblk) * block;
    *len = (uint32_t)block;
    return true;
  };
  uint64_t bytes = 0;
  double sec = 0;
  const int rc = raw_reads(fd, mode, threads, qd, block, next, &bytes, &sec);
  if (rc) return rc;
  if (iops) *iops = nreq / sec;
  if (gibps) *gibps = (double)nreq * block / sec / (1 << 30);
  return 0;
}

// The same rings reading exactly the requests (off[i], len[i]) — 4 KiB
// aligned, in order, thread t taking the t-th contiguous share of the list:
// the storage's own rate for an access pattern an engine call produced
// (the Arrow read probe's comparator for a column's extent requests).
extern "C" int strom_raw_read_list(int fd, const uint64_t *off, const uint32_t *len, uint32_t n,
                                   uint32_t threads, uint32_t qd, int mode, double *iops,
                                   double *gibps) {
  if (!off || !len || n == 0 || threads == 0 || qd == 0 || qd > 256) return -EINVAL;
  uint32_t slot = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if ((off[i] & 4095) || len[i] == 0 || (len[i] & 4095) || len[i] > (64u << 20)) return -EINVAL;
    slot = std::max(slot, len[i]);
  }
  threads = std::min(threads, n);
  auto next = [&](uint32_t tid, uint32_t k, uint64_t *o, uint32_t *l) {
    const uint64_t lo = (uint64_t)n * tid / threads, hi = (uint64_t)n * (tid + 1) / threads;
    if (lo + k >= hi) return false;
    *o = off[lo + k];
    *l = len[lo + k];
    return true;
  };
  uint64_t bytes = 0;                           // a read at the end may come back short
  double sec = 0;
  const int rc = raw_reads(fd, mode & ~1, threads, qd, slot, next, &bytes, &sec);
  if (rc) return rc;
  if (iops) *iops = n / sec;
  if (gibps) *gibps = (double)bytes / sec / (1 << 30);
  return 0;
}
