// core.cc — configuration, statistics, task table, fault injection.
//
// Task table semantics follow the reference's strom_dma_task lifecycle
// (kmod/nvme_strom.c:575-731): refcnt = 1 submitter + 1 per request, the
// first non-zero status wins, a failed task survives its last put on a
// per-slot failed list until WAIT consumes it or its session closes
// (strom_proc_release, :2064-2091).  Two deliberate fixes: WAIT on an id
// that was never issued returns -ENOENT (reference returns success,
// :1189-1190), and WAIT can carry a deadline.
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>
#include <x86intrin.h>

#include <new>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "engine.h"

namespace strom {

// ------------------------------------------------------------------ config
static bool parse_bool(const std::string &v) {
  return v == "1" || v == "true" || v == "yes" || v == "on";
}

Config Config::from_env() {
  Config c;
  static const char *keys[] = {"backend", "workers", "queue_depth", "max_request",
                               "staging_slots", "staging_bytes", "spin_us", "inline_max",
                               "bar_map", "bar_max", "bar_nt", "inline_plain", "coalesce", "trace",
                               "ingest", "ingest_grid", "ingest_piece", "ingest_min", "ingest_prio", "hdp_sync",
                               "fixed_bufs", "io_prof", "fd_kcmp", "stage_by_bytes", "slot_lifo",
                               "strict", "direct_io",
                               "pgcache_probe", "gpu_emulation", "numa_bind", "check_freed",
                               "stat_info", "verbose"};
  for (const char *k : keys) {
    std::string env = "STROM_";
    for (const char *p = k; *p; ++p) env += (char)toupper(*p);
    if (const char *v = getenv(env.c_str())) c.set(k, v);
  }
  // Ranks sharing one backing device split the pool: the parallel layer
  // counts them per device (nvme_strom_amd/parallel/placement.py) and sets
  // `workers`; one SSD per GPU keeps the full pool.
  return c;
}

int Config::set(const std::string &k, const std::string &v) {
  char *end = nullptr;
  long n = strtol(v.c_str(), &end, 0);
  bool num_ok = end && *end == '\0' && !v.empty();
  if (k == "backend") {
    if (v == "psync") backend = BackendKind::kPsync;
    else if (v == "uring") backend = BackendKind::kUring;
    else if (v == "fake") backend = BackendKind::kFake;
    else if (v == "cache") backend = BackendKind::kCache;
    else return -EINVAL;
    return 0;
  }
  if (k == "strict") { strict = parse_bool(v); return 0; }
  if (k == "direct_io") { direct_io = parse_bool(v); return 0; }
  if (k == "pgcache_probe") { pgcache_probe = parse_bool(v); return 0; }
  if (k == "gpu_emulation") { gpu_emulation = parse_bool(v); return 0; }
  if (k == "numa_bind") { numa_bind = parse_bool(v); return 0; }
  if (k == "check_freed") { check_freed = parse_bool(v); return 0; }
  if (!num_ok) return -EINVAL;
  if (k == "workers") { if (n < 1 || n > 256) return -EINVAL; workers = (int)n; return 0; }
  if (k == "queue_depth") { if (n < 1 || n > 4096) return -EINVAL; queue_depth = (int)n; return 0; }
  if (k == "max_request") {
    if (n < 4096 || n > (64l << 20) || (n & 4095)) return -EINVAL;
    max_request = (uint32_t)n;
    return 0;
  }
  if (k == "staging_slots") { if (n < 1 || n > 1024) return -EINVAL; staging_slots = (int)n; return 0; }
  if (k == "staging_bytes") {
    if (n < 0 || n > (1l << 30)) return -EINVAL;
    staging_bytes = (uint32_t)n;
    return 0;
  }
  if (k == "spin_us") { if (n < 0 || n > 10000) return -EINVAL; spin_us = (uint32_t)n; return 0; }
  if (k == "bar_map") { bar_map = parse_bool(v); return 0; }
  if (k == "coalesce") { coalesce = parse_bool(v); return 0; }
  if (k == "ingest") { ingest = parse_bool(v); return 0; }
  if (k == "hdp_sync") {
    if (!num_ok) { hdp_sync = parse_bool(v) ? 1 : 0; return 0; }
    if (n < 0 || n > 2) return -EINVAL;
    hdp_sync = (int)n;
    return 0;
  }
  if (k == "fixed_bufs") { fixed_bufs = parse_bool(v); return 0; }
  if (k == "io_prof") { io_prof = parse_bool(v); return 0; }
  if (k == "fd_kcmp") { fd_kcmp = parse_bool(v); return 0; }
  if (k == "stage_by_bytes") { stage_by_bytes = parse_bool(v); return 0; }
  if (k == "slot_lifo") { slot_lifo = parse_bool(v); return 0; }
  if (k == "ingest_min") {
    if (n < 0 || n > (64l << 20)) return -EINVAL;
    ingest_min = (uint32_t)n;
    return 0;
  }
  if (k == "ingest_prio") { if (n < 0 || n > 1) return -EINVAL; ingest_prio = (int)n; return 0; }
  if (k == "ingest_grid") { if (n < 1 || n > 256) return -EINVAL; ingest_grid = (int)n; return 0; }
  if (k == "ingest_piece") {
    if (n < 4096 || n > (16l << 20) || (n & 4095)) return -EINVAL;
    ingest_piece = (uint32_t)n;
    return 0;
  }
  if (k == "trace") { trace = parse_bool(v); return 0; }
  if (k == "bar_max") {
    if (n < 0 || n > (64l << 20)) return -EINVAL;
    bar_max = (uint32_t)n;
    return 0;
  }
  if (k == "inline_plain") { inline_plain = parse_bool(v); return 0; }
  if (k == "bar_nt") {
    if (!num_ok) { bar_nt = parse_bool(v) ? 1 : 0; return 0; }
    if (n < 0 || n > 1) return -EINVAL;
    bar_nt = (int)n;
    return 0;
  }
  if (k == "inline_max") {
    if (n < 0 || n > (16l << 20) || (n & 4095)) return -EINVAL;
    inline_max = (uint32_t)n;
    return 0;
  }
  if (k == "stat_info") { stat_info = (int)n; return 0; }
  if (k == "verbose") { verbose = (int)n; return 0; }
  return -ENOENT;
}

int Config::get(const std::string &k, std::string *out) const {
  char buf[64];
  if (k == "backend") {
    *out = backend == BackendKind::kPsync   ? "psync"
           : backend == BackendKind::kUring ? "uring"
           : backend == BackendKind::kCache ? "cache"
                                            : "fake";
    return 0;
  }
  long v;
  if (k == "workers") v = workers;
  else if (k == "queue_depth") v = queue_depth;
  else if (k == "max_request") v = max_request;
  else if (k == "staging_slots") v = staging_slots;
  else if (k == "staging_bytes") v = staging_bytes;
  else if (k == "spin_us") v = spin_us;
  else if (k == "inline_max") v = inline_max;
  else if (k == "bar_map") v = bar_map;
  else if (k == "coalesce") v = coalesce;
  else if (k == "ingest") v = ingest;
  else if (k == "ingest_grid") v = ingest_grid;
  else if (k == "ingest_prio") v = ingest_prio;
  else if (k == "ingest_piece") v = ingest_piece;
  else if (k == "hdp_sync") v = hdp_sync;
  else if (k == "fixed_bufs") v = fixed_bufs;
  else if (k == "io_prof") v = io_prof;
  else if (k == "fd_kcmp") v = fd_kcmp;
  else if (k == "stage_by_bytes") v = stage_by_bytes;
  else if (k == "slot_lifo") v = slot_lifo;
  else if (k == "ingest_min") v = ingest_min;
  else if (k == "trace") v = trace;
  else if (k == "bar_max") v = bar_max;
  else if (k == "bar_nt") v = bar_nt;
  else if (k == "inline_plain") v = inline_plain;
  else if (k == "strict") v = strict;
  else if (k == "direct_io") v = direct_io;
  else if (k == "pgcache_probe") v = pgcache_probe;
  else if (k == "gpu_emulation") v = gpu_emulation;
  else if (k == "numa_bind") v = numa_bind;
  else if (k == "check_freed") v = check_freed;
  else if (k == "stat_info") v = stat_info;
  else if (k == "verbose") v = verbose;
  else return -ENOENT;
  snprintf(buf, sizeof buf, "%ld", v);
  *out = buf;
  return 0;
}

Config &config() {
  static Config c = Config::from_env();
  return c;
}

// ------------------------------------------------------------------- stats
uint64_t tsc_now() { return __rdtsc(); }

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

uint64_t tsc_khz() {
  static const uint64_t khz = [] {
    const uint64_t n0 = mono_ns(), c0 = tsc_now();
    while (mono_ns() - n0 < 5000000) _mm_pause();
    const uint64_t n1 = mono_ns(), c1 = tsc_now();
    return (c1 - c0) * 1000000ull / (n1 - n0);
  }();
  return khz;
}

void Hist::add(uint64_t ns) { b[bucket(ns)].fetch_add(1, std::memory_order_relaxed); }

void Hist::copy_to(uint64_t *out, bool reset) {
  for (int i = 0; i < STROM_HIST_BUCKETS; ++i)
    out[i] = reset ? b[i].exchange(0) : b[i].load();
}

void Stats::inflight_inc(uint64_t n) {
  uint64_t cur = cur_dma_count.fetch_add(n, std::memory_order_relaxed) + n;
  uint64_t mx = max_dma_count.load(std::memory_order_relaxed);
  while (cur > mx && !max_dma_count.compare_exchange_weak(mx, cur)) {
  }
}

void Stats::inflight_dec(uint64_t n) { cur_dma_count.fetch_sub(n, std::memory_order_relaxed); }

int Stats::fill(strom_stat_info *o) {
  if (o->version != 1) return -EINVAL;
  int level = config().stat_info;
  if (level == 0) return -ENODATA;
  o->has_debug = level >= 2;
  o->tsc = tsc_now();
  o->nr_ssd2gpu = nr_ssd2gpu.load();
  o->clk_ssd2gpu = clk_ssd2gpu.load();
  o->nr_setup_prps = nr_setup_prps.load();
  o->clk_setup_prps = clk_setup_prps.load();
  o->nr_submit_dma = nr_submit_dma.load();
  o->clk_submit_dma = clk_submit_dma.load();
  o->nr_wait_dtask = nr_wait_dtask.load();
  o->clk_wait_dtask = clk_wait_dtask.load();
  o->nr_wrong_wakeup = nr_wrong_wakeup.load();
  o->cur_dma_count = cur_dma_count.load();
  o->max_dma_count = max_dma_count.exchange(cur_dma_count.load());  // read-and-reset
  uint64_t *dn[4] = {&o->nr_debug1, &o->nr_debug2, &o->nr_debug3, &o->nr_debug4};
  uint64_t *dc[4] = {&o->clk_debug1, &o->clk_debug2, &o->clk_debug3, &o->clk_debug4};
  for (int i = 0; i < 4; ++i) {
    *dn[i] = o->has_debug ? nr_debug[i].load() : 0;
    *dc[i] = o->has_debug ? clk_debug[i].load() : 0;
  }
  return 0;
}

int Stats::fill_hist(strom_stat_hist *o) {
  if (o->version != 1) return -EINVAL;
  bool r = o->reset != 0;
  io_ns.copy_to(o->io_ns, r);
  copy_ns.copy_to(o->copy_ns, r);
  task_ns.copy_to(o->task_ns, r);
  return 0;
}

// The counters live in /dev/shm/nvme-strom.<pid> when possible so that
// strom_stat (the nvme_stat analogue, reference utils/nvme_stat.c) can watch
// a running process: the reference's counters were kernel-global, a
// userspace engine's are per process.  Layout: StatsShmHeader then Stats.
static Stats *make_stats() {
  const char *off = getenv("STROM_STAT_SHM");
  if (!(off && strcmp(off, "0") == 0)) {
    char path[96];
    snprintf(path, sizeof path, "/dev/shm/nvme-strom.%d", (int)getpid());
    int fd = open(path, O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd >= 0) {
      size_t len = sizeof(StatsShmHeader) + sizeof(Stats);
      if (ftruncate(fd, (off_t)len) == 0) {
        void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (p != MAP_FAILED) {
          close(fd);
          auto *h = new (p) StatsShmHeader();
          h->magic = kStatsShmMagic;
          h->version = 1;
          h->pid = getpid();
          h->stats_bytes = sizeof(Stats);
          h->tsc_hz_hint = 0;
          static char saved[96];
          memcpy(saved, path, sizeof saved);
          atexit([] { unlink(saved); });
          return new ((char *)p + sizeof(StatsShmHeader)) Stats();
        }
      }
      close(fd);
      unlink(path);
    }
  }
  return new Stats();
}

Stats &stats() {
  static Stats *s = make_stats();
  return *s;
}

CallerProf &caller_prof() {
  static CallerProf p;
  return p;
}

// ------------------------------------------------------------- task table
Task *TaskTable::create(int session) {
  Task *t = new Task();
  t->id = next_id_.fetch_add(1);
  t->session = session;
  t->t_start_ns = mono_ns();
  Slot &s = slot_of(t->id);
  std::lock_guard<std::mutex> g(s.mu);
  s.running.emplace(t->id, t);
  return t;
}

void TaskTable::get(Task *t, int n) {
  // a frozen task accepts no new requests (reference :663 Assert)
  t->refcnt.fetch_add(n, std::memory_order_relaxed);
}

void TaskTable::put_n(Task *t, int n, long status) {
  if (status != 0) {
    long zero = 0;
    t->status.compare_exchange_strong(zero, status);
  }
  if (t->refcnt.fetch_sub(n, std::memory_order_acq_rel) != n) return;
  stats().task_ns.add(mono_ns() - t->t_start_ns);
  Slot &s = slot_of(t->id);
  {
    std::lock_guard<std::mutex> g(s.mu);
    s.running.erase(t->id);
    s.done_seq.fetch_add(1, std::memory_order_release);
    if (t->status.load() != 0) {
      t->gmap.reset();
      t->dbuf.reset();
      s.failed.emplace(t->id, t);
      t = nullptr;
    }
  }
  s.cv.notify_all();
  delete t;  // null when parked on the failed list
}

int TaskTable::wait(uint64_t id, long *status, int64_t timeout_ns) {
  Slot &s = slot_of(id);
  uint64_t t0 = tsc_now();
  bool slept = false;
  auto deadline = std::chrono::steady_clock::now() +
                  std::chrono::nanoseconds(timeout_ns < 0 ? 0 : timeout_ns);
  std::unique_lock<std::mutex> g(s.mu);
  int rc;
  bool spun = false;
  uint64_t spin_end = 0;
  for (;;) {
    auto f = s.failed.find(id);
    if (f != s.failed.end()) {
      *status = f->second->status.load();
      delete f->second;
      s.failed.erase(f);
      rc = -EIO;
      break;
    }
    if (s.running.count(id)) {
      if (timeout_ns == 0) { rc = -ETIME; break; }
      // short I/O finishes within a futex wake-up's latency: poll the
      // slot's completion counter (no lock) until one overall deadline
      if (!spun) {
        spun = true;
        uint64_t spin_ns = (uint64_t)config().spin_us * 1000;
        if (timeout_ns > 0 && (uint64_t)timeout_ns < spin_ns) spin_ns = (uint64_t)timeout_ns;
        spin_end = mono_ns() + spin_ns;
      }
      if (mono_ns() < spin_end) {
        const uint64_t seq0 = s.done_seq.load(std::memory_order_acquire);
        g.unlock();
        while (s.done_seq.load(std::memory_order_acquire) == seq0 && mono_ns() < spin_end)
          for (int i = 0; i < 32; ++i) _mm_pause();
        g.lock();
        continue;
      }
      if (slept) stats().nr_wrong_wakeup++;
      slept = true;
      if (timeout_ns < 0) {
        s.cv.wait(g);
      } else if (s.cv.wait_until(g, deadline) == std::cv_status::timeout &&
                 s.running.count(id)) {
        rc = -ETIME;
        break;
      }
      continue;
    }
    *status = 0;
    rc = (id == 0 || id > last_id()) ? -ENOENT : 0;
    break;
  }
  if (slept) {
    stats().nr_wait_dtask++;
    stats().clk_wait_dtask += tsc_now() - t0;
  }
  return rc;
}

int TaskTable::reclaim(int session) {
  int n = 0;
  for (auto &s : slots_) {
    std::lock_guard<std::mutex> g(s.mu);
    for (auto it = s.failed.begin(); it != s.failed.end();) {
      if (it->second->session == session) {
        delete it->second;
        it = s.failed.erase(it);
        ++n;
      } else {
        ++it;
      }
    }
  }
  return n;
}

TaskTable &tasks() {
  static TaskTable t;
  return t;
}

// ---------------------------------------------------------- fault injector
int FaultInjector::on_request(uint32_t *len) {
  long fa = fail_at.load(std::memory_order_relaxed);
  long sa = short_at.load(std::memory_order_relaxed);
  int d = delay_us.load(std::memory_order_relaxed);
  if (!fa && !sa && !d) return 0;
  long n = counter.fetch_add(1) + 1;
  if (d) {
    timespec ts{0, (long)d * 1000};
    nanosleep(&ts, nullptr);
  }
  if (fa && n == fa) return -err.load();
  if (sa && n == sa) {
    int sb = short_bytes.load();
    *len = (uint32_t)sb >= *len ? 0 : *len - (uint32_t)sb;
  }
  return 0;
}

FaultInjector &faults() {
  static FaultInjector f;
  return f;
}

}  // namespace strom
