// engine.h — internal interfaces of libstrom's userspace engine.
//
// Mapping to the reference (kmod/nvme_strom.c, kmod/pmemmap.c):
//   Stats          <- atomic64 counters + STAT_INFO        (nvme_strom.c:64-99, 1986-2028)
//   TaskTable      <- strom_dma_task slots / wait          (nvme_strom.c:504-731, 1127-1235)
//   GpuRegistry    <- mapped_gpu_memory hash               (pmemmap.c:19-495)
//   DmaBufRegistry <- strom_dma_buffer anon-inode + mmap   (pmemmap.c:497-717)
//   classify_file  <- file_is_supported_nvme               (nvme_strom.c:146-502)
//   Raid0Geometry  <- strom_raid0_map_sector               (nvme_strom.c:733-820)
//   plan_chunks    <- do_memcpy_ssd2{gpu,ram} + memcpy_from_nvme_ssd
//                                                          (nvme_strom.c:1303-1405, 1488-1604, 1767-1884)
//   IoEngine       <- PRP pool + async NVMe submit/complete (nvme_strom.c:822-1120)
//
// The design is MI355X-first rather than a translation: requests are
// executed by per-worker io_uring / pread pipelines that land in pinned,
// NUMA-local staging and stream into HBM through per-worker SDMA queues
// (hipMemcpyAsync on non-blocking streams), with completions retired by
// the same worker that issued them (no callback threads).
#pragma once

#include <sys/types.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "strom/strom.h"
#include "../../kmod/strom_core.h"

namespace strom {

// ------------------------------------------------------------------ config
// kCache: the uring path on the buffered descriptor (page-cache reads):
// the engine + HBM ingest ceiling with the storage taken out (tools.ceiling)
enum class BackendKind { kPsync, kUring, kFake, kCache };

struct Config {
  // defaults from the MI355X-host sweep (nvme_strom_amd/tools/tune.py)
  BackendKind backend = BackendKind::kUring;
  int workers = 4;               // I/O worker threads (one SDMA stream each)
  int queue_depth = 8;           // in-flight reads per worker (uring)
  uint32_t max_request = 1u << 20;  // merge limit (bytes); v0.6 used 128 KiB
  int staging_slots = 4;         // minimum pinned slots per worker (GPU dest)
  bool slot_lifo = true;         // hand out the most recently freed staging slot
                                 // (false: FIFO, adjacent requests in adjacent slots).
                                 // Bench A/B over three boxes, 9 alternated pairs: LIFO
                                 // ahead or level in 8, 18.5 -> 21.3 GiB/s mean on a
                                 // noisy box, +3 % on a quiet one, and steadier
                                 // (profiles/r6/staging/*_r6{n,o,p}.json)
  bool stage_by_bytes = true;    // at least queue_depth slots, in-flight reads bounded
                                 // by staging bytes (short requests go deeper).  With
                                 // FIFO slots it cost the bench 12 % (8 slots rotating
                                 // instead of 4, profiles/r6/staging/*_r6m.json); with
                                 // slot_lifo the bench is level (27.7 vs 27.2 GiB/s) and
                                 // 227-488 KiB extent reads gain 5-14 % (*_r6t.json)
  uint32_t staging_bytes = 0;    // opt-in: pinned staging per worker, slots =
                                 // max(staging_slots, staging_bytes / max_request),
                                 // queue depth grows to match.  Off by default:
                                 // the box's storage lost throughput with more
                                 // in flight (profiles/r1e/sweep_*.json)
  uint32_t spin_us = 20;         // idle workers / WAIT spin this long before
                                 // sleeping on a futex (hand-off latency)
  uint32_t inline_max = 64u << 10;  // single requests up to this run inline
  bool bar_map = true;           // CPU-map HBM through the large BAR (dma-buf)
  bool coalesce = true;          // workers merge adjacent staged HBM copies
  bool ingest = true;            // staged reads reach HBM through the GPU ingest
                                 // grid (ingest.hip) instead of SDMA copies
  int ingest_grid = 16;          // workgroups of the ingest grid (CUs it holds)
  int ingest_prio = 1;           // 1: the grid's stream is a greatest-priority
                                 // non-blocking one (a hardware queue of its own);
                                 // 0: a CU-masked stream (its own queue too, but
                                 // blocking: it synchronizes with the NULL stream)
  uint32_t ingest_piece = 256u << 10;  // bytes per ingest descriptor
  int hdp_sync = 2;              // HDP flush after CPU stores through the BAR:
                                 // 0 posted; 1 read back after every write; 2 read
                                 // back once per worker batch / per ioctl's page-cache
                                 // chunks, posted on the synchronous small-read path
                                 // (same-thread consumer; A/B in profiles/r4/hdp)
  bool fixed_bufs = true;        // register each worker's pinned staging with its
                                 // io_uring (IORING_REGISTER_BUFFERS) and read
                                 // into it with READ_FIXED (no per-I/O page
                                 // pinning); falls back to READ when the
                                 // kernel or RLIMIT_MEMLOCK refuses
  uint32_t bar_max = 256u << 10; // requests up to this go staging -> BAR by CPU
  int bar_nt = 1;                // BAR stores: 1 whole-line non-temporal (AVX-512 /
                                 // AVX2), 0 memcpy.  QD1 4 KiB: the drain paid at
                                 // the next locked instruction 554 -> 382 ns, p50
                                 // 5.04 -> 4.16 us on storage, 1.62 -> 1.44 engine-only
                                 // (profiles/r5/qd1/qd1_ab_r5p.json)
  bool inline_plain = false;     // synchronous reads bound for the BAR land in plain
                                 // (unpinned) memory: CPU stores need no pinning
  uint32_t ingest_min = 0;       // worker requests below this go staging -> BAR by
                                 // CPU stores even when the ingest grid runs
  bool io_prof = false;          // per-worker phase attribution (strom_io_prof)
  bool fd_kcmp = false;          // synchronous reads on a plain descriptor: keep a
                                 // dup of it and check identity with kcmp (~90 ns
                                 // below an fstat).  Opt-in: closing that dup when
                                 // the thread moves to another file drops the
                                 // process's fcntl record locks on the file, and
                                 // while held it keeps flock locks and an unlinked
                                 // file's space alive; registered
                                 // files (strom_register_file) skip both costs
  bool strict = false;           // reference CHECK_FILE rules only
  bool direct_io = true;         // O_DIRECT reads of uncached chunks
  bool pgcache_probe = true;     // residency scoring (mincore)
  bool gpu_emulation = false;    // accept host memory as "GPU" (CPU tests)
  bool numa_bind = true;         // pin workers near the GPU / SSD
  bool check_freed = true;       // re-check a mapping's allocation identity per
                                 // SSD2GPU (freed / recycled range -> -ENOENT)
  int stat_info = 1;             // 0 off, 1 on, 2 +debug fields
  int verbose = 0;
  bool trace = false;            // roctx ranges around engine calls

  static Config from_env();
  int set(const std::string &key, const std::string &value);
  int get(const std::string &key, std::string *out) const;
};

Config &config();                // process-wide, guarded by engine lock

// ------------------------------------------------------------------- stats
uint64_t tsc_now();
uint64_t mono_ns();
uint64_t tsc_khz();   // calibrated once against CLOCK_MONOTONIC

struct Hist {
  std::atomic<uint64_t> b[STROM_HIST_BUCKETS];
  static int bucket(uint64_t ns) {   // bucket k: [2^(k-1), 2^k)
    int k = ns ? 64 - __builtin_clzll(ns) : 0;
    return k >= STROM_HIST_BUCKETS ? STROM_HIST_BUCKETS - 1 : k;
  }
  void add(uint64_t ns);
  void copy_to(uint64_t *out, bool reset);
};

struct Stats {
  std::atomic<uint64_t> nr_ssd2gpu{0}, clk_ssd2gpu{0};
  std::atomic<uint64_t> nr_setup_prps{0}, clk_setup_prps{0};
  std::atomic<uint64_t> nr_submit_dma{0}, clk_submit_dma{0};
  std::atomic<uint64_t> nr_wait_dtask{0}, clk_wait_dtask{0};
  std::atomic<uint64_t> nr_wrong_wakeup{0};
  std::atomic<uint64_t> cur_dma_count{0}, max_dma_count{0};
  std::atomic<uint64_t> nr_debug[4]{}, clk_debug[4]{};
  Hist io_ns, copy_ns, task_ns;

  void inflight_inc(uint64_t n = 1);
  void inflight_dec(uint64_t n = 1);
  int fill(strom_stat_info *out);
  int fill_hist(strom_stat_hist *out);
};

Stats &stats();

// submitting-thread side of the attribution (config io_prof): SSD2GPU /
// SSD2RAM calls and the TSC cycles they spent planning, building requests
// and handing them to the workers
struct CallerProf {
  std::atomic<uint64_t> calls{0}, plan{0}, build{0}, submit{0};
};
CallerProf &caller_prof();

// Readers (strom_stat, nvme_strom_amd/utils/stat.py) index the export as a
// flat array of u64: 11 scalars, debug nr[4], debug clk[4], 3 x 48 buckets.
static_assert(sizeof(Stats) == (11 + 8 + 3 * STROM_HIST_BUCKETS) * 8, "Stats export layout");

// shared-memory export header (/dev/shm/nvme-strom.<pid>), Stats follows
constexpr uint64_t kStatsShmMagic = 0x53544f524d535431ull;  // "STORMST1"
struct StatsShmHeader {
  uint64_t magic;
  uint32_t version;
  int32_t pid;
  uint64_t stats_bytes;
  uint64_t tsc_hz_hint;
  uint64_t reserved[4];
};

// ------------------------------------------------------------- task table
struct GpuMapping;
struct DmaBuffer;

struct Task {
  uint64_t id = 0;
  int session = 0;
  std::atomic<int> refcnt{1};       // 1 (submitter) + 1 per request
  std::atomic<long> status{0};      // first error wins
  bool frozen = false;              // submission finished
  uint64_t t_start_ns = 0;
  std::shared_ptr<GpuMapping> gmap; // pinned for the task's lifetime
  std::shared_ptr<DmaBuffer> dbuf;
};

class TaskTable {
 public:
  static constexpr int kSlots = 512;
  Task *create(int session);
  void get(Task *t, int n = 1);
  void put(Task *t, long status) { put_n(t, 1, status); }
  // drop n references at once (a worker's batch of completions of one task);
  // a non-zero status is recorded first (first error wins)
  void put_n(Task *t, int n, long status);
  // 0 done OK; -EIO failed (status set); -ENOENT never issued; -ETIME timeout
  int wait(uint64_t id, long *status, int64_t timeout_ns);
  int reclaim(int session);         // fd-close analogue: drop failed records
  uint64_t last_id() const { return next_id_.load() - 1; }

 private:
  struct Slot {
    std::mutex mu;
    std::condition_variable cv;
    std::unordered_map<uint64_t, Task *> running;
    std::unordered_map<uint64_t, Task *> failed;
    std::atomic<uint64_t> done_seq{0};  // bumped per finished task (lock-free spin)
  };
  Slot &slot_of(uint64_t id) { return slots_[(id * 0x9E3779B97F4A7C15ull) >> 55]; }
  Slot slots_[kSlots];
  std::atomic<uint64_t> next_id_{1};
};

TaskTable &tasks();

// ------------------------------------------------------ GPU memory registry
struct GpuMapping {
  unsigned long handle = 0;
  uint64_t va = 0;            // user VA
  uint64_t base = 0;          // va aligned down to 64 KiB
  size_t length = 0;          // user length
  size_t map_offset = 0;      // va - base
  size_t map_length = 0;      // map_offset + length
  int device = -1;            // HIP ordinal, -1 = host-emulated
  uid_t owner = 0;
  int dmabuf_fd = -1;
  uint32_t version = 1;
  // identity of the allocation behind the range, taken at MAP time and
  // re-checked per request (GpuRegistry::validate): the HIP buffer id of a
  // device allocation, or the covering VMA of emulated (host) memory
  uint64_t ident = 0;
  // Large-BAR CPU mapping of the range (dma-buf export + mmap), or null.
  // bar_va is the device VA that bar[0] aliases.
  uint8_t *bar = nullptr;
  uint64_t bar_va = 0;
  size_t bar_len = 0;
  volatile uint32_t *hdp = nullptr;  // HDP_MEM_FLUSH_CNTL of the device, or null
  std::atomic<int> inflight{0};
  // CPU store of [src, src+len) into HBM at device VA dst through the BAR;
  // false when the range is not BAR-mapped.  Ends with a read-back that
  // flushes the posted writes, so the data is in HBM when this returns.
  bool bar_write(uint64_t dst, const void *src, size_t len, bool flush = true) const;
  bool bar_write_mode(uint64_t dst, const void *src, size_t len, int mode) const;
  // make CPU stores through the BAR (ending at `last`) visible to shaders:
  // sfence, then an HDP flush (write + read back the flush register, as
  // the runtime does for CPU-written kernargs in VRAM); without the
  // register, a read-back of the last dword drains the posted writes
  // `batch`: the flush ends a batch / ioctl (hdp_sync=2 reads it back)
  void bar_flush(const uint8_t *last, bool batch = false) const;
  ~GpuMapping();
  bool detached = false;
  std::atomic<bool> draining{false};  // an UNMAP waits for inflight == 0
  std::mutex mu;
  std::condition_variable cv;
};

class GpuRegistry {
 public:
  int map(uint64_t va, size_t len, int dmabuf_fd, strom_map_gpu_memory *out);
  int unmap(unsigned long handle);
  int list(strom_list_gpu_memory *out);
  int info(strom_info_gpu_memory *out);
  std::shared_ptr<GpuMapping> get(unsigned long handle);
  // get() through a per-thread one-entry cache, valid while no mapping was
  // added, removed or detached since (the generation): the synchronous
  // small-read path then takes no lock and makes no geteuid() call.  The
  // reference stays valid until this thread's next get_cached().
  const std::shared_ptr<GpuMapping> &get_cached(unsigned long handle);
  // 0 while the allocation that was mapped still backs the range; else the
  // mapping is detached (like the reference's free callback,
  // kmod/pmemmap.c:150-208) and -ENOENT returned
  int validate(const std::shared_ptr<GpuMapping> &m);
  uint64_t detached_count() const { return detached_.load(); }

 private:
  std::mutex mu_;
  std::map<unsigned long, std::shared_ptr<GpuMapping>> maps_;
  unsigned long next_ = 0x5350000000000000ul;  // 'S','P' tag + counter
  std::atomic<uint64_t> detached_{0};
  std::atomic<uint64_t> gen_{1};
};

GpuRegistry &gpu_registry();

// ----------------------------------------------------- DMA buffer registry
struct DmaBuffer {
  dev_t dev = 0;
  ino_t ino = 0;
  size_t length = 0;
  int node = -1;
  uint64_t gen = 0;                 // registration order (gc only drops older ones)
};

// Which VMA covers an address (PROCMAP_QUERY on /proc/self/maps, Linux
// >= 6.11, else a text scan): the userspace find_vma().
struct VmaInfo {
  uint64_t start = 0, end = 0, pgoff = 0, ino = 0;
  dev_t dev = 0;
  bool dmabuf = false;   // a mapping of one of our "strom-dmabuf" memfds
};
// 0 and *out filled; -ENOENT nothing mapped at addr; other -errno on failure
int vma_query(uint64_t addr, VmaInfo *out);

class DmaBufRegistry {
 public:
  int alloc(size_t length, int node, int *user_fd);
  // Resolve a user VA range to (buffer, byte offset).  -EINVAL when the
  // range is not inside an ALLOC_DMA_BUFFER mapping (find_vma analogue).
  // Mappings made through map() are found in an address index without a
  // syscall; others (a caller's own mmap of the fd) by one VMA query.
  int resolve(const void *uaddr, size_t len, std::shared_ptr<DmaBuffer> *buf,
              size_t *offset);
  // mmap a DMA-buffer fd (MAP_SHARED) and index the range / drop it again
  int map(int fd, size_t len, void **addr);
  int unmap(void *addr, size_t len);
  // Drop buffers no fd and no mapping of this process refers to any more
  // (the fd-close analogue of the reference's anon-inode release); returns
  // the number still registered
  int gc();
  size_t count();

 private:
  struct Range {
    uint64_t end;
    size_t pgoff;
    std::shared_ptr<DmaBuffer> buf;
  };
  std::mutex mu_;
  uint64_t next_gen_ = 1;              // under mu_
  std::map<std::pair<dev_t, ino_t>, std::shared_ptr<DmaBuffer>> bufs_;
  std::map<uint64_t, Range> ranges_;   // start -> engine-made mapping
};

DmaBufRegistry &dmabuf_registry();

// ------------------------------------------------------- file classifier
// md raid0 geometry: the C struct of the shared core (kmod/strom_core.h)
// that both providers remap with.
using Raid0Geometry = strom_raid0;

struct FileClass {
  dev_t dev = 0;
  ino_t ino = 0;
  off_t size = 0;
  uint32_t fs_bsize = 0;
  uint64_t fs_magic = 0;
  std::string fs_name;
  std::string disk;          // nvme0n1 / md0 / "" (virtual)
  bool nvme = false;
  bool md_raid0 = false;
  int numa_node = -1;
  bool dma64 = true;
  uint64_t part_start_sect = 0;
  Raid0Geometry raid0{};
  std::vector<std::string> members;
};

int classify_file(int fd, FileClass *out, bool strict);
// PCI function "dddd:bb:dd.f" of the NVMe controller of a namespace disk
// (first path of a multipath head), "" when not found
std::string nvme_controller_bdf(const std::string &disk);

// ------------------------------------------------------------ chunk plan
struct IoRange {
  uint64_t file_off;
  uint64_t dest_off;
  uint32_t len;
  int member;                // raid0 / stripe-set member (-1 = whole device)
  uint64_t msect = 0;        // member 512-B sector (member >= 0)
};

struct ChunkPlan {
  std::vector<IoRange> ssd;          // merged storage requests
  std::vector<uint64_t> ram_fpos;    // page-cache chunks: file positions
  std::vector<uint64_t> ram_dest;    //   and their destination offsets
  std::vector<uint32_t> ids_out;     // landing order
  uint32_t nr_ram = 0, nr_ssd = 0, nr_submit = 0, nr_blocks = 0;
};

struct PlanParams {
  const uint32_t *ids = nullptr;
  uint32_t nr_chunks = 0;
  uint32_t chunk_sz = 0;
  uint32_t relseg_sz = 0;
  uint64_t file_size = 0;
  uint32_t max_request = 1u << 20;
  uint64_t dest_segment = 0;         // 0 = no segment boundary rule
  bool reorder = true;               // SSD2GPU: SSD head / RAM tail
  const Raid0Geometry *raid0 = nullptr;   // split requests at stripe chunks
  uint64_t part_start_sect = 0;
  // file 4 KiB page -> volume block (4 KiB units); null = identity (the
  // engine reads by file offset, so merging never needs the device layout)
  int (*bmap)(void *ctx, uint64_t fblk, uint64_t *dblk) = nullptr;
  void *bmap_ctx = nullptr;
  // resident pages of [fpos, fpos+len) or -1 unknown; null = never cached
  std::function<long(uint64_t, uint32_t)> resident;
};

int plan_chunks(const PlanParams &p, ChunkPlan *out);
int plan_xfer(const PlanParams &p, strom_file_extent *x, uint32_t n, uint32_t gap_max,
              bool planner, ChunkPlan *out, uint64_t *dst_bytes, uint64_t *read_bytes);

// ------------------------------------------------------------ I/O engine
struct IoReq {
  Task *task = nullptr;
  int fd = -1;                // O_DIRECT descriptor when available
  int fd_buffered = -1;       // fallback when O_DIRECT refuses a request
  uint64_t off = 0;
  uint32_t len = 0;
  uint32_t valid = 0;         // bytes before EOF (rest zero-filled)
  uint8_t *host_dst = nullptr;
  uint64_t gpu_dst = 0;       // device VA, 0 if host destination
  int device = -1;            // -1 host-emulated GPU
  uint64_t t_submit_ns = 0;
  uint64_t t_submit_tsc = 0;
  GpuMapping *gmap = nullptr; // inflight counter owner
  long *status_out = nullptr; // task-less synchronous request: status lands here
};

class IoEngine {
 public:
  explicit IoEngine(const Config &cfg);
  ~IoEngine();
  void submit(std::vector<IoReq> &reqs);
  // per-worker phase attribution summed over the workers (config io_prof):
  // out[0] workers, out[1] TSC kHz, then kProfPhases cycle sums, then
  // kProfCounts counters; returns the number of u64 written
  static constexpr int kProfPhases = 11, kProfCounts = 5;
  int prof(uint64_t *out, int nout, bool reset);
  // Small single-request tasks run on the caller's thread (no worker
  // hand-off, no WAIT wake-up): the 4 KiB latency path.
  void run_inline(IoReq &r);
  int workers() const { return (int)workers_.size(); }

  struct Worker;
 private:
  std::vector<std::unique_ptr<Worker>> workers_;
  std::mutex prof_mu_;            // prof(): the workers' counter baselines
  std::atomic<uint32_t> rr_{0};
};

// Completion helper shared by the workers.
void finish_request(IoReq &r, long status);

// ---------------------------------------------------------- fault injector
struct FaultInjector {
  std::atomic<long> counter{0};
  std::atomic<long> fail_at{0};
  std::atomic<int> err{5};
  std::atomic<long> short_at{0};
  std::atomic<int> short_bytes{0};
  std::atomic<int> delay_us{0};
  // returns 0 or -errno; may shrink *len
  int on_request(uint32_t *len);
  // fake backend: completions delivered in a seeded random order
  std::atomic<uint64_t> fake_seed{0x5eed};
  std::atomic<uint64_t> fake_completions{0}, fake_reordered{0};
};
FaultInjector &faults();

// ------------------------------------------------------------- HBM ingest
// Host side of the persistent GPU pull grid (ingest.cc / ingest.hip): staged
// bytes in pinned host memory are posted as descriptors and copied into HBM
// by the GPU; completion is a host-memory word per descriptor.
class Ingest {
 public:
  static Ingest *get(int device);   // null when disabled or unavailable
  // Post [src, src+len) -> device VA dst as ceil(len / piece) descriptors with
  // consecutive sequence numbers *first .. *first + *n - 1.  false: not
  // postable (alignment, grid failure) — the caller falls back to SDMA.
  bool post(const void *src, uint64_t dst, uint32_t len, uint64_t *seq);
  bool post_many(const void *src, uint64_t dst, uint32_t len, uint32_t piece, uint64_t *first,
                 uint32_t *n);
  // Post several ranges under one lock acquisition (a worker's batch of
  // finished reads); each run's ok / first / n are filled in.
  struct Run {
    const void *src;
    uint64_t dst;
    uint32_t len;
    bool ok;
    uint64_t first;
    uint32_t n;
  };
  void post_runs(Run *runs, size_t nruns, uint32_t piece);
  bool is_done(uint64_t seq) const;
  void retired(uint32_t n);         // the poster observed n descriptors done
  void idle();                      // stop the grid when nothing is outstanding
  void shutdown();
  void info(uint64_t *out);         // {available, launches, posted, outstanding}

 private:
  explicit Ingest(int device);
  bool init();
  int launch_grid();
  int start_locked();
  bool write_desc(uint64_t s, const void *src, uint64_t dst, uint32_t len);

  int device_;
  uint32_t nslots_ = 0, grid_ = 0;
  void *host_ = nullptr, *ring_ = nullptr, *next_ = nullptr;
  volatile uint64_t *done_ = nullptr, *stop_ = nullptr;
  void *stream_ = nullptr, *end_ev_ = nullptr;
  std::mutex mu_;                      // grid start / stop only
  std::atomic<uint64_t> post_seq_{0};  // next sequence number to reserve
  // 2 x descriptors outstanding | grid running: a poster adds before it
  // reserves, and the grid is stopped only by a CAS from exactly "running,
  // nothing outstanding", so no reservation can race a stop
  std::atomic<uint64_t> state_{0};
  bool launched_ = false;              // under mu_
  std::atomic<bool> dead_{false};
  std::atomic<bool> gone_{false};     // shutdown() saw the grid exit
  uint64_t nr_launch_ = 0;
};

// ------------------------------------------------------------- HIP glue
namespace hip {
bool available();
int device_count();
// device ordinal of a device pointer, -1 when not device memory; sets
// *alloc_base/*alloc_size to the enclosing allocation when known.
int pointer_device(uint64_t va, uint64_t *alloc_base, size_t *alloc_size);
void *host_alloc(size_t bytes, bool coherent = false);  // pinned, portable
void host_free(void *p);
// THP-backed, hipHostRegister'ed; `uncached`: GPU reads bypass its caches
// (staging the ingest grid pulls from)
void *host_alloc_thp(size_t bytes, bool uncached = false);
void host_free_thp(void *p, size_t bytes);
// CPU mapping of device memory [va, va+len) through its dma-buf export;
// returns the mapping (and sets *map_va/*map_len to what it covers) or null.
uint8_t *bar_map(uint64_t va, size_t len, uint64_t *map_va, size_t *map_len);
volatile uint32_t *hdp_flush_reg(int device);  // null when not exposed
void bar_unmap(uint8_t *p, size_t len);
// dma-buf fd of the whole allocation holding [va, va+len) (PCIe mapping
// type, for peer-to-peer importers) and va's byte offset inside it
int export_dmabuf(uint64_t va, size_t len, int *fd, uint64_t *offset, int *device);
int copy_dtoh(void *dst, uint64_t src, size_t len);   // synchronous, 0 / -EIO
int copy_htod(uint64_t dst, const void *src, size_t len);
int numa_node_of_device(int device);
// unique id of the live allocation holding va (HIP buffer id), 0 if none
uint64_t buffer_id(uint64_t va);
}  // namespace hip

// -------------------------------------------------------------- engine
class Engine {
 public:
  const uint64_t gen_;           // instance number (per-thread caches key on it)
  Engine();
  ~Engine();
  int ioctl(int session, unsigned long cmd, void *arg);
  // Synchronous read of [file_off, file_off+len) into a mapped GPU range on
  // the caller's thread: no task, no residency probe (O_DIRECT reads see
  // dirty page-cache data: the kernel writes the range back first).  The
  // 4 KiB latency path of strom_pread_gpu.  -EAGAIN: use the task path.
  // `checked`: the file's size was just re-read (no second retry).
  long pread_sync(unsigned long handle, size_t offset, int fd, uint64_t file_off, uint64_t len,
                  bool checked = false);
  IoEngine &io() { return *io_; }
  struct OpenFile;
  // Stripe sets (PAR2 without md): a logical file striped in `unit`-byte
  // stripes over member files, usually one per SSD; the returned pseudo
  // descriptor is accepted wherever a file descriptor is (CHECK_FILE,
  // SSD2GPU, SSD2RAM).  Process-wide: survives engine resets.
  int stripe_open(const int *fds, uint32_t n, uint32_t unit, uint64_t size);
  int stripe_close(int sfd);
  struct StripeSet;

  // the per-file cache (fstat-validated): classification, descriptors, map
  std::shared_ptr<OpenFile> open_file(int fd, int *err);
  // open_file() for the synchronous small-read path: when this thread's
  // last descriptor still names the same open file description (kcmp
  // against a dup of it; *fast set — the cached size may be stale) or, where
  // kcmp is refused, the same (device, inode, ctime, size) by an fstat, the
  // cached entry is returned without the lock, map lookup or reference
  // count.  The reference stays valid until this thread's next call.
  const std::shared_ptr<OpenFile> &open_file_cached(int fd, int *err, bool *fast = nullptr);
  // drop this thread's cached file (the next open_file_cached stats again)
  void forget_cached_file();

  // Registered files (io_uring's IORING_REGISTER_FILES, for this engine):
  // register_file() resolves a descriptor once and returns an id
  // (kRegFdBase + slot) accepted wherever a file descriptor is.  The engine
  // reads through its own descriptors of the file, so an id needs no
  // per-read identity check (no fstat, no kcmp: the caller may even close
  // its descriptor); only a read past the cached size or a short one
  // re-reads the size.  Ids end with unregister_file() or an engine reset.
  int register_file(int fd);
  int unregister_file(int rfd);
  // the registered file of rfd (nullptr: none); per-thread cache validated
  // by one atomic load of the table's version
  const std::shared_ptr<OpenFile> &registered(int rfd);

 private:
  int check_file(strom_check_file *a);
  int memcpy_ssd2gpu(int session, strom_memcpy_ssd2gpu *a);
  int memcpy_extents(int session, strom_memcpy_ssd2gpu_extents *a);
  int memcpy_ssd2ram(int session, strom_memcpy_ssd2ram *a);
  int memcpy_wait(strom_memcpy_wait *a);
  int memcpy_wait_timed(strom_memcpy_wait_timed *a);

  std::shared_ptr<StripeSet> stripe(int fd);
  // re-read a registered file's size (open_file on the engine's descriptor)
  void refresh_registered(int rfd);
  // the file of an asynchronous task (MEMCPY_SSD2GPU / SSD2RAM / CHECK_FILE):
  // a registered id's size is re-read first — such a task cannot redo a
  // read after it returned, so a grown or shrunk file (a PostgreSQL segment)
  // must be planned with its size now, not the one cached at registration
  std::shared_ptr<OpenFile> task_file(int fd, int *err);

  std::unique_ptr<IoEngine> io_;
  std::mutex files_mu_;
  std::map<std::pair<dev_t, ino_t>, std::shared_ptr<OpenFile>> files_;
  std::mutex reg_mu_;
  std::vector<std::shared_ptr<OpenFile>> reg_;   // slot i: id kRegFdBase + i
  std::atomic<uint64_t> reg_ver_{0};             // bumped by every (un)registration
};

// pseudo descriptors of stripe sets: far above any real fd
constexpr int kStripeFdBase = 0x7f000000;
// ids of registered files: below the stripe sets, above any real fd
constexpr int kRegFdBase = 0x7e000000;
constexpr int kRegMax = 4096;
inline bool is_registered_id(int fd) { return fd >= kRegFdBase && fd < kRegFdBase + kRegMax; }

Engine &engine();
void engine_reset();

// Phase probe of the synchronous small-read path (strom_pread_gpu_phases):
// while a caller thread has tl_phase set, the path stamps mono_ns() at the
// end of each phase (STROM_NPHASE points, strom.h).
extern thread_local uint64_t *tl_phase;
inline void phase_mark(int k) {
  if (__builtin_expect(tl_phase != nullptr, 0)) tl_phase[k] = mono_ns();
}

#define STROM_LOG(lvl, ...)                                   \
  do {                                                        \
    if (::strom::config().verbose >= (lvl)) {                 \
      fprintf(stderr, "[strom] " __VA_ARGS__);                \
      fputc('\n', stderr);                                    \
    }                                                         \
  } while (0)

}  // namespace strom
