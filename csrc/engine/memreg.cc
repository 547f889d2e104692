// memreg.cc — GPU memory mapping registry and NUMA DMA buffers.
//
// GpuRegistry re-designs the reference's mapped_gpu_memory table
// (kmod/pmemmap.c:33-495) for HIP: a mapping is a validated HBM range of a
// hipMalloc allocation (hipPointerGetAttributes + hipMemGetAddressRange),
// aligned down to the same 64 KiB granule, owned by the caller's euid.
// Handles are opaque tagged counters (never kernel pointers).  UNMAP waits
// for in-flight requests that target the range and then frees the record,
// fixing reference defect #7 (pmemmap.c:375-388 never freed nor waited).
// INFO returns per-page device addresses; the kmod fills bus addresses
// from the imported dma-buf sg_table instead.
//
// A freed allocation is detected per request: MAP records the identity of
// the allocation (HIP buffer id), SSD2GPU re-reads it, and a mismatch (the
// range was hipFree'd, or freed and re-allocated at the same VA) detaches
// the mapping with -ENOENT instead of writing into whatever now lives there
// (reference: nvidia's free callback, kmod/pmemmap.c:150-208).  Ranges a
// caching allocator recycles INSIDE one live hipMalloc block keep their
// identity — exactly what the reference's callback saw too.
//
// DmaBufRegistry replaces the anon-inode DMA buffer (pmemmap.c:497-717):
// a memfd named "strom-dmabuf<node>:<size>", whose shared NUMA policy is
// bound to the requested node and whose pages are pre-faulted there.  The
// SSD2RAM destination check is the find_vma()/f_op test: mappings made
// through DmaBufRegistry::map sit in an address index (no syscall); any
// other address is looked up with one PROCMAP_QUERY ioctl on
// /proc/self/maps (Linux >= 6.11; a text scan before that).  The range must
// lie inside a mapping of one of our memfds, and the byte offset is
// vm_pgoff + (uaddr - vm_start).  Buffers nothing refers to any more are
// dropped by gc() (run on every ALLOC_DMA_BUFFER).
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/ioctl.h>
#include <sys/ioctl.h>
#include <sys/sysmacros.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <x86intrin.h>

#include <set>

#include "engine.h"

#ifndef MPOL_BIND
#define MPOL_BIND 2
#endif
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

namespace strom {

// ------------------------------------------------------- GPU registry
GpuMapping::~GpuMapping() { hip::bar_unmap(bar, bar_len); }

// Copy into write-combining BAR memory with whole-line (64-byte)
// non-temporal stores, so every WC buffer leaves the core as one full-line
// PCIe write (config bar_nt; memcpy's store mix is the default).
__attribute__((target("avx512f"))) static void bar_copy_nt512(uint8_t *d, const uint8_t *s,
                                                              size_t n) {
  size_t i = 0;
  for (; i + 64 <= n; i += 64)
    _mm512_stream_si512((__m512i *)(d + i), _mm512_loadu_si512((const void *)(s + i)));
  if (i < n) memcpy(d + i, s + i, n - i);
}

__attribute__((target("avx2"))) static void bar_copy_nt256(uint8_t *d, const uint8_t *s,
                                                           size_t n) {
  size_t i = 0;
  for (; i + 32 <= n; i += 32)
    _mm256_stream_si256((__m256i *)(d + i), _mm256_loadu_si256((const __m256i *)(s + i)));
  if (i < n) memcpy(d + i, s + i, n - i);
}

// probe-only orders (strom_engine_costs modes 2 / 3): whole lines last to
// first, and the string move (ERMS) — does another store order shorten the
// write-combining drain paid after a 4 KiB store?
__attribute__((target("avx512f"))) static void bar_copy_nt512_rev(uint8_t *d, const uint8_t *s,
                                                                  size_t n) {
  size_t i = n & ~(size_t)63;
  if (i < n) memcpy(d + i, s + i, n - i);
  while (i) {
    i -= 64;
    _mm512_stream_si512((__m512i *)(d + i), _mm512_loadu_si512((const void *)(s + i)));
  }
}

static void bar_copy_movsb(uint8_t *d, const uint8_t *s, size_t n) {
  asm volatile("rep movsb" : "+D"(d), "+S"(s), "+c"(n) : : "memory");
}

static void bar_copy(uint8_t *d, const void *src, size_t n, int mode) {
  static const int have512 = __builtin_cpu_supports("avx512f") ? 1 : 0;
  static const int have256 = __builtin_cpu_supports("avx2") ? 1 : 0;
  const uint8_t *s = (const uint8_t *)src;
  if (mode == 2 && have512 && !((uintptr_t)d & 63)) return bar_copy_nt512_rev(d, s, n);
  if (mode == 3) return bar_copy_movsb(d, s, n);
  // 64-byte aligned destinations only: a line split over two WC buffers
  // gains nothing
  if (mode && !((uintptr_t)d & 63)) {
    if (have512) return bar_copy_nt512(d, s, n);
    if (have256) return bar_copy_nt256(d, s, n);
  }
  memcpy(d, s, n);
}

// one BAR store of len bytes with the given copy mode and its HDP flush
// (strom_engine_costs A/B)
bool GpuMapping::bar_write_mode(uint64_t dst, const void *src, size_t len, int mode) const {
  if (!bar || len == 0 || dst < bar_va || dst + len > bar_va + bar_len) return false;
  uint8_t *p = bar + (dst - bar_va);
  bar_copy(p, src, len, mode);
  bar_flush(p + ((len - 1) & ~(size_t)3));
  return true;
}

bool GpuMapping::bar_write(uint64_t dst, const void *src, size_t len, bool flush) const {
  if (!bar || len == 0 || dst < bar_va || dst + len > bar_va + bar_len) return false;
  uint8_t *p = bar + (dst - bar_va);
  bar_copy(p, src, len, config().bar_nt);
  phase_mark(4);
  if (flush) bar_flush(p + ((len - 1) & ~(size_t)3));
  phase_mark(5);
  return true;
}

// HDP flush after CPU stores through the BAR (config hdp_sync):
//   2 (default)  read back once per worker batch and per ioctl's page-cache
//                chunks (`batch`): the flush has completed before the task
//                completes, for any consumer (another thread's kernel, an RCCL
//                peer).  Posted on the synchronous small-read path (pread_gpu):
//                there the consumer is started by the same thread, whose
//                doorbell write is posted behind the flush, and the read-back
//                would add its PCIe round trip to every 4 KiB read
//                (profiles/r4/hdp has the A/B).
//   1            read back after every write (what the runtime does for
//                kernargs it writes into VRAM).
//   0            posted everywhere.
// tests/test_gpu_core.py checks the posted form (next kernel, SDMA readback,
// a kernel on another stream) on hundreds of distinct offsets.
void GpuMapping::bar_flush(const uint8_t *last, bool batch) const {
  _mm_sfence();
  if (hdp) {
    *hdp = 1u;
    const int mode = config().hdp_sync;
    if (mode == 1 || (mode == 2 && batch)) (void)*hdp;
  } else {
    // no flush register: a read from the device cannot pass the posted
    // writes before it
    (void)*(const volatile uint32_t *)last;
  }
}

int GpuRegistry::map(uint64_t va, size_t len, int dmabuf_fd, strom_map_gpu_memory *out) {
  if (va == 0 || len == 0) return -EINVAL;
  if (va + len < va) return -EINVAL;
  int device = -1;
  uint64_t abase = 0;
  size_t asize = 0;
  if (hip::available()) device = hip::pointer_device(va, &abase, &asize);
  if (device >= 0) {
    if (asize && (va < abase || va + len > abase + asize)) return -ERANGE;
  } else if (!config().gpu_emulation) {
    return -EINVAL;  // not device memory
  }
  auto m = std::make_shared<GpuMapping>();
  m->va = va;
  m->base = va & ~(uint64_t)(STROM_GPU_BOUND_SIZE - 1);
  m->map_offset = va - m->base;
  m->length = len;
  m->map_length = m->map_offset + len;
  m->device = device;
  m->owner = geteuid();
  m->dmabuf_fd = dmabuf_fd;
  // identity: the HIP buffer id; emulated (host) memory has none that
  // survives VMA merges, so there it is "both ends still mapped"
  m->ident = device >= 0 ? hip::buffer_id(va) : 1;
  uint64_t npages = (m->map_length + STROM_GPU_BOUND_SIZE - 1) >> STROM_GPU_BOUND_SHIFT;
  if (npages > 0xffffffffull) return -E2BIG;
  if (device >= 0 && config().bar_map) {
    m->bar = hip::bar_map(va, len, &m->bar_va, &m->bar_len);
    if (m->bar) m->hdp = hip::hdp_flush_reg(device);
    STROM_LOG(1, "bar map of %#lx: %s", (unsigned long)va, m->bar ? "yes" : "no");
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    m->handle = ++next_;
    maps_.emplace(m->handle, m);
    gen_.fetch_add(1, std::memory_order_acq_rel);
  }
  out->handle = m->handle;
  out->gpu_page_sz = (uint32_t)STROM_GPU_BOUND_SIZE;
  out->gpu_npages = (uint32_t)npages;
  STROM_LOG(1, "map va=%#lx len=%zu dev=%d handle=%#lx", (unsigned long)va, len, device,
            m->handle);
  return 0;
}

const std::shared_ptr<GpuMapping> &GpuRegistry::get_cached(unsigned long handle) {
  static thread_local struct {
    unsigned long handle = 0;
    uint64_t gen = 0;
    std::shared_ptr<GpuMapping> m;
  } tl;
  // the generation is read before the lookup: a change racing with it
  // leaves the entry one generation old, so the next call looks up again
  const uint64_t gen = gen_.load(std::memory_order_acquire);
  if (tl.handle == handle && tl.gen == gen && tl.m) return tl.m;
  tl.m = get(handle);
  tl.handle = handle;
  tl.gen = gen;
  return tl.m;
}

std::shared_ptr<GpuMapping> GpuRegistry::get(unsigned long handle) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = maps_.find(handle);
  if (it == maps_.end() || it->second->owner != geteuid()) return nullptr;
  return it->second;
}

int GpuRegistry::validate(const std::shared_ptr<GpuMapping> &m) {
  if (!config().check_freed || m->ident == 0) return 0;
  uint64_t now = 0;
  if (m->device >= 0) {
    now = hip::buffer_id(m->va);
    // the range must still end inside the allocation (a smaller one at the
    // same VA has a new id anyway)
  } else {
    VmaInfo v;
    if (vma_query(m->va, &v) == 0 && vma_query(m->va + m->length - 1, &v) == 0) now = 1;
  }
  if (now == m->ident) return 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = maps_.find(m->handle);
    if (it != maps_.end() && it->second == m) maps_.erase(it);
    gen_.fetch_add(1, std::memory_order_acq_rel);
  }
  m->detached = true;
  detached_.fetch_add(1);
  STROM_LOG(0, "mapping %#lx (va %#lx): allocation freed or replaced, detached", m->handle,
            (unsigned long)m->va);
  return -ENOENT;
}

int GpuRegistry::unmap(unsigned long handle) {
  std::shared_ptr<GpuMapping> m;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = maps_.find(handle);
    if (it == maps_.end()) return -ENOENT;
    if (it->second->owner != geteuid()) return -EACCES;
    m = it->second;
    maps_.erase(it);
    gen_.fetch_add(1, std::memory_order_acq_rel);
  }
  // wait for in-flight DMA targeting the range (free-callback semantics);
  // completions notify only while someone drains
  std::unique_lock<std::mutex> g(m->mu);
  m->draining.store(true);  // seq_cst: pairs with the completion's inflight RMW + load
  m->cv.wait(g, [&] { return m->inflight.load() == 0; });
  m->detached = true;
  return 0;
}

int GpuRegistry::list(strom_list_gpu_memory *out) {
  std::lock_guard<std::mutex> g(mu_);
  uint32_t n = 0;
  uid_t me = geteuid();
  for (auto &kv : maps_) {
    if (kv.second->owner != me) continue;
    if (n < out->nrooms) out->handles[n] = kv.first;
    ++n;
  }
  out->nitems = n;
  return 0;
}

int GpuRegistry::info(strom_info_gpu_memory *out) {
  auto m = get(out->handle);
  if (!m) return -ENOENT;
  uint32_t npages =
      (uint32_t)((m->map_length + STROM_GPU_BOUND_SIZE - 1) >> STROM_GPU_BOUND_SHIFT);
  out->nitems = npages;
  out->version = m->version;
  out->gpu_page_sz = (uint32_t)STROM_GPU_BOUND_SIZE;
  out->owner = (uint32_t)m->owner;
  out->map_offset = m->map_offset;
  out->map_length = m->map_length;
  for (uint32_t i = 0; i < npages && i < out->nrooms; ++i)
    out->paddrs[i] = m->base + (uint64_t)i * STROM_GPU_BOUND_SIZE;
  return 0;
}

GpuRegistry &gpu_registry() {
  static GpuRegistry r;
  return r;
}

// ---------------------------------------------------------- DMA buffers
namespace {
constexpr const char kDmaBufName[] = "strom-dmabuf";

// struct procmap_query / PROCMAP_QUERY of <linux/fs.h> (Linux 6.11+), kept
// here so the build does not depend on the installed headers
struct ProcmapQuery {
  uint64_t size, query_flags, query_addr;
  uint64_t vma_start, vma_end, vma_flags, vma_page_size, vma_offset, inode;
  uint32_t dev_major, dev_minor, vma_name_size, build_id_size;
  uint64_t vma_name_addr, build_id_addr;
};
static_assert(sizeof(ProcmapQuery) == 104, "procmap_query layout");
constexpr unsigned long kProcmapQuery = _IOWR('f', 17, ProcmapQuery);

std::atomic<int> g_maps_fd{-2};  // -2 not opened, -1 no PROCMAP_QUERY

int vma_query_scan(uint64_t a, VmaInfo *out) {
  FILE *f = fopen("/proc/self/maps", "r");
  if (!f) return -errno;
  char line[4096];
  int rc = -ENOENT;
  while (fgets(line, sizeof line, f)) {
    unsigned long lo, hi, off, ino;
    unsigned dmaj, dmin;
    char perms[8];
    int pos = 0;
    if (sscanf(line, "%lx-%lx %7s %lx %x:%x %lu %n", &lo, &hi, perms, &off, &dmaj, &dmin, &ino,
               &pos) < 7)
      continue;
    if (a < lo || a >= hi) continue;
    out->start = lo;
    out->end = hi;
    out->pgoff = off;
    out->ino = ino;
    out->dev = makedev(dmaj, dmin);
    out->dmabuf = strstr(line + pos, kDmaBufName) != nullptr;
    rc = 0;
    break;
  }
  fclose(f);
  return rc;
}
}  // namespace

int vma_query(uint64_t addr, VmaInfo *out) {
  int fd = g_maps_fd.load(std::memory_order_acquire);
  if (fd == -2) {
    int nfd = open("/proc/self/maps", O_RDONLY | O_CLOEXEC);
    int expect = -2;
    if (!g_maps_fd.compare_exchange_strong(expect, nfd < 0 ? -1 : nfd)) {
      if (nfd >= 0) close(nfd);
    }
    fd = g_maps_fd.load();
  }
  if (fd >= 0) {
    char name[256];
    ProcmapQuery q{};
    q.size = sizeof q;
    q.query_addr = addr;
    q.vma_name_addr = (uint64_t)name;
    q.vma_name_size = sizeof name;
    if (ioctl(fd, kProcmapQuery, &q) == 0) {
      out->start = q.vma_start;
      out->end = q.vma_end;
      out->pgoff = q.vma_offset;
      out->ino = q.inode;
      out->dev = makedev(q.dev_major, q.dev_minor);
      out->dmabuf = q.vma_name_size > 0 && strstr(name, kDmaBufName) != nullptr;
      return 0;
    }
    if (errno == ENOENT) return -ENOENT;
    if (errno != ENOTTY && errno != EINVAL && errno != EOPNOTSUPP) return -errno;
    // kernel without PROCMAP_QUERY: scan from now on
    int expect = fd;
    if (g_maps_fd.compare_exchange_strong(expect, -1)) close(fd);
  }
  return vma_query_scan(addr, out);
}

int DmaBufRegistry::alloc(size_t length, int node, int *user_fd) {
  if (length == 0) return -EINVAL;
  size_t len = (length + STROM_DMABUF_SEGMENT - 1) / STROM_DMABUF_SEGMENT * STROM_DMABUF_SEGMENT;
  (void)gc();
  char name[64];
  snprintf(name, sizeof name, "%s%d:%zu", kDmaBufName, node, len);
  int fd = (int)syscall(SYS_memfd_create, name, 0u);
  if (fd < 0) return -errno;
  if (ftruncate(fd, (off_t)len) != 0) {
    int e = errno;
    close(fd);
    return -e;
  }
  void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    int e = errno;
    close(fd);
    return -e;
  }
  if (node >= 0) {
    unsigned long mask[16] = {0};
    if (node < 1024) {
      mask[node / 64] = 1ul << (node % 64);
      // shared policy lives in the shmem inode: every mapping inherits it
      if (syscall(SYS_mbind, p, len, MPOL_BIND, mask, 1024ul, 0u) != 0)
        STROM_LOG(1, "mbind(node=%d) failed: %s", node, strerror(errno));
    }
  }
  if (madvise(p, len, MADV_POPULATE_WRITE) != 0) {
    for (size_t off = 0; off < len; off += 4096) ((volatile char *)p)[off] = 0;
  }
  munmap(p, len);  // pages stay with the memfd; the user's fd owns them
  struct stat st;
  fstat(fd, &st);
  auto b = std::make_shared<DmaBuffer>();
  b->dev = st.st_dev;
  b->ino = st.st_ino;
  b->length = len;
  b->node = node;
  {
    std::lock_guard<std::mutex> g(mu_);
    b->gen = next_gen_++;
    bufs_[{b->dev, b->ino}] = b;
  }
  *user_fd = fd;
  return 0;
}

int DmaBufRegistry::resolve(const void *uaddr, size_t len, std::shared_ptr<DmaBuffer> *buf,
                            size_t *offset) {
  const uint64_t a = (uint64_t)uaddr;
  if (a + len < a) return -EINVAL;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = ranges_.upper_bound(a);
    if (it != ranges_.begin()) {
      --it;
      if (a < it->second.end) {
        if (a + len > it->second.end) return -EINVAL;  // crosses the mapping end
        const size_t o = it->second.pgoff + (a - it->first);
        if (o + len > it->second.buf->length) return -EINVAL;
        *buf = it->second.buf;
        *offset = o;
        return 0;
      }
    }
  }
  VmaInfo v;
  int rc = vma_query(a, &v);
  if (rc) return rc == -ENOENT ? -EINVAL : rc;
  if (!v.dmabuf || a + len > v.end) return -EINVAL;  // wrong kind of mapping / crosses its end
  std::lock_guard<std::mutex> g(mu_);
  auto it = bufs_.find({v.dev, (ino_t)v.ino});
  if (it == bufs_.end()) return -EINVAL;
  const size_t o = v.pgoff + (a - v.start);
  if (o + len > it->second->length) return -EINVAL;
  *buf = it->second;
  *offset = o;
  return 0;
}

int DmaBufRegistry::map(int fd, size_t len, void **addr) {
  struct stat st;
  if (fstat(fd, &st) != 0) return -errno;
  std::shared_ptr<DmaBuffer> b;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = bufs_.find({st.st_dev, st.st_ino});
    if (it == bufs_.end()) return -EINVAL;  // not one of ours
    b = it->second;
  }
  if (len == 0 || len > b->length) return -EINVAL;
  void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) return -errno;
  std::lock_guard<std::mutex> g(mu_);
  ranges_[(uint64_t)p] = Range{(uint64_t)p + len, 0, b};
  *addr = p;
  return 0;
}

int DmaBufRegistry::unmap(void *addr, size_t len) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = ranges_.find((uint64_t)addr);
    if (it == ranges_.end() || it->second.end - it->first != len) return -EINVAL;
    ranges_.erase(it);
  }
  return munmap(addr, len) == 0 ? 0 : -errno;
}

int DmaBufRegistry::gc() {
  // Only buffers registered before the /proc snapshot below may be judged
  // by it: one another thread registers while we scan is live but absent
  // from the snapshot (gc erased a buffer allocated concurrently).
  uint64_t before;
  {
    std::lock_guard<std::mutex> g(mu_);
    before = next_gen_;
  }
  // inodes this process still holds: open fds, then mappings
  std::set<std::pair<dev_t, ino_t>> live;
  if (DIR *d = opendir("/proc/self/fd")) {
    while (struct dirent *e = readdir(d)) {
      if (e->d_name[0] == '.') continue;
      char path[16 + sizeof e->d_name], tgt[256];
      snprintf(path, sizeof path, "/proc/self/fd/%s", e->d_name);
      ssize_t n = readlink(path, tgt, sizeof tgt - 1);
      if (n <= 0) continue;
      tgt[n] = 0;
      struct stat st;
      if (strstr(tgt, kDmaBufName) && stat(path, &st) == 0) live.insert({st.st_dev, st.st_ino});
    }
    closedir(d);
  } else {
    std::lock_guard<std::mutex> g(mu_);
    return (int)bufs_.size();  // cannot tell: keep everything
  }
  if (FILE *f = fopen("/proc/self/maps", "r")) {
    char line[4096];
    while (fgets(line, sizeof line, f)) {
      if (!strstr(line, kDmaBufName)) continue;
      unsigned long lo, hi, off, ino;
      unsigned dmaj, dmin;
      char perms[8];
      if (sscanf(line, "%lx-%lx %7s %lx %x:%x %lu", &lo, &hi, perms, &off, &dmaj, &dmin, &ino) == 7)
        live.insert({makedev(dmaj, dmin), (ino_t)ino});
    }
    fclose(f);
  }
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = bufs_.begin(); it != bufs_.end();) {
    if (live.count(it->first) || it->second->gen >= before) ++it;
    else it = bufs_.erase(it);   // in-flight SSD2RAM tasks keep their shared_ptr
  }
  return (int)bufs_.size();
}

size_t DmaBufRegistry::count() {
  std::lock_guard<std::mutex> g(mu_);
  return bufs_.size();
}

DmaBufRegistry &dmabuf_registry() {
  static DmaBufRegistry r;
  return r;
}

}  // namespace strom
