// engine_selftest — host-only exercise of the engine through its C ABI, built
// plain and under ASAN / TSAN (make selftest selftest-asan selftest-tsan).
//
// Covers the concurrency-sensitive paths the reference protected with
// irqsave spinlocks, RCU and refcounts (kmod/nvme_strom.c:648-731,
// 1148-1187): many threads issuing SSD2RAM tasks and waiting on them,
// injected device errors racing with completions, session close reclaiming
// failed tasks, emulated-GPU SSD2GPU with the page-cache hybrid, byte-range
// (extent) reads from several threads, the fake
// backend's out-of-order completions over a stripe set, and engine teardown
// while idle.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "strom/strom.h"

#define CHECK(c)                                                                \
  do {                                                                          \
    if (!(c)) {                                                                 \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);              \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static const uint32_t CH = 8192;

int main() {
  char path[] = "/tmp/strom_selftest.XXXXXX";
  int wfd = mkstemp(path);
  CHECK(wfd >= 0);
  const size_t nch = 512, fsz = nch * CH;
  std::vector<uint8_t> data(fsz);
  std::mt19937_64 rng(1);
  for (auto &b : data) b = (uint8_t)rng();
  CHECK(write(wfd, data.data(), fsz) == (ssize_t)fsz);
  fsync(wfd);
  close(wfd);
  int fd = open(path, O_RDONLY);
  CHECK(fd >= 0);
  strom_evict_file(fd);
  strom_config_set("gpu_emulation", "1");
  strom_config_set("workers", "4");
  strom_engine_reset();

  // DMA buffer
  strom_alloc_dma_buffer ab{};
  ab.length = fsz;
  ab.node_id = -1;
  CHECK(nvme_strom_ioctl(STROM_IOCTL__ALLOC_DMA_BUFFER, &ab) == 0);
  uint8_t *buf = (uint8_t *)mmap(nullptr, fsz, PROT_READ | PROT_WRITE, MAP_SHARED, ab.dmabuf_fdesc, 0);
  CHECK(buf != MAP_FAILED);

  // 1. concurrent SSD2RAM from 8 threads, each its own session + slice
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t) {
    th.emplace_back([&, t] {
      int s = strom_open();
      std::vector<uint32_t> ids(nch / 8);
      for (int rep = 0; rep < 20; ++rep) {
        for (size_t i = 0; i < ids.size(); ++i) ids[i] = (uint32_t)(t * ids.size() + i);
        strom_memcpy_ssd2ram a{};
        a.dest_uaddr = buf + t * ids.size() * CH;
        a.file_desc = fd;
        a.nr_chunks = (unsigned)ids.size();
        a.chunk_sz = CH;
        a.chunk_ids = ids.data();
        if (strom_ioctl(s, STROM_IOCTL__MEMCPY_SSD2RAM, &a) != 0) { bad++; continue; }
        strom_memcpy_wait w{};
        w.dma_task_id = a.dma_task_id;
        if (strom_ioctl(s, STROM_IOCTL__MEMCPY_WAIT, &w) != 0) bad++;
      }
      strom_close(s);
    });
  }
  for (auto &x : th) x.join();
  CHECK(bad == 0);
  CHECK(memcmp(buf, data.data(), fsz) == 0);

  // 2. injected failure on the 7th request, waited from another thread
  strom_config_set("max_request", "8192");
  strom_engine_reset();
  strom_fault_inject(7, EIO, 0, 0, 0);
  {
    int s = strom_open();
    std::vector<uint32_t> ids(64);
    for (int i = 0; i < 64; ++i) ids[i] = i;
    strom_memcpy_ssd2ram a{};
    a.dest_uaddr = buf;
    a.file_desc = fd;
    a.nr_chunks = 64;
    a.chunk_sz = CH;
    a.chunk_ids = ids.data();
    CHECK(strom_ioctl(s, STROM_IOCTL__MEMCPY_SSD2RAM, &a) == 0);
    long status = 0;
    int rc = 0;
    std::thread waiter([&] {
      strom_memcpy_wait w{};
      w.dma_task_id = a.dma_task_id;
      rc = strom_ioctl(s, STROM_IOCTL__MEMCPY_WAIT, &w);
      status = w.status;
    });
    waiter.join();
    CHECK(rc == -EIO && status == -EIO);
    // an unwaited failure is reclaimed by close
    strom_fault_inject(3, EIO, 0, 0, 0);
    CHECK(strom_ioctl(s, STROM_IOCTL__MEMCPY_SSD2RAM, &a) == 0);
    strom_memcpy_wait_timed tw{};
    tw.dma_task_id = a.dma_task_id;
    tw.timeout_ns = 5000000000ull;
    // wait with a deadline on another session: finishes, record stays
    int s2 = strom_open();
    (void)strom_ioctl(s2, STROM_IOCTL__MEMCPY_WAIT_TIMED, &tw);
    strom_close(s2);
    strom_fault_inject(0, 0, 0, 0, 0);
    strom_close(s);
  }

  // 3. emulated SSD2GPU with some chunks cached (RAM tail) from 4 threads
  strom_config_set("max_request", "1048576");
  strom_engine_reset();
  {
    std::vector<uint8_t> hbm(fsz + 65536), wb(fsz);
    uint8_t *dst = (uint8_t *)(((uintptr_t)hbm.data() + 65535) & ~(uintptr_t)65535);
    strom_map_gpu_memory m{};
    m.vaddress = (uint64_t)dst;
    m.length = fsz;
    CHECK(nvme_strom_ioctl(STROM_IOCTL__MAP_GPU_MEMORY, &m) == 0);
    char tmp[CH];
    for (int c : {3, 9, 100}) CHECK(pread(fd, tmp, CH, (off_t)c * CH) == CH);
    std::vector<std::thread> g;
    for (int t = 0; t < 4; ++t) {
      g.emplace_back([&, t] {
        int s = strom_open();
        const size_t per = nch / 4;
        std::vector<uint32_t> ids(per);
        for (size_t i = 0; i < per; ++i) ids[i] = (uint32_t)(t * per + i);
        strom_memcpy_ssd2gpu a{};
        a.handle = m.handle;
        a.offset = t * per * CH;
        a.file_desc = fd;
        a.nr_chunks = (unsigned)per;
        a.chunk_sz = CH;
        a.chunk_ids = ids.data();
        a.wb_buffer = (char *)wb.data() + t * per * CH;
        if (strom_ioctl(s, STROM_IOCTL__MEMCPY_SSD2GPU, &a) != 0) { bad++; return; }
        strom_memcpy_wait w{};
        w.dma_task_id = a.dma_task_id;
        if (strom_ioctl(s, STROM_IOCTL__MEMCPY_WAIT, &w) != 0) bad++;
        // landed order: storage chunks at the head, cached ones at the tail
        for (unsigned i = 0; i < a.nr_ssd2gpu; ++i)
          if (memcmp(dst + (t * per + i) * CH, data.data() + (size_t)ids[i] * CH, CH)) bad++;
        for (unsigned i = a.nr_ssd2gpu; i < per; ++i)
          if (memcmp(wb.data() + (t * per + i) * CH, data.data() + (size_t)ids[i] * CH, CH)) bad++;
        strom_close(s);
      });
    }
    for (auto &x : g) x.join();
    CHECK(bad == 0);
    strom_unmap_gpu_memory um{m.handle};
    CHECK(nvme_strom_ioctl(STROM_IOCTL__UNMAP_GPU_MEMORY, &um) == 0);
  }

  // 4. MEMCPY_SSD2GPU_EXTENTS from 4 threads into emulated HBM: random
  //    sorted extents (some empty, some holes read through), a plan-only call
  //    first for the layout, every landed extent checked against the file
  {
    std::vector<uint8_t> hbm(2 * fsz + 65536);
    uint8_t *dst = (uint8_t *)(((uintptr_t)hbm.data() + 65535) & ~(uintptr_t)65535);
    strom_map_gpu_memory m{};
    m.vaddress = (uint64_t)dst;
    m.length = 2 * fsz;
    CHECK(nvme_strom_ioctl(STROM_IOCTL__MAP_GPU_MEMORY, &m) == 0);
    std::vector<std::thread> g;
    for (int t = 0; t < 4; ++t) {
      g.emplace_back([&, t] {
        int s = strom_open();
        std::mt19937_64 r(100 + t);
        const size_t room = fsz / 2;                     // this thread's destination slice
        for (int rep = 0; rep < 30; ++rep) {
          std::vector<strom_file_extent> x;
          uint64_t pos = r() % 5000;
          while (x.size() < 64 && pos < fsz - 1) {
            strom_file_extent e{};
            e.file_off = pos;
            e.len = (uint32_t)std::min<uint64_t>((r() % 3 == 0) ? 0 : 1 + r() % 40000, fsz - pos);
            x.push_back(e);
            pos += e.len + (r() % 2 ? r() % 64 : r() % 90000);
          }
          strom_memcpy_ssd2gpu_extents a{};
          a.handle = m.handle;
          a.offset = t * room;
          a.file_desc = fd;
          a.nr_extents = (unsigned)x.size();
          a.gap_max = (unsigned)(r() % 2 ? 16384 : 0);
          a.flags = STROM_EXTENTS_PLAN_ONLY;
          a.extents = x.data();
          if (strom_ioctl(s, STROM_IOCTL__MEMCPY_SSD2GPU_EXTENTS, &a) != 0) { bad++; continue; }
          if (a.dst_bytes > room) continue;              // does not fit this slice: skip
          const uint64_t span = a.dst_bytes;
          a.flags = 0;
          if (strom_ioctl(s, STROM_IOCTL__MEMCPY_SSD2GPU_EXTENTS, &a) != 0) { bad++; continue; }
          strom_memcpy_wait w{};
          w.dma_task_id = a.dma_task_id;
          if (strom_ioctl(s, STROM_IOCTL__MEMCPY_WAIT, &w) != 0) bad++;
          if (a.dst_bytes != span) bad++;
          for (const strom_file_extent &e : x)
            if (e.len && memcmp(dst + t * room + e.dst_off, data.data() + e.file_off, e.len)) bad++;
        }
        strom_close(s);
      });
    }
    for (auto &x : g) x.join();
    CHECK(bad == 0);
    strom_unmap_gpu_memory um{m.handle};
    CHECK(nvme_strom_ioctl(STROM_IOCTL__UNMAP_GPU_MEMORY, &um) == 0);
  }

  // 5. fake namespace backend (completions in a seeded random order) under
  //    concurrency, reading a stripe set over two member files: chunk ids
  //    reversed per thread, each thread its own session and buffer slice
  {
    char m0[] = "/tmp/strom_selftest_m0.XXXXXX", m1[] = "/tmp/strom_selftest_m1.XXXXXX";
    int f0 = mkstemp(m0), f1 = mkstemp(m1);
    CHECK(f0 >= 0 && f1 >= 0);
    const uint32_t unit = 4 * CH;
    for (size_t s0 = 0, k = 0; s0 < fsz; s0 += unit, ++k)
      CHECK(write(k % 2 ? f1 : f0, data.data() + s0, unit) == (ssize_t)unit);
    fsync(f0);
    fsync(f1);
    strom_config_set("backend", "fake");
    strom_config_set("max_request", "8192");
    strom_fake_backend(77, nullptr, nullptr);
    strom_engine_reset();
    int mfd[2] = {f0, f1};
    const int sfd = strom_stripe_open(mfd, 2, unit, fsz);
    CHECK(sfd >= 0);
    memset(buf, 0, fsz);
    std::vector<std::thread> g;
    for (int t = 0; t < 4; ++t) {
      g.emplace_back([&, t] {
        int s = strom_open();
        const size_t per = nch / 4;
        std::vector<uint32_t> ids(per);
        for (size_t i = 0; i < per; ++i) ids[i] = (uint32_t)(t * per + per - 1 - i);
        strom_memcpy_ssd2ram a{};
        a.dest_uaddr = buf + t * per * CH;
        a.file_desc = sfd;
        a.nr_chunks = (unsigned)per;
        a.chunk_sz = CH;
        a.chunk_ids = ids.data();
        if (strom_ioctl(s, STROM_IOCTL__MEMCPY_SSD2RAM, &a) != 0) { bad++; return; }
        strom_memcpy_wait w{};
        w.dma_task_id = a.dma_task_id;
        if (strom_ioctl(s, STROM_IOCTL__MEMCPY_WAIT, &w) != 0) bad++;
        for (size_t i = 0; i < per; ++i)
          if (memcmp(buf + (t * per + i) * CH, data.data() + (size_t)ids[i] * CH, CH)) bad++;
        strom_close(s);
      });
    }
    for (auto &x : g) x.join();
    CHECK(bad == 0);
    uint64_t comps = 0, reord = 0;
    strom_fake_backend(0, &comps, &reord);
    CHECK(comps >= nch && reord > 0);
    CHECK(strom_stripe_close(sfd) == 0);
    close(f0);
    close(f1);
    unlink(m0);
    unlink(m1);
    strom_config_set("backend", "uring");
    strom_config_set("max_request", "1048576");
    strom_engine_reset();
  }

  // concurrent ALLOC_DMA_BUFFER: each alloc's gc snapshot must not drop a
  // buffer another thread registered meanwhile (memreg.cc gc)
  {
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 6; t++)
      th.emplace_back([&bad] {
        for (int i = 0; i < 25; i++) {
          strom_alloc_dma_buffer a{};
          a.length = 4096;
          a.node_id = -1;
          if (nvme_strom_ioctl(STROM_IOCTL__ALLOC_DMA_BUFFER, &a) != 0) {
            bad++;
            continue;
          }
          void *m = strom_dmabuf_mmap(a.dmabuf_fdesc, 4096);
          if (!m) bad++;
          else strom_dmabuf_munmap(m, 4096);
          close(a.dmabuf_fdesc);
        }
      });
    for (auto &t : th) t.join();
    CHECK(bad.load() == 0);
  }

  strom_stat_info si{};
  si.version = 1;
  CHECK(nvme_strom_ioctl(STROM_IOCTL__STAT_INFO, &si) == 0);
  CHECK(si.nr_ssd2gpu > 0 && si.cur_dma_count == 0);
  munmap(buf, fsz);
  close(ab.dmabuf_fdesc);
  close(fd);
  unlink(path);
  strom_engine_reset();
  printf("engine_selftest: ok (%llu requests)\n", (unsigned long long)si.nr_ssd2gpu);
  return 0;
}
