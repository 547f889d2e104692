// ssd2ram_test — SSD → NUMA-local DMA buffer benchmark
// (the reference's utils/ssd2ram_test.c, re-designed; same options).
//
//   ssd2ram_test [-n threads] [-s buffer_MiB] [-u unit_KiB] [-b chunk_KiB] [-c] [-p] FILE
//
//   -c  verify every unit against pread (the reference's check was a TODO)
//   -p  print the CHECK_FILE answer and exit
//
// CHECK_FILE gives the device's NUMA node; the process binds to that node's
// CPUs, allocates the DMA buffer there (ALLOC_DMA_BUFFER + mmap) and each
// thread claims file units with an atomic cursor, issuing MEMCPY_SSD2RAM
// into its own ring slots and WAITing when a slot is reused.  Ring indices
// start at zero (reference defect #4: they were uninitialised).
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "strom/strom.h"

static double now() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void bind_node(int node) {
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!(f >> list)) return;
  cpu_set_t want, allowed, use;
  CPU_ZERO(&want);
  size_t pos = 0;
  while (pos <= list.size()) {
    size_t c = list.find(',', pos);
    std::string part = list.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
    int a, b;
    if (sscanf(part.c_str(), "%d-%d", &a, &b) == 2)
      for (int i = a; i <= b && i < CPU_SETSIZE; ++i) CPU_SET(i, &want);
    else if (sscanf(part.c_str(), "%d", &a) == 1 && a < CPU_SETSIZE)
      CPU_SET(a, &want);
    if (c == std::string::npos) break;
    pos = c + 1;
  }
  sched_getaffinity(0, sizeof allowed, &allowed);
  CPU_AND(&use, &want, &allowed);
  if (CPU_COUNT(&use)) sched_setaffinity(0, sizeof use, &use);
}

int main(int argc, char **argv) {
  int nthreads = 4;
  size_t buf_mib = 32, unit_kib = 1024, chunk_kib = 8;
  bool check = false, print = false;
  int opt;
  while ((opt = getopt(argc, argv, "n:s:u:b:cp")) != -1) {
    switch (opt) {
      case 'n': nthreads = atoi(optarg); break;
      case 's': buf_mib = strtoul(optarg, nullptr, 0); break;
      case 'u': unit_kib = strtoul(optarg, nullptr, 0); break;
      case 'b': chunk_kib = strtoul(optarg, nullptr, 0); break;
      case 'c': check = true; break;
      case 'p': print = true; break;
      default:
        fprintf(stderr, "usage: %s [-n threads] [-s buffer_MiB] [-u unit_KiB] [-b chunk_KiB] [-c] [-p] FILE\n",
                argv[0]);
        return 1;
    }
  }
  if (optind >= argc) {
    fprintf(stderr, "missing FILE\n");
    return 1;
  }
  const char *path = argv[optind];
  int fd = open(path, O_RDONLY);
  if (fd < 0) {
    perror(path);
    return 1;
  }
  struct stat sb;
  fstat(fd, &sb);
  const size_t fsize = (size_t)sb.st_size, unit = unit_kib << 10, chunk = chunk_kib << 10;
  strom_check_file cf{};
  cf.fdesc = fd;
  if (nvme_strom_ioctl(STROM_IOCTL__CHECK_FILE, &cf) != 0) {
    perror("CHECK_FILE");
    return 1;
  }
  if (print) {
    printf("file: %s numa_node_id: %d support_dma64: %d\n", path, cf.numa_node_id, cf.support_dma64);
    return 0;
  }
  if (!cf.support_dma64) {
    fprintf(stderr, "device does not support 64-bit DMA: SSD2RAM unavailable\n");
    return 1;
  }
  if (cf.numa_node_id >= 0) bind_node(cf.numa_node_id);
  const size_t per_thread = std::max(unit, (buf_mib << 20) / nthreads / unit * unit);
  const int slots = (int)(per_thread / unit);
  strom_alloc_dma_buffer ab{};
  ab.length = per_thread * nthreads;
  ab.node_id = cf.numa_node_id;
  if (nvme_strom_ioctl(STROM_IOCTL__ALLOC_DMA_BUFFER, &ab) != 0) {
    perror("ALLOC_DMA_BUFFER");
    return 1;
  }
  // mapped through the engine: SSD2RAM then finds the destination in the
  // registry's address index instead of querying the VMA per call
  char *buf = (char *)strom_dmabuf_mmap(ab.dmabuf_fdesc, ab.length);
  if (!buf) {
    perror("strom_dmabuf_mmap");
    return 1;
  }
  std::atomic<size_t> cursor{0};
  std::atomic<uint64_t> nr_ram{0}, nr_ssd{0}, nr_submit{0}, nr_blocks{0}, bad{0};
  std::atomic<int> failed{0};
  std::vector<double> waits(nthreads, 0.0);
  double t0 = now();
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([&, t] {
      struct Pend {
        unsigned long task;
        size_t pos, len;
        bool busy;
      };
      std::vector<Pend> ring(slots, Pend{0, 0, 0, false});
      std::vector<uint32_t> ids(unit / chunk);
      std::vector<char> ref(check ? unit : 0);
      int windex = 0;
      auto retire = [&](int s) {
        if (!ring[s].busy) return;
        double w0 = now();
        strom_memcpy_wait w{};
        w.dma_task_id = ring[s].task;
        if (nvme_strom_ioctl(STROM_IOCTL__MEMCPY_WAIT, &w) != 0) {
          fprintf(stderr, "MEMCPY_WAIT: %s status=%ld\n", strerror(errno), w.status);
          failed = 1;
        }
        waits[t] += now() - w0;
        if (check) {
          char *d = buf + ((size_t)t * slots + s) * unit;
          ssize_t got = pread(fd, ref.data(), ring[s].len, (off_t)ring[s].pos);
          if (got != (ssize_t)ring[s].len || memcmp(ref.data(), d, ring[s].len) != 0) bad++;
        }
        ring[s].busy = false;
      };
      for (;;) {
        size_t pos = cursor.fetch_add(unit);
        if (pos >= fsize || failed) break;
        int s = windex % slots;
        retire(s);
        size_t len = std::min(unit, fsize - pos);
        uint32_t n = (uint32_t)((len + chunk - 1) / chunk);
        for (uint32_t i = 0; i < n; ++i) ids[i] = (uint32_t)(pos / chunk + i);
        strom_memcpy_ssd2ram a{};
        a.dest_uaddr = buf + ((size_t)t * slots + s) * unit;
        a.file_desc = fd;
        a.nr_chunks = n;
        a.chunk_sz = (unsigned)chunk;
        a.chunk_ids = ids.data();
        if (nvme_strom_ioctl(STROM_IOCTL__MEMCPY_SSD2RAM, &a) != 0) {
          perror("MEMCPY_SSD2RAM");
          failed = 1;
          break;
        }
        nr_ram += a.nr_ram2ram;
        nr_ssd += a.nr_ssd2ram;
        nr_submit += a.nr_dma_submit;
        nr_blocks += a.nr_dma_blocks;
        ring[s] = Pend{a.dma_task_id, pos, len, true};
        ++windex;
      }
      for (int s = 0; s < slots; ++s) retire(s);
    });
  }
  for (auto &x : th) x.join();
  double dt = now() - t0, wsum = 0;
  for (double w : waits) wsum += w;
  printf("file: %s, read: %zu MB, time: %.3f sec, throughput: %.2f GB/s (%.2f GiB/s)\n", path,
         fsize >> 20, dt, fsize / dt / 1e9, fsize / dt / (1 << 30));
  printf("threads: %d, buffer: %zu MiB on node %d, unit: %zu KiB, chunk: %zu KiB, wait: %.3f sec\n",
         nthreads, (size_t)(ab.length >> 20), cf.numa_node_id, unit_kib, chunk_kib, wsum / nthreads);
  printf("nr_ram2ram: %llu, nr_ssd2ram: %llu, average DMA size: %.1f KB\n",
         (unsigned long long)nr_ram.load(), (unsigned long long)nr_ssd.load(),
         nr_submit ? 0.5 * nr_blocks.load() / nr_submit.load() : 0.0);
  if (check) printf("verify: %llu corrupted unit(s)\n", (unsigned long long)bad.load());
  return failed || bad ? 2 : 0;
}
