// strom_stat — live view of engine statistics (reference utils/nvme_stat.c).
//
//   strom_stat            one dump of every counter (all engine processes)
//   strom_stat <sec>      per-interval means, header every 25 lines
//   strom_stat -p <pid>   one process only
//
// Sources: the kernel provider's STAT_INFO ioctl when /proc|/dev/nvme-strom
// exists, otherwise the userspace engines' shared-memory exports
// (/dev/shm/nvme-strom.<pid>, written by libstrom).  Besides the reference's
// means (clk/nr converted with the measured TSC rate) it prints p50/p99 of
// the per-request latency histograms.
#include <dirent.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <x86intrin.h>

#include <string>
#include <vector>

#include "strom/strom.h"

namespace {

constexpr uint64_t kMagic = 0x53544f524d535431ull;
constexpr int kScalars = 11, kDbg = 8, kB = STROM_HIST_BUCKETS;
constexpr int kWords = kScalars + kDbg + 3 * kB;
constexpr size_t kHdr = 64;

struct Sample {
  uint64_t w[kWords] = {0};
  uint64_t tsc = 0;
  double wall = 0;
  int nproc = 0;
};

double now() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

bool read_shm(int only_pid, Sample *s) {
  DIR *d = opendir("/dev/shm");
  if (!d) return false;
  while (dirent *e = readdir(d)) {
    if (strncmp(e->d_name, "nvme-strom.", 11) != 0) continue;
    int pid = atoi(e->d_name + 11);
    if (only_pid && pid != only_pid) continue;
    if (kill(pid, 0) != 0) continue;  // stale export
    std::string p = std::string("/dev/shm/") + e->d_name;
    int fd = open(p.c_str(), O_RDONLY);
    if (fd < 0) continue;
    size_t len = kHdr + kWords * 8;
    void *m = mmap(nullptr, len, PROT_READ, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) continue;
    if (*(const uint64_t *)m == kMagic) {
      const uint64_t *w = (const uint64_t *)((const char *)m + kHdr);
      for (int i = 0; i < kWords; ++i) {
        // cur/max in-flight are gauges: sum across processes is still meaningful
        s->w[i] += __atomic_load_n(&w[i], __ATOMIC_RELAXED);
      }
      s->nproc++;
    }
    munmap(m, len);
  }
  closedir(d);
  return s->nproc > 0;
}

bool read_kernel(Sample *s) {
  if (strom_provider() != 1) return false;
  strom_stat_info a;
  memset(&a, 0, sizeof a);
  a.version = 1;
  if (nvme_strom_ioctl(STROM_IOCTL__STAT_INFO, &a) != 0) return false;
  uint64_t v[kScalars + kDbg] = {a.nr_ssd2gpu, a.clk_ssd2gpu, a.nr_setup_prps, a.clk_setup_prps,
                                 a.nr_submit_dma, a.clk_submit_dma, a.nr_wait_dtask,
                                 a.clk_wait_dtask, a.nr_wrong_wakeup, a.cur_dma_count,
                                 a.max_dma_count, a.nr_debug1, a.nr_debug2, a.nr_debug3,
                                 a.nr_debug4, a.clk_debug1, a.clk_debug2, a.clk_debug3,
                                 a.clk_debug4};
  memcpy(s->w, v, sizeof v);
  s->nproc = 1;
  return true;
}

bool sample(int pid, Sample *s) {
  *s = Sample();
  s->tsc = __rdtsc();
  s->wall = now();
  return read_kernel(s) || read_shm(pid, s);
}

double pct(const uint64_t *h, double q) {
  uint64_t tot = 0;
  for (int i = 0; i < kB; ++i) tot += h[i];
  if (!tot) return 0;
  double target = q * tot, run = 0;
  for (int i = 0; i < kB; ++i) {
    if (h[i] && run + h[i] >= target) {
      double lo = i ? (double)(1ull << (i - 1)) : 0, hi = (double)(1ull << i);
      return lo + (hi - lo) * (target - run) / h[i];
    }
    run += h[i];
  }
  return (double)(1ull << (kB - 1));
}

const char *names[] = {"ssd2gpu", "setup_prps", "submit_dma", "wait_dtask"};

void dump(const Sample &s, double tsc_hz) {
  printf("processes: %d\n", s.nproc);
  for (int i = 0; i < 4; ++i) {
    uint64_t nr = s.w[2 * i], clk = s.w[2 * i + 1];
    printf("%-12s nr=%-12llu clk=%-16llu avg=%.2fus\n", names[i], (unsigned long long)nr,
           (unsigned long long)clk, nr ? clk / tsc_hz * 1e6 / nr : 0.0);
  }
  printf("wrong_wakeup %llu\ncur_dma      %llu\nmax_dma      %llu\n",
         (unsigned long long)s.w[8], (unsigned long long)s.w[9], (unsigned long long)s.w[10]);
  const char *dbg[4] = {"hbm_copy", "ram_chunk", "resid_probe", "debug4"};
  for (int i = 0; i < 4; ++i)
    printf("%-12s nr=%-12llu clk=%llu\n", dbg[i], (unsigned long long)s.w[11 + i],
           (unsigned long long)s.w[15 + i]);
  const uint64_t *io = s.w + 19, *cp = io + kB, *tk = cp + kB;
  printf("latency(us)  io p50=%.1f p99=%.1f | hbm-copy p50=%.1f p99=%.1f | task p50=%.1f p99=%.1f\n",
         pct(io, .5) / 1e3, pct(io, .99) / 1e3, pct(cp, .5) / 1e3, pct(cp, .99) / 1e3,
         pct(tk, .5) / 1e3, pct(tk, .99) / 1e3);
}

}  // namespace

int main(int argc, char **argv) {
  int pid = 0, interval = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "-p") && i + 1 < argc) pid = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-h")) {
      fprintf(stderr, "usage: %s [-p pid] [interval_sec]\n", argv[0]);
      return 1;
    } else interval = atoi(argv[i]);
  }
  // TSC rate from a short calibration (the reference used dTSC/dwall)
  uint64_t t0 = __rdtsc();
  double w0 = now();
  usleep(50000);
  double tsc_hz = (__rdtsc() - t0) / (now() - w0);
  Sample prev;
  if (!sample(pid, &prev)) {
    fprintf(stderr, "no nvme-strom engine found (kernel provider or /dev/shm/nvme-strom.*)\n");
    return 1;
  }
  if (interval <= 0) {
    dump(prev, tsc_hz);
    return 0;
  }
  for (int line = 0;; ++line) {
    sleep(interval);
    Sample cur;
    if (!sample(pid, &cur)) break;
    if (line % 25 == 0)
      printf("%10s %10s %10s %10s %10s %8s %10s %10s %8s\n", "ssd2gpu/s", "avg-dma", "avg-prps",
             "avg-sub", "avg-wait", "bad-wk", "GiB/s*", "io-p99us", "dma-cur");
    double dt = cur.wall - prev.wall;
    auto mean_us = [&](int i) {
      uint64_t dn = cur.w[2 * i] - prev.w[2 * i], dc = cur.w[2 * i + 1] - prev.w[2 * i + 1];
      return dn ? dc / tsc_hz * 1e6 / dn : 0.0;
    };
    uint64_t dreq = cur.w[0] - prev.w[0];
    uint64_t dhist[kB];
    for (int i = 0; i < kB; ++i) dhist[i] = cur.w[19 + i] - prev.w[19 + i];
    // requests are <= max_request; throughput column is requests * 1 MiB / s as a guide
    printf("%10.0f %9.1fu %9.1fu %9.1fu %9.1fu %8llu %10.2f %10.1f %8llu\n", dreq / dt, mean_us(0),
           mean_us(1), mean_us(2), mean_us(3),
           (unsigned long long)(cur.w[8] - prev.w[8]), dreq / dt / 1024.0, pct(dhist, .99) / 1e3,
           (unsigned long long)cur.w[9]);
    fflush(stdout);
    prev = cur;
  }
  return 0;
}
