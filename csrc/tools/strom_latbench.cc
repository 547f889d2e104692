// strom_latbench — latency of small (4 KiB .. 64 KiB) host → HBM moves on
// MI355X, to pick the mechanism behind the engine's inline 4 KiB path:
//   async+stream   hipMemcpyAsync + hipStreamSynchronize
//   async+event    hipMemcpyAsync + hipEventRecord + hipEventSynchronize
//   sync           hipMemcpy
//   pull-kernel    zero-copy kernel reading pinned host memory + sync
//   dmabuf-mmap    CPU stores into an mmap of the buffer's dma-buf export
//                  (hipMemGetHandleForAddressRange); reported if available
// Also exports the dma-buf (the kmod's import path) and prints whether it works.
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

static double now_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

__global__ void pull(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) d[i] = s[i];
}

template <typename F>
static void run(const char *name, size_t sz, F fn) {
  std::vector<double> t;
  for (int i = 0; i < 1100; ++i) {
    double a = now_us();
    fn();
    if (i >= 100) t.push_back(now_us() - a);
  }
  std::sort(t.begin(), t.end());
  printf("%-14s %6zuB p50=%7.2fus p99=%7.2fus\n", name, sz, t[t.size() / 2], t[t.size() * 99 / 100]);
}

int main() {
  const size_t maxsz = 64 << 10;
  void *h = nullptr, *dh = nullptr, *d = nullptr;
  CK(hipHostMalloc(&h, maxsz, hipHostMallocPortable));
  memset(h, 7, maxsz);
  CK(hipHostGetDevicePointer(&dh, h, 0));
  CK(hipMalloc(&d, 4 << 20));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  int fd = -1;
  hipError_t e = hipMemGetHandleForAddressRange(&fd, (hipDeviceptr_t)d, 4 << 20,
                                                hipMemRangeHandleTypeDmaBufFd, 0);
  printf("dmabuf export: %s fd=%d\n", hipGetErrorString(e), fd);
  void *map = MAP_FAILED;
  if (e == hipSuccess && fd >= 0) {
    map = mmap(nullptr, 4 << 20, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    printf("dmabuf mmap: %s\n", map == MAP_FAILED ? strerror(errno) : "ok");
  }
  for (size_t sz : {(size_t)4096, (size_t)16384, (size_t)65536}) {
    run("async+stream", sz, [&] {
      CK(hipMemcpyAsync(d, h, sz, hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
    });
    run("async+event", sz, [&] {
      CK(hipMemcpyAsync(d, h, sz, hipMemcpyHostToDevice, st));
      CK(hipEventRecord(ev, st));
      CK(hipEventSynchronize(ev));
    });
    run("sync", sz, [&] { CK(hipMemcpy(d, h, sz, hipMemcpyHostToDevice)); });
    run("pull-kernel", sz, [&] {
      hipLaunchKernelGGL(pull, dim3(4), dim3(256), 0, st, (const uint4 *)dh, (uint4 *)d, (uint32_t)(sz / 16));
      CK(hipStreamSynchronize(st));
    });
    if (map != MAP_FAILED) {
      run("dmabuf-mmap", sz, [&] {
        memcpy(map, h, sz);
        __builtin_ia32_sfence();
      });
    }
  }
  if (map != MAP_FAILED) {
    // can the kernel's read paths target the BAR mapping directly?
    char tmpl[] = "/tmp/strom_latbench.XXXXXX";
    int tfd = mkstemp(tmpl);
    std::vector<char> junk(1 << 20, 0x33);
    if (tfd >= 0 && write(tfd, junk.data(), junk.size()) == (ssize_t)junk.size()) {
      fsync(tfd);
      ssize_t r = pread(tfd, map, 1 << 20, 0);
      printf("buffered pread -> BAR map: %zd (%s)\n", r, r < 0 ? strerror(errno) : "ok");
      if (r > 0) {
        run("pread->bar", 65536, [&] { (void)!pread(tfd, map, 65536, 0); });
        run("pread->bar", 1 << 20, [&] { (void)!pread(tfd, map, 1 << 20, 0); });
      }
      int dfd = open(tmpl, O_RDONLY | O_DIRECT);
      if (dfd >= 0) {
        r = pread(dfd, map, 1 << 20, 0);
        printf("O_DIRECT pread -> BAR map: %zd (%s)\n", r, r < 0 ? strerror(errno) : "ok");
        close(dfd);
      }
      close(tfd);
      unlink(tmpl);
    }
    // correctness of the CPU-mapped write as seen by the GPU
    memset(h, 0x5a, 4096);
    memcpy(map, h, 4096);
    __builtin_ia32_sfence();
    std::vector<char> back(4096);
    CK(hipMemcpy(back.data(), d, 4096, hipMemcpyDeviceToHost));
    printf("dmabuf-mmap coherent: %s\n", memcmp(back.data(), h, 4096) == 0 ? "yes" : "NO");
  }
  return 0;
}
