// strom_microbench — isolates the costs of the SSD→HBM bounce path on the
// box it runs on:
//   h2d    : hipMemcpyAsync pinned → HBM with 1..N streams (SDMA or blit)
//   pull   : a GPU kernel reading pinned host memory (zero-copy) into HBM
//   odirect: O_DIRECT pread throughput into different destination kinds
//            (hipHostMalloc, malloc+THP, registered THP) with T threads
// Usage: strom_microbench <file> [threads]
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void pull_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    uint4 a = src[i];
    uint4 b = src[i + stride];
    uint4 c = src[i + 2 * stride];
    uint4 d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

static void *thp_alloc(size_t n) {
  void *p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  madvise(p, n, MADV_HUGEPAGE);
  memset(p, 0, n);
  return p;
}

int main(int argc, char **argv) {
  const char *file = argc > 1 ? argv[1] : nullptr;
  int threads = argc > 2 ? atoi(argv[2]) : 8;
  const size_t N = 1ull << 30;
  void *pin = nullptr, *dev = nullptr;
  CK(hipHostMalloc(&pin, N, hipHostMallocPortable));
  memset(pin, 1, N);
  CK(hipMalloc(&dev, N));
  // ---- h2d with streams
  for (int ns : {1, 2, 4, 8}) {
    for (size_t blk : {(size_t)1 << 20, (size_t)8 << 20, (size_t)64 << 20}) {
      std::vector<hipStream_t> st(ns);
      for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipDeviceSynchronize());
        double t0 = now();
        size_t k = 0;
        for (size_t off = 0; off < N; off += blk, ++k)
          CK(hipMemcpyAsync((char *)dev + off, (char *)pin + off, blk, hipMemcpyHostToDevice, st[k % ns]));
        CK(hipDeviceSynchronize());
        double dt = now() - t0;
        if (rep) printf("h2d streams=%d blk=%zuMiB %.2f GiB/s\n", ns, blk >> 20, 1.0 / dt);
      }
      for (auto &s : st) CK(hipStreamDestroy(s));
    }
  }
  // ---- zero-copy pull kernel
  void *dpin = nullptr;
  CK(hipHostGetDevicePointer(&dpin, pin, 0));
  for (int grid : {256, 1024, 4096}) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      double t0 = now();
      hipLaunchKernelGGL(pull_kernel, dim3(grid), dim3(256), 0, 0, (const uint4 *)dpin, (uint4 *)dev, N / 16);
      CK(hipDeviceSynchronize());
      double dt = now() - t0;
      if (rep) printf("pull grid=%d %.2f GiB/s\n", grid, 1.0 / dt);
    }
  }
  // ---- registered THP memory h2d
  void *thp = thp_alloc(N);
  CK(hipHostRegister(thp, N, hipHostRegisterPortable));
  for (int ns : {1, 4}) {
    std::vector<hipStream_t> st(ns);
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      double t0 = now();
      size_t blk = 8 << 20, k = 0;
      for (size_t off = 0; off < N; off += blk, ++k)
        CK(hipMemcpyAsync((char *)dev + off, (char *)thp + off, blk, hipMemcpyHostToDevice, st[k % ns]));
      CK(hipDeviceSynchronize());
      if (rep) printf("h2d-registered-thp streams=%d %.2f GiB/s\n", ns, 1.0 / (now() - t0));
    }
  }
  if (!file) return 0;
  // ---- O_DIRECT read throughput into buffer kinds
  int fd = open(file, O_RDONLY | O_DIRECT);
  if (fd < 0) {
    perror("open");
    return 1;
  }
  struct stat sb;
  fstat(fd, &sb);
  size_t fsz = (size_t)sb.st_size / N * N;
  if (fsz == 0) fsz = (size_t)sb.st_size & ~((size_t)(4 << 20) - 1);
  void *mal = thp_alloc(N);
  struct Kind { const char *name; char *buf; } kinds[] = {
      {"hipHostMalloc", (char *)pin}, {"malloc-thp", (char *)mal}, {"registered-thp", (char *)thp}};
  for (auto &kd : kinds) {
    for (size_t req : {(size_t)256 << 10, (size_t)1 << 20, (size_t)4 << 20}) {
      for (int T : {1, threads}) {
        size_t total = std::min(fsz, N);
        std::atomic<size_t> next{0};
        double t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
          th.emplace_back([&] {
            for (;;) {
              size_t off = next.fetch_add(req);
              if (off >= total) break;
              ssize_t r = pread(fd, kd.buf + off, req, (off_t)off);
              if (r <= 0) break;
            }
          });
        for (auto &x : th) x.join();
        double dt = now() - t0;
        printf("odirect %-15s req=%4zuKiB threads=%2d %.2f GiB/s\n", kd.name, req >> 10, T,
               total / dt / (1 << 30));
      }
    }
  }
  return 0;
}
