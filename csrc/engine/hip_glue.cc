// hip_glue.cc — the few HIP runtime services the engine needs.
//
// Everything here is lazy: the engine runs (SSD2RAM, planning, the fake
// backend) on machines without a GPU, and only touches the HIP runtime
// when a request targets HBM.  Pinned staging is allocated under the
// calling thread's NUMA policy (hipHostMallocNumaUser), which the I/O
// workers set to the node of the GPU's PCIe root before allocating.
#include <hip/hip_runtime_api.h>  // host API only: builds with g++ (sanitizers)
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <errno.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>
#include <x86intrin.h>

#include <cctype>
#include <map>
#include <mutex>
#include <string>

#include "engine.h"

namespace strom {
namespace hip {

static int g_count = -2;
static std::once_flag g_once;

static void probe() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  g_count = n;
}

bool available() {
  std::call_once(g_once, probe);
  return g_count > 0;
}

int device_count() {
  std::call_once(g_once, probe);
  return g_count;
}

int pointer_device(uint64_t va, uint64_t *alloc_base, size_t *alloc_size) {
  hipPointerAttribute_t attr;
  memset(&attr, 0, sizeof attr);
  if (hipPointerGetAttributes(&attr, (void *)va) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  if (attr.type != hipMemoryTypeDevice) return -1;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)va) == hipSuccess) {
    *alloc_base = (uint64_t)base;
    *alloc_size = size;
  } else {
    (void)hipGetLastError();
  }
  return attr.device;
}

// `coherent`: fine-grained, so that GPU reads (the ingest grid) never hit
// stale cached lines when the CPU refills the buffer
void *host_alloc(size_t bytes, bool coherent) {
  void *p = nullptr;
  const unsigned cf = coherent ? hipHostMallocCoherent : 0u;
  if (hipHostMalloc(&p, bytes, hipHostMallocPortable | hipHostMallocNumaUser | cf) != hipSuccess) {
    (void)hipGetLastError();
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable | cf) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
  }
  return p;
}

void host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

// Staging for O_DIRECT reads: anonymous memory backed by transparent huge
// pages, then registered (pinned + GPU-mapped).  Measured on MI355X hosts:
// O_DIRECT into 2 MiB pages costs the kernel far less page pinning than
// into hipHostMalloc's 4 KiB pages (single-thread 19-20 vs 14 GiB/s), and
// SDMA reads it at the same ~50 GiB/s.
void *host_alloc_thp(size_t bytes, bool uncached) {
  const size_t huge = 2u << 20;
  size_t len = (bytes + huge - 1) / huge * huge;
  void *raw = mmap(nullptr, len + huge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (raw == MAP_FAILED) return nullptr;
  uintptr_t a = ((uintptr_t)raw + huge - 1) & ~(uintptr_t)(huge - 1);
  if (a > (uintptr_t)raw) munmap(raw, a - (uintptr_t)raw);
  size_t tail = (uintptr_t)raw + len + huge - (a + len);
  if (tail) munmap((void *)(a + len), tail);
  void *p = (void *)a;
  madvise(p, len, MADV_HUGEPAGE);
  memset(p, 0, len);  // fault in (under the caller's NUMA policy)
  // uncached for the GPU: the ingest grid reads each slot again after the
  // CPU refilled it, and must not be served a stale L2 copy
  const unsigned fl = hipHostRegisterPortable | (uncached ? hipExtHostRegisterUncached : 0u);
  if (hipHostRegister(p, len, fl) != hipSuccess) {
    (void)hipGetLastError();
    munmap(p, len);
    return nullptr;
  }
  return p;
}

void host_free_thp(void *p, size_t bytes) {
  if (!p) return;
  const size_t huge = 2u << 20;
  size_t len = (bytes + huge - 1) / huge * huge;
  (void)hipHostUnregister(p);
  munmap(p, len);
}

// CPU mapping of the page-aligned cover of [va, va+len): the WHOLE
// allocation holding it is exported (allocators sub-allocate inside larger
// blocks) and the cover is mapped at its offset inside the export.
static uint8_t *map_cover(uint64_t va, size_t len, uint64_t *map_va, size_t *map_len,
                          double *export_ms, double *mmap_ms) {
  const uint64_t page = 4096;
  hipDeviceptr_t abase = nullptr;
  size_t asize = 0;
  if (hipMemGetAddressRange(&abase, &asize, (hipDeviceptr_t)va) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  const uint64_t base = (uint64_t)abase;
  const uint64_t lo = va & ~(page - 1);
  const uint64_t hi = (va + len + page - 1) & ~(page - 1);
  if (lo < base || hi > base + ((asize + page - 1) & ~(page - 1))) return nullptr;
  int fd = -1;
  const uint64_t t0 = mono_ns();
  if (hipMemGetHandleForAddressRange(&fd, abase, asize, hipMemRangeHandleTypeDmaBufFd, 0) !=
          hipSuccess ||
      fd < 0) {
    (void)hipGetLastError();
    return nullptr;
  }
  const uint64_t t1 = mono_ns();
  void *p = mmap(nullptr, hi - lo, PROT_READ | PROT_WRITE, MAP_SHARED, fd, (off_t)(lo - base));
  close(fd);  // the mapping keeps the dma-buf alive
  if (p == MAP_FAILED) return nullptr;
  if (export_ms) *export_ms = (t1 - t0) / 1e6;
  if (mmap_ms) *mmap_ms = (mono_ns() - t1) / 1e6;
  *map_va = lo;
  *map_len = hi - lo;
  return (uint8_t *)p;
}

// The CPU alias of HBM through a dma-buf mmap needs a large BAR (or the
// driver falls back to something the GPU does not see).  Checked ONCE per
// device on a private allocation — never by storing into a user's live
// tensor, which kernels on other streams may be using.
static bool bar_alias_ok(int device) {
  static std::mutex mu;
  static std::map<int, bool> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  bool ok = false;
  int cur = -1;
  (void)hipGetDevice(&cur);
  void *probe = nullptr;
  const size_t len = 2u << 20;
  if (hipSetDevice(device) == hipSuccess && hipMalloc(&probe, len) == hipSuccess) {
    uint64_t mva = 0;
    size_t mlen = 0;
    const uint64_t at = (uint64_t)probe + 4096;
    if (uint8_t *p = map_cover(at, 8, &mva, &mlen, nullptr, nullptr)) {
      const uint64_t canary = 0x5354524f4d424152ull ^ at;
      uint64_t back = 0;
      volatile uint64_t *q = (volatile uint64_t *)(p + (at - mva));
      *q = canary;
      _mm_sfence();
      (void)*q;  // drains the posted write
      ok = hipMemcpy(&back, (void *)at, 8, hipMemcpyDeviceToHost) == hipSuccess && back == canary;
      munmap(p, mlen);
    }
    (void)hipFree(probe);
  }
  (void)hipGetLastError();
  if (cur >= 0) (void)hipSetDevice(cur);
  STROM_LOG(ok ? 1 : 0, "device %d: BAR alias of HBM %s", device, ok ? "verified" : "unusable");
  cache[device] = ok;
  return ok;
}

uint8_t *bar_map(uint64_t va, size_t len, uint64_t *map_va, size_t *map_len) {
  hipPointerAttribute_t attr;
  memset(&attr, 0, sizeof attr);
  if (hipPointerGetAttributes(&attr, (void *)va) != hipSuccess || attr.type != hipMemoryTypeDevice) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (!bar_alias_ok(attr.device)) return nullptr;
  double ex = 0, mm = 0;
  uint8_t *p = map_cover(va, len, map_va, map_len, &ex, &mm);
  if (p) STROM_LOG(1, "bar_map %zu KiB: export %.2f ms, mmap %.2f ms", *map_len >> 10, ex, mm);
  return p;
}

uint64_t buffer_id(uint64_t va) {
  unsigned long long id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)va) !=
      hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (uint64_t)id;
}

namespace {
struct HdpFind {
  uint32_t domain, bdf;
  volatile uint32_t *reg;
};
hsa_status_t hdp_agent_cb(hsa_agent_t a, void *p) {
  auto *f = (HdpFind *)p;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS ||
      t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, dom = 0;
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
  if (bdf != f->bdf || dom != f->domain) return HSA_STATUS_SUCCESS;
  hsa_amd_hdp_flush_t h{};
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &h) == HSA_STATUS_SUCCESS)
    f->reg = h.HDP_MEM_FLUSH_CNTL;
  return HSA_STATUS_INFO_BREAK;
}
}  // namespace

// The HSA agent of a HIP device is found by PCI location (HIP and HSA may
// order devices differently); hsa_init is reference counted and HIP has
// already initialised the runtime.
volatile uint32_t *hdp_flush_reg(int device) {
  static std::mutex mu;
  static std::map<int, volatile uint32_t *> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  volatile uint32_t *reg = nullptr;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) == hipSuccess && hsa_init() == HSA_STATUS_SUCCESS) {
    HdpFind f{(uint32_t)p.pciDomainID, ((uint32_t)p.pciBusID << 8) | ((uint32_t)p.pciDeviceID << 3),
              nullptr};
    (void)hsa_iterate_agents(hdp_agent_cb, &f);
    reg = f.reg;
  } else {
    (void)hipGetLastError();
  }
  STROM_LOG(1, "device %d: HDP flush register %p", device, (void *)reg);
  cache[device] = reg;
  return reg;
}

void bar_unmap(uint8_t *p, size_t len) {
  if (p) munmap(p, len);
}

int export_dmabuf(uint64_t va, size_t len, int *fd, uint64_t *offset, int *device) {
  uint64_t base = 0;
  size_t size = 0;
  *device = pointer_device(va, &base, &size);
  if (*device < 0 || size == 0) return -EINVAL;
  if (va + len > base + size) return -ERANGE;
  *fd = -1;
  if (hipMemGetHandleForAddressRange(fd, (hipDeviceptr_t)base, size, hipMemRangeHandleTypeDmaBufFd,
                                     hipMemRangeFlagDmaBufMappingTypePcie) != hipSuccess ||
      *fd < 0) {
    (void)hipGetLastError();
    *fd = -1;
    if (hipMemGetHandleForAddressRange(fd, (hipDeviceptr_t)base, size,
                                       hipMemRangeHandleTypeDmaBufFd, 0) != hipSuccess ||
        *fd < 0) {
      (void)hipGetLastError();
      return -EOPNOTSUPP;
    }
  }
  *offset = va - base;
  return 0;
}

int copy_dtoh(void *dst, uint64_t src, size_t len) {
  return hipMemcpy(dst, (const void *)src, len, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -EIO;
}

int copy_htod(uint64_t dst, const void *src, size_t len) {
  return hipMemcpy((void *)dst, src, len, hipMemcpyHostToDevice) == hipSuccess ? 0 : -EIO;
}

int numa_node_of_device(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  for (char *c = bus; *c; ++c) *c = (char)tolower(*c);
  std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
  FILE *f = fopen(path.c_str(), "r");
  if (!f) return -1;
  int node = -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  return node;
}

}  // namespace hip
}  // namespace strom

extern "C" int strom_gpu_count(void) { return strom::hip::device_count(); }

extern "C" int strom_gpu_pci_bdf(int device, char *buf, size_t len) {
  if (!strom::hip::available()) return -ENODEV;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return -ENODEV;
  }
  for (char *c = bus; *c; ++c) *c = (char)tolower(*c);
  snprintf(buf, len, "%s", bus);
  return 0;
}

