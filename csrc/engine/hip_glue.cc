// hip_glue.cc — the few HIP runtime services the engine needs.
//
// Everything here is lazy: the engine runs (SSD2RAM, planning, the fake
// backend) on machines without a GPU, and only touches the HIP runtime
// when a request targets HBM.  Pinned staging is allocated under the
// calling thread's NUMA policy (hipHostMallocNumaUser), which the I/O
// workers set to the node of the GPU's PCIe root before allocating.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <cctype>
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

void *host_alloc(size_t bytes) {
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocPortable | hipHostMallocNumaUser) != hipSuccess) {
    (void)hipGetLastError();
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
  }
  return p;
}

void host_free(void *p) {
  if (p) (void)hipHostFree(p);
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
