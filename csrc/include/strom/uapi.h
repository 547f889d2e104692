/*
 * strom/uapi.h — user/kernel ABI of the MI355X direct-storage engine.
 *
 * Byte-compatible with nvme-strom v0.6's ioctl surface (reference:
 * kmod/nvme_strom.h:17-165): the ten request codes keep their values and
 * every argument block keeps its size and field offsets on x86-64 (the
 * offsets are pinned by the static assertions at the bottom, and again by
 * tests/test_abi.py through ctypes).  Programs written against the
 * reference header compile unchanged against this one via the
 * StromCmd__* typedefs.
 *
 * The same header serves three providers:
 *   - the userspace engine (libstrom.so, `strom_ioctl()`), which runs
 *     without privileges: O_DIRECT reads into pinned staging + SDMA copy
 *     into HBM;
 *   - the kernel module in kmod/ (dma-buf importer of HBM, NVMe reads whose
 *     scatter lists point at the GPU BAR);
 *   - the fake backend used by the CPU test-suite.
 *
 * MI355X additions use fresh request numbers (0x86, 0x87, 0x93, 0x94, 0x9a) so that a
 * reference-era binary never reaches them by accident.
 */
#ifndef STROM_UAPI_H
#define STROM_UAPI_H

#ifdef __KERNEL__
#include <linux/types.h>
#include <linux/ioctl.h>
typedef __u32 strom_u32;
typedef __u64 strom_u64;
#else
#include <stddef.h>
#include <stdint.h>
#include <sys/ioctl.h>
#ifndef __user
#define __user
#endif
typedef uint32_t strom_u32;
typedef uint64_t strom_u64;
#endif

/* ---- request codes (no size/direction encoded, as in v0.6) ---------- */
#define STROM_IOC_MAGIC 'S'
#define STROM_IOCTL__CHECK_FILE         _IO(STROM_IOC_MAGIC, 0x80)
#define STROM_IOCTL__MAP_GPU_MEMORY     _IO(STROM_IOC_MAGIC, 0x81)
#define STROM_IOCTL__UNMAP_GPU_MEMORY   _IO(STROM_IOC_MAGIC, 0x82)
#define STROM_IOCTL__LIST_GPU_MEMORY    _IO(STROM_IOC_MAGIC, 0x83)
#define STROM_IOCTL__INFO_GPU_MEMORY    _IO(STROM_IOC_MAGIC, 0x84)
#define STROM_IOCTL__ALLOC_DMA_BUFFER   _IO(STROM_IOC_MAGIC, 0x85)
#define STROM_IOCTL__MEMCPY_SSD2GPU     _IO(STROM_IOC_MAGIC, 0x90)
#define STROM_IOCTL__MEMCPY_SSD2RAM     _IO(STROM_IOC_MAGIC, 0x91)
#define STROM_IOCTL__MEMCPY_WAIT        _IO(STROM_IOC_MAGIC, 0x92)
#define STROM_IOCTL__STAT_INFO          _IO(STROM_IOC_MAGIC, 0x99)
/* MI355X extensions */
#define STROM_IOCTL__MAP_GPU_DMABUF     _IO(STROM_IOC_MAGIC, 0x86)
#define STROM_IOCTL__MEMCPY_WAIT_TIMED  _IO(STROM_IOC_MAGIC, 0x93)
#define STROM_IOCTL__STAT_HIST          _IO(STROM_IOC_MAGIC, 0x9a)
#define STROM_IOCTL__SET_ROUTE          _IO(STROM_IOC_MAGIC, 0x87)
#define STROM_IOCTL__MEMCPY_SSD2GPU_EXTENTS _IO(STROM_IOC_MAGIC, 0x94)

/* Kernel provider entry points.  /proc keeps v0.6 compatibility; /dev is
 * what the MI355X kmod registers as a misc device. */
#define NVME_STROM_IOCTL_PATHNAME  "/proc/nvme-strom"
#define STROM_DEVICE_PATHNAME      "/dev/nvme-strom"

/* Limits shared by every provider. */
#define STROM_GPU_BOUND_SHIFT      16                 /* 64 KiB map granule */
#define STROM_GPU_BOUND_SIZE       (1UL << STROM_GPU_BOUND_SHIFT)
#define STROM_LEGACY_MAX_REQUEST   (128U << 10)       /* v0.6 MDTS guess */
#define STROM_DMABUF_SEGMENT       (4UL << 20)        /* DMA-buffer segment */

/* ---- CHECK_FILE ----------------------------------------------------- */
struct strom_check_file {
	int fdesc;          /* in:  file to classify */
	int numa_node_id;   /* out: node of the backing device, -1 if mixed */
	int support_dma64;  /* out: nonzero when SSD2RAM may target any page */
};

/* ---- MAP / UNMAP / LIST / INFO GPU memory --------------------------- */
struct strom_map_gpu_memory {
	unsigned long handle;      /* out */
	strom_u32     gpu_page_sz; /* out */
	strom_u32     gpu_npages;  /* out */
	strom_u64     vaddress;    /* in:  device VA (hipMalloc'd HBM) */
	size_t        length;      /* in */
};

struct strom_unmap_gpu_memory {
	unsigned long handle;      /* in */
};

struct strom_list_gpu_memory {
	strom_u32     nrooms;      /* in:  capacity of handles[] */
	strom_u32     nitems;      /* out: total live mappings of the caller */
	unsigned long handles[1];  /* out: flexible tail */
};

struct strom_info_gpu_memory {
	unsigned long handle;      /* in */
	strom_u32     nrooms;      /* in:  capacity of paddrs[] */
	strom_u32     nitems;      /* out: number of GPU pages */
	strom_u32     version;     /* out: page-table generation */
	strom_u32     gpu_page_sz; /* out */
	strom_u32     owner;       /* out: euid of the mapper */
	unsigned long map_offset;  /* out: VA - aligned base */
	unsigned long map_length;  /* out */
	strom_u64     paddrs[1];   /* out: per-page bus/device addresses */
};

/* MI355X: register HBM exported as a dma-buf (hipMemGetHandleForAddressRange
 * with hipMemRangeHandleTypeDmaBufFd).  The kmod imports it and DMAs into
 * the sg_table's bus addresses; the userspace engine records the VA. */
struct strom_map_gpu_dmabuf {
	unsigned long handle;      /* out */
	strom_u32     gpu_page_sz; /* out */
	strom_u32     gpu_npages;  /* out */
	int           dmabuf_fd;   /* in */
	int           device_id;   /* in:  HIP ordinal (informational) */
	strom_u64     vaddress;    /* in:  device VA of the mapped range */
	size_t        length;      /* in */
	strom_u64     dmabuf_offset; /* in: byte offset of vaddress inside the dma-buf */
};

/* ---- MEMCPY_SSD2GPU ------------------------------------------------- */
struct strom_memcpy_ssd2gpu {
	unsigned long dma_task_id;   /* out */
	unsigned int  nr_ram2gpu;    /* out: chunks served from page cache */
	unsigned int  nr_ssd2gpu;    /* out: chunks read from storage */
	unsigned int  nr_dma_submit; /* out: storage requests issued */
	unsigned int  nr_dma_blocks; /* out: 512-B sectors requested */
	unsigned long handle;        /* in:  GPU mapping */
	size_t        offset;        /* in:  byte offset inside the mapping */
	int           file_desc;     /* in */
	unsigned int  nr_chunks;     /* in */
	unsigned int  chunk_sz;      /* in */
	unsigned int  relseg_sz;     /* in:  chunks per segment file, 0 = none */
	strom_u32 __user *chunk_ids; /* in/out: rewritten to landing order */
	char __user  *wb_buffer;     /* in:  page-cache chunks land at its tail */
};

/* ---- MEMCPY_SSD2GPU_EXTENTS (MI355X) --------------------------------
 * Exact reads of a list of byte ranges (an Arrow scan's column buffers)
 * instead of fixed-size chunk ids: extents sorted by file offset and
 * disjoint; each is widened to whole 4 KiB pages, and an extent starting
 * within gap_max bytes of the previous one's last page is read in the same
 * run (the hole with it).  Runs land back to back from `offset`, an extent
 * at the same distance from its run's start as in the file: dst_off says
 * where.  Runs split into requests of at most the provider's request size.
 * Every byte comes from storage (O_DIRECT / NVMe READ after the range's
 * dirty page-cache pages were written back): no reordering.  bytes_read =
 * the extents' bytes + gap_bytes (holes and page padding).  flags
 * STROM_EXTENTS_PLAN_ONLY: fill the outputs, read nothing (handle unused):
 * how a caller sizes its destination. */
#define STROM_EXTENTS_PLAN_ONLY 1u
struct strom_file_extent {
	strom_u64 file_off;          /* in */
	strom_u64 dst_off;           /* out: bytes from `offset` */
	strom_u32 len;               /* in */
	strom_u32 reserved;
};

struct strom_memcpy_ssd2gpu_extents {
	unsigned long dma_task_id;   /* out */
	unsigned int  nr_dma_submit; /* out: storage requests issued */
	unsigned int  nr_dma_blocks; /* out: 512-B sectors requested */
	strom_u64     bytes_read;    /* out */
	strom_u64     gap_bytes;     /* out: bytes_read - the extents' bytes */
	strom_u64     dst_bytes;     /* out: destination span used from offset */
	unsigned long handle;        /* in:  GPU mapping */
	size_t        offset;        /* in:  byte offset inside the mapping */
	int           file_desc;     /* in */
	unsigned int  nr_extents;    /* in */
	unsigned int  gap_max;       /* in:  bytes of hole worth reading through */
	unsigned int  flags;         /* in:  STROM_EXTENTS_* */
	struct strom_file_extent __user *extents;  /* in/out */
};

/* ---- MEMCPY_WAIT ---------------------------------------------------- */
struct strom_memcpy_wait {
	unsigned long dma_task_id;   /* in */
	long          status;        /* out: first device error, 0 if none */
};

/* MI355X: WAIT with a deadline; returns -ETIME when it expires. */
struct strom_memcpy_wait_timed {
	unsigned long dma_task_id;   /* in */
	long          status;        /* out */
	strom_u64     timeout_ns;    /* in:  0 = poll */
};

/* ---- MEMCPY_SSD2RAM ------------------------------------------------- */
struct strom_memcpy_ssd2ram {
	unsigned long dma_task_id;   /* out */
	unsigned int  nr_ram2ram;    /* out */
	unsigned int  nr_ssd2ram;    /* out */
	unsigned int  nr_dma_submit; /* out */
	unsigned int  nr_dma_blocks; /* out */
	void __user  *dest_uaddr;    /* in:  inside an ALLOC_DMA_BUFFER mapping */
	int           file_desc;     /* in */
	unsigned int  nr_chunks;     /* in */
	unsigned int  chunk_sz;      /* in */
	unsigned int  relseg_sz;     /* in */
	strom_u32 __user *chunk_ids; /* in:  chunk i lands at dest + i*chunk_sz */
};

/* ---- ALLOC_DMA_BUFFER ----------------------------------------------- */
struct strom_alloc_dma_buffer {
	size_t length;        /* in */
	int    node_id;       /* in:  NUMA node, -1 = local */
	int    dmabuf_fdesc;  /* out: mmap(MAP_SHARED) this fd */
};

/* ---- STAT_INFO (version 1 layout) ----------------------------------- */
struct strom_stat_info {
	unsigned int  version;     /* in:  must be 1 */
	unsigned char has_debug;   /* out */
	strom_u64 tsc;             /* out: time-stamp counter at sampling */
	strom_u64 nr_ssd2gpu;      /* completed storage requests */
	strom_u64 clk_ssd2gpu;     /*   submit -> completion, TSC cycles */
	strom_u64 nr_setup_prps;   /* request builds (PRP/SGL or staging) */
	strom_u64 clk_setup_prps;
	strom_u64 nr_submit_dma;   /* submissions to the backend */
	strom_u64 clk_submit_dma;
	strom_u64 nr_wait_dtask;   /* WAIT calls that slept */
	strom_u64 clk_wait_dtask;
	strom_u64 nr_wrong_wakeup;
	strom_u64 cur_dma_count;   /* requests in flight now */
	strom_u64 max_dma_count;   /* high-water mark, reset on read */
	strom_u64 nr_debug1;       /* debug1: staging -> HBM copies */
	strom_u64 clk_debug1;
	strom_u64 nr_debug2;       /* debug2: page-cache (RAM) chunks */
	strom_u64 clk_debug2;
	strom_u64 nr_debug3;       /* debug3: residency probes */
	strom_u64 clk_debug3;
	strom_u64 nr_debug4;       /* debug4: bytes moved (nr) / reserved */
	strom_u64 clk_debug4;
};

/* MI355X: per-request latency histograms, log2(ns) buckets. */
#define STROM_HIST_BUCKETS 48
struct strom_stat_hist {
	unsigned int version;          /* in:  must be 1 */
	unsigned int reset;            /* in:  nonzero clears after copy-out */
	strom_u64 io_ns[STROM_HIST_BUCKETS];    /* submit -> storage done */
	strom_u64 copy_ns[STROM_HIST_BUCKETS];  /* storage done -> in HBM */
	strom_u64 task_ns[STROM_HIST_BUCKETS];  /* ioctl entry -> task done */
};

/* ---- SET_ROUTE (MI355X, kernel provider, CAP_SYS_ADMIN) --------------
 * How the kernel provider reaches the NVMe namespaces behind a volume it
 * cannot decode without md/nvme private structures: an md raid0 array
 * (geometry + members, reference kmod/nvme_strom.c:755-820) or a native
 * multipath head (one member: the path namespace to submit on).  Userspace
 * derives it from sysfs (nvme_strom_amd/utils/route.py); the module checks
 * the geometry (strom_core_raid0_check), the members' sizes against it and
 * that every member is an NVMe namespace with a blk-mq queue.  nmembers == 0
 * removes the volume's route. */
#define STROM_ROUTE_MAX_ZONES  16
#define STROM_ROUTE_MAX_DISKS  32
struct strom_set_route {
	strom_u32 volume_major;     /* in: md array / nvme head block device */
	strom_u32 volume_minor;
	strom_u32 nmembers;         /* in: 0 = drop the route */
	strom_u32 chunk_sects;      /* in: raid0 stripe chunk (sectors); 0 = single path */
	strom_u32 nzones;
	strom_u32 reserved;
	strom_u64 zone_end[STROM_ROUTE_MAX_ZONES];        /* md sector, exclusive */
	strom_u64 zone_dev_start[STROM_ROUTE_MAX_ZONES];  /* member sector of zone start */
	strom_u32 zone_nb_dev[STROM_ROUTE_MAX_ZONES];
	unsigned char zone_devs[STROM_ROUTE_MAX_ZONES][STROM_ROUTE_MAX_DISKS];
	strom_u32 member_major[STROM_ROUTE_MAX_DISKS];
	strom_u32 member_minor[STROM_ROUTE_MAX_DISKS];
	strom_u64 data_offset[STROM_ROUTE_MAX_DISKS];     /* sectors */
	/* a member with major 0 is named instead, "<pci>/<ctrl>/<disk>", e.g.
	 * "0000:41:00.0/nvme0/nvme0c0n1": the hidden path disk of a multipath
	 * namespace, which has no openable dev_t */
	char member_name[STROM_ROUTE_MAX_DISKS][40];
};

/* ---- v0.6 source-compatible names ----------------------------------- */
typedef struct strom_check_file        StromCmd__CheckFile;
typedef struct strom_map_gpu_memory    StromCmd__MapGpuMemory;
typedef struct strom_unmap_gpu_memory  StromCmd__UnmapGpuMemory;
typedef struct strom_list_gpu_memory   StromCmd__ListGpuMemory;
typedef struct strom_info_gpu_memory   StromCmd__InfoGpuMemory;
typedef struct strom_memcpy_ssd2gpu    StromCmd__MemCopySsdToGpu;
typedef struct strom_memcpy_wait       StromCmd__MemCopyWait;
typedef struct strom_memcpy_ssd2ram    StromCmd__MemCopySsdToRam;
typedef struct strom_alloc_dma_buffer  StromCmd__AllocDMABuffer;
typedef struct strom_stat_info         StromCmd__StatInfo;

/* ---- layout pins (x86-64 LP64) -------------------------------------- */
#if !defined(__KERNEL__) && defined(__x86_64__)
#ifdef __cplusplus
#define STROM_ASSERT(c, m) static_assert(c, m)
#else
#define STROM_ASSERT(c, m) _Static_assert(c, m)
#endif
STROM_ASSERT(sizeof(struct strom_check_file) == 12, "CheckFile");
STROM_ASSERT(sizeof(struct strom_map_gpu_memory) == 32, "MapGpuMemory");
STROM_ASSERT(offsetof(struct strom_map_gpu_memory, vaddress) == 16, "Map.va");
STROM_ASSERT(offsetof(struct strom_map_gpu_memory, length) == 24, "Map.len");
STROM_ASSERT(sizeof(struct strom_unmap_gpu_memory) == 8, "Unmap");
STROM_ASSERT(sizeof(struct strom_list_gpu_memory) == 16, "List");
STROM_ASSERT(offsetof(struct strom_list_gpu_memory, handles) == 8, "List.h");
STROM_ASSERT(sizeof(struct strom_info_gpu_memory) == 56, "Info");
STROM_ASSERT(offsetof(struct strom_info_gpu_memory, map_offset) == 32, "Info.off");
STROM_ASSERT(offsetof(struct strom_info_gpu_memory, paddrs) == 48, "Info.pa");
STROM_ASSERT(sizeof(struct strom_memcpy_ssd2gpu) == 72, "SsdToGpu");
STROM_ASSERT(offsetof(struct strom_memcpy_ssd2gpu, handle) == 24, "S2G.handle");
STROM_ASSERT(offsetof(struct strom_memcpy_ssd2gpu, offset) == 32, "S2G.offset");
STROM_ASSERT(offsetof(struct strom_memcpy_ssd2gpu, file_desc) == 40, "S2G.fd");
STROM_ASSERT(offsetof(struct strom_memcpy_ssd2gpu, chunk_ids) == 56, "S2G.ids");
STROM_ASSERT(offsetof(struct strom_memcpy_ssd2gpu, wb_buffer) == 64, "S2G.wb");
STROM_ASSERT(sizeof(struct strom_memcpy_wait) == 16, "Wait");
STROM_ASSERT(sizeof(struct strom_memcpy_ssd2ram) == 56, "SsdToRam");
STROM_ASSERT(offsetof(struct strom_memcpy_ssd2ram, dest_uaddr) == 24, "S2R.dest");
STROM_ASSERT(offsetof(struct strom_memcpy_ssd2ram, chunk_ids) == 48, "S2R.ids");
STROM_ASSERT(sizeof(struct strom_alloc_dma_buffer) == 16, "AllocDMABuffer");
STROM_ASSERT(sizeof(struct strom_stat_info) == 168, "StatInfo");
STROM_ASSERT(offsetof(struct strom_stat_info, tsc) == 8, "Stat.tsc");
STROM_ASSERT(offsetof(struct strom_stat_info, nr_debug1) == 104, "Stat.dbg1");
STROM_ASSERT(sizeof(struct strom_set_route) == 2648, "SetRoute");
STROM_ASSERT(sizeof(struct strom_file_extent) == 24, "FileExtent");
STROM_ASSERT(sizeof(struct strom_memcpy_ssd2gpu_extents) == 80, "SsdToGpuExtents");
STROM_ASSERT(offsetof(struct strom_memcpy_ssd2gpu_extents, handle) == 40, "S2GX.handle");
STROM_ASSERT(offsetof(struct strom_memcpy_ssd2gpu_extents, extents) == 72, "S2GX.ext");
STROM_ASSERT(offsetof(struct strom_set_route, zone_devs) == 344, "Route.devs");
STROM_ASSERT(STROM_IOCTL__CHECK_FILE == 0x5380, "code");
STROM_ASSERT(STROM_IOCTL__MEMCPY_SSD2GPU == 0x5390, "code");
STROM_ASSERT(STROM_IOCTL__STAT_INFO == 0x5399, "code");
#undef STROM_ASSERT
#endif

#endif /* STROM_UAPI_H */
