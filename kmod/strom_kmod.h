/* SPDX-License-Identifier: GPL-2.0 */
/*
 * strom_kmod.h — internals of the MI355X nvme-strom kernel provider.
 *
 * True SSD -> HBM peer-to-peer: HBM is imported as a dma-buf exported by
 * amdgpu (userspace: hipMemGetHandleForAddressRange(.., DmaBufFd, ..)), the
 * attachment is made for the NVMe controller's PCI device with
 * allow_peer2peer, pinned, and mapped; the resulting sg_table carries
 * IOMMU-correct bus addresses of the VRAM pages behind the large BAR, and
 * those addresses go straight into NVMe READ PRP lists.  No
 * nvidia_p2p_get_pages, no raw physical addresses (reference defect #8), no
 * kallsyms lookups (unexported since 5.7): file extents come from bmap(),
 * NVMe commands are passthrough requests on the namespace's blk-mq queue.
 *
 * Kernel interface: Linux >= 6.8, EXPORTED interfaces only — no private
 * drivers/nvme or drivers/md headers (the reference vendored RHEL7 copies of
 * nvme.h / md.h / raid0.h, kmod/514.6.2.el7/).  What those headers gave the
 * reference is obtained here as follows:
 *   namespace id       the disk's own NVME_IOCTL_ID ioctl (as the reference's
 *                      CHECK_FILE ping did)
 *   LBA size           queue_logical_block_size()
 *   DMA device         the nearest PCI ancestor of the disk's struct device
 *   command setup      nvme_init_request() — EXPORT_SYMBOL_GPL of nvme-core;
 *                      its prototype is declared below (checked against a
 *                      kernel tree by kmod/kernel-check.sh)
 *   multipath paths    a hidden path disk (nvmeXcYnZ) is found by name under
 *                      its controller with device_find_child_by_name()
 *   md raid0 geometry  registered by userspace (STROM_IOCTL__SET_ROUTE,
 *                      CAP_SYS_ADMIN) from sysfs and checked here
 * The one piece of NVMe state read from a completed request is the
 * blk_status_t handed to end_io (nvme_end_req translates the NVMe status).
 *
 * Version gates (LINUX_VERSION_CODE) exist only where an API moved inside
 * [6.8, 6.18]: MODULE_IMPORT_NS takes a string literal from 6.13, block
 * devices are opened with bdev_file_open_by_dev() from 6.9 (bdev_open_by_dev()
 * handles in 6.8), and struct fd is read through fd_file() from 6.12.
 */
#ifndef STROM_KMOD_H
#define STROM_KMOD_H

#include <linux/atomic.h>
#include <linux/blk-mq.h>
#include <linux/blkdev.h>
#include <linux/dma-buf.h>
#include <linux/fs.h>
#include <linux/kref.h>
#include <linux/list.h>
#include <linux/mutex.h>
#include <linux/nvme.h>
#include <linux/spinlock.h>
#include <linux/types.h>
#include <linux/version.h>
#include <linux/wait.h>
#include <linux/workqueue.h>

#include "strom/uapi.h"       /* -I$(src)/include (DKMS) or ../csrc/include (tree) */
#include "strom_core.h"

#if LINUX_VERSION_CODE < KERNEL_VERSION(6, 8, 0)
#error "nvme-strom (MI355X) needs Linux >= 6.8"
#endif
#if LINUX_VERSION_CODE < KERNEL_VERSION(6, 12, 0)
#define fd_file(f) ((f).file)          /* accessor introduced in 6.12 */
#endif

#define STROM_NAME "nvme-strom"
#define STROM_NR_TASK_SLOTS 512
#define STROM_NR_MAP_SLOTS 64
#define STROM_MAX_ATTACH 8               /* NVMe controllers per HBM mapping */

/* nvme-core, EXPORT_SYMBOL_GPL (drivers/nvme/host/core.c); declared in the
 * private drivers/nvme/host/nvme.h, so declared here */
void nvme_init_request(struct request *req, struct nvme_command *cmd);

extern int strom_verbose;
extern int strom_stat_level;

#define prDebug(fmt, ...)                                                      \
	do {                                                                   \
		if (strom_verbose > 1)                                         \
			pr_info("nvme-strom: %s:%d " fmt "\n", __func__,       \
				__LINE__, ##__VA_ARGS__);                      \
		else if (strom_verbose)                                        \
			pr_info("nvme-strom: " fmt "\n", ##__VA_ARGS__);       \
	} while (0)

/* invariant checks: panic in debug builds like the reference's Assert(),
 * warn once otherwise */
#ifdef STROM_DEBUG
#define STROM_ASSERT(c) BUG_ON(!(c))
#define strom_assert_sleepable() might_sleep()
#else
#define STROM_ASSERT(c) WARN_ON_ONCE(!(c))
#define strom_assert_sleepable() do { } while (0)
#endif

/* ---- per-open-file session (strom_proc_release reclaims failures) ---- */
struct strom_session {
	struct list_head failed;         /* strom_task records nobody waited */
	spinlock_t lock;
	struct file *filp;               /* the /dev or /proc file: every task
	                                    pins it, so release() (and kfree of
	                                    the session) follows the last
	                                    completion */
};

/* ---- NVMe namespaces behind a volume ------------------------------------ */
struct strom_member {
	struct device *disk_dev;         /* held (get_device) */
	struct gendisk *disk;            /* blk-mq namespace (path) disk */
	struct request_queue *q;
	struct device *dma_dev;          /* the controller's PCI function (held) */
	u32 nsid;
	u32 lba_shift;
	u32 max_bytes;                   /* queue_max_hw_sectors, bytes */
	sector_t nr_sects;               /* capacity */
	struct dma_pool *prp_pool;
};

struct strom_volume {
	struct kref ref;
	struct work_struct free_work;    /* members are released in process context */
	struct list_head node;           /* route table (registered volumes) */
	dev_t devt;                      /* md array / nvme head / plain namespace */
	u64 diskseq;                     /* unregistered: the disk instance cached */
	bool registered;
	bool raid0;
	struct strom_raid0 geo;
	int nmembers;
	struct strom_member m[STROM_ROUTE_MAX_DISKS];
};

/* The volume under a file: its route when registered, else the file's own
 * disk when that is a blk-mq NVMe namespace.  Reference held. */
struct strom_volume *strom_volume_of_file(struct file *filp, int *err);
void strom_volume_put(struct strom_volume *v);
int strom_set_route(const struct strom_set_route *r);
int strom_route_init(void);
void strom_route_exit(void);

/* ---- HBM mapping: imported dma-buf ------------------------------------ */
struct strom_attach {                    /* one per NVMe controller device */
	struct device *dev;
	struct dma_buf_attachment *att;
	struct sg_table *sgt;
	/* the sg table flattened once (strom_core_sg_lookup searches it) */
	u32 nsegs;
	u64 *seg_addr, *seg_len, *seg_start;
};

struct strom_gpumap {
	struct hlist_node node;
	unsigned long handle;
	kuid_t owner;
	struct dma_buf *dmabuf;
	u64 vaddress;                    /* user VA of the mapped range */
	u64 dmabuf_off;                  /* byte offset of vaddress in the dma-buf */
	size_t length;
	struct strom_attach att[STROM_MAX_ATTACH];   /* lazily per controller */
	int natt;
	struct mutex att_lock;
	atomic_t inflight;               /* requests targeting the range */
	wait_queue_head_t drain;
	struct kref ref;
	struct work_struct free_work;    /* teardown sleeps: never in IRQ */
};

int strom_map_dmabuf(struct strom_map_gpu_dmabuf *arg);
int strom_unmap_gpu(unsigned long handle);
int strom_list_gpu(struct strom_list_gpu_memory __user *uarg);
int strom_info_gpu(struct strom_info_gpu_memory __user *uarg);
struct strom_gpumap *strom_gpumap_get(unsigned long handle);
void strom_gpumap_put(struct strom_gpumap *m);
/* bus addresses of the dma-buf as seen by `dev` (attach + pin + map once per
 * controller): *sg maps byte offsets of the WHOLE dma-buf, so a destination
 * offset inside the mapped range is looked up at dmabuf_off + offset */
int strom_gpumap_sgmap(struct strom_gpumap *m, struct device *dev, struct strom_sgmap *sg);
int strom_gpumap_init(void);
void strom_gpumap_exit(void);

/* ---- DMA task table ---------------------------------------------------- */
struct strom_task {
	struct hlist_node node;          /* running slot */
	struct list_head failed_node;    /* session failed list */
	unsigned long id;
	struct strom_session *sess;
	atomic_t refcnt;                 /* 1 submitter + 1 per request */
	long status;                     /* first error wins */
	bool frozen;
	struct strom_gpumap *gmap;       /* SSD2GPU target (ref held) */
	struct file *filp;               /* source (ref held) */
	struct file *dbuf_filp;          /* SSD2RAM destination buffer (ref held) */
	struct strom_volume *vol;        /* namespaces the requests go to (ref held) */
	u64 t_start;
};

struct strom_task *strom_task_create(struct strom_session *s, struct file *filp,
				     struct strom_gpumap *gmap);
void strom_task_get(struct strom_task *t);
void strom_task_put(struct strom_task *t, long status);
int strom_task_wait(unsigned long id, long *status, long timeout_jiffies);
/* WAIT as seen by userspace: also consumes the failed record (-EIO+status) */
int strom_task_wait_session(struct strom_session *s, unsigned long id, long *status,
			    long timeout_jiffies);
int strom_session_reclaim(struct strom_session *s);
void strom_task_init(void);

/* ---- I/O --------------------------------------------------------------- */
int strom_check_file(struct strom_check_file *arg);
int strom_memcpy_ssd2gpu(struct strom_session *s,
			 struct strom_memcpy_ssd2gpu __user *uarg);
int strom_memcpy_ssd2ram(struct strom_session *s,
			 struct strom_memcpy_ssd2ram __user *uarg);
int strom_memcpy_ssd2gpu_extents(struct strom_session *s,
				 struct strom_memcpy_ssd2gpu_extents __user *uarg);

/* ---- DMA buffers (anon inode) -------------------------------------------- */
int strom_alloc_dma_buffer(struct strom_alloc_dma_buffer *arg);
bool strom_is_dma_buffer(struct vm_area_struct *vma);
struct page *strom_dma_buffer_page(struct vm_area_struct *vma, unsigned long off);
struct strom_dbuf_map;
struct strom_dbuf_map *strom_dma_buffer_map(struct file *filp, struct device *dev);
int strom_dma_buffer_addr(struct file *filp, const struct strom_dbuf_map *m, u64 off, u64 *addr,
			  u64 *contig);
void strom_dma_buffer_sync_for_cpu(struct file *filp, const struct strom_dbuf_map *m, u64 off,
				   u64 len);

/* ---- statistics ---------------------------------------------------------- */
struct strom_stats {
	atomic64_t nr_ssd2gpu, clk_ssd2gpu;
	atomic64_t nr_setup_prps, clk_setup_prps;
	atomic64_t nr_submit_dma, clk_submit_dma;
	atomic64_t nr_wait_dtask, clk_wait_dtask;
	atomic64_t nr_wrong_wakeup;
	atomic64_t cur_dma_count, max_dma_count;
	atomic64_t nr_debug[4], clk_debug[4];
};
extern struct strom_stats strom_stats;
int strom_stat_info(struct strom_stat_info *arg);
void strom_stat_inflight_inc(void);

static inline u64 strom_tsc(void)
{
	return rdtsc_ordered();
}

#endif /* STROM_KMOD_H */
