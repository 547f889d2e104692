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
 * NVMe commands are passthrough requests on the namespace queue.
 *
 * Status: written against Linux 6.8+ APIs (ns_id / lba_shift live in
 * struct nvme_ns_head since 6.8); compile-untested in this repo's
 * environment (no kernel headers, no root on the GPU pool).  Build with
 * KSRC pointing at a configured kernel tree (drivers/nvme/host/nvme.h is
 * needed for struct nvme_ns and nvme_init_request()).
 */
#ifndef STROM_KMOD_H
#define STROM_KMOD_H

#include <linux/atomic.h>
#include <linux/blkdev.h>
#include <linux/dma-buf.h>
#include <linux/fs.h>
#include <linux/kref.h>
#include <linux/list.h>
#include <linux/mutex.h>
#include <linux/spinlock.h>
#include <linux/types.h>
#include <linux/wait.h>
#include <linux/workqueue.h>

#include "../csrc/include/strom/uapi.h"

#define STROM_NAME "nvme-strom"
#define STROM_MAX_REQ (1U << 20)         /* merge limit, clamped by MDTS */
#define STROM_NR_TASK_SLOTS 512
#define STROM_NR_MAP_SLOTS 64

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

/* ---- HBM mapping: imported dma-buf ------------------------------------ */
struct strom_attach {                    /* one per NVMe controller device */
	struct device *dev;
	struct dma_buf_attachment *att;
	struct sg_table *sgt;
};

struct strom_gpumap {
	struct hlist_node node;
	unsigned long handle;
	kuid_t owner;
	struct dma_buf *dmabuf;
	u64 vaddress;                    /* user VA of the mapped range */
	u64 dmabuf_off;                  /* byte offset of vaddress in the dma-buf */
	size_t length;
	struct strom_attach att[4];      /* lazily per target controller */
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
/* bus address of byte `off` of the mapping as seen by `dev`, and how many
 * contiguous bytes follow it */
int strom_gpumap_dma(struct strom_gpumap *m, struct device *dev, size_t off,
		     dma_addr_t *addr, size_t *contig);
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

/* ---- DMA buffers (anon inode) -------------------------------------------- */
int strom_alloc_dma_buffer(struct strom_alloc_dma_buffer *arg);
bool strom_is_dma_buffer(struct vm_area_struct *vma);
struct page *strom_dma_buffer_page(struct vm_area_struct *vma, unsigned long off);

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
