// SPDX-License-Identifier: GPL-2.0
/*
 * strom_io.c — CHECK_FILE, MEMCPY_SSD2GPU / MEMCPY_SSD2RAM, NVMe submission.
 *
 * Same semantics as the userspace engine (csrc/engine/fileplan.cc, the
 * reference's kmod/nvme_strom.c:1299-1981): relseg modulo addressing, the
 * page-cache majority score with dirty pages forcing the RAM path, SSD
 * chunks packed at the head / RAM chunks at the tail with chunk_ids
 * rewritten, merging of contiguous 4 KiB pages up to the device's max
 * transfer, reject of chunks starting at/after EOF (defect #10).
 *
 * Submission: one NVMe READ passthrough request per merged range on the
 * namespace's queue, carrying our own PRP1/PRP2/PRP list built from the
 * dma-buf sg_table (SSD2GPU) or dma_map_page() of the DMA buffer pages
 * (SSD2RAM).  A request with no bio keeps the command's data pointers
 * untouched in nvme_setup_cmd(), so the controller DMAs straight into the
 * BAR.  Completion runs in IRQ/softirq context and puts the task.
 *
 * Needs drivers/nvme/host/nvme.h from the kernel tree (struct nvme_ns,
 * nvme_init_request, nvme_sect_to_lba).  md-raid0 volumes are answered
 * -EOPNOTSUPP here (their members' queues are not reachable without md
 * internals); the userspace engine serves them through the md layer.
 */
#include <linux/dmapool.h>
#include <linux/file.h>
#include <linux/mm.h>
#include <linux/pagemap.h>
#include <linux/slab.h>
#include <linux/uaccess.h>

#include "nvme.h"   /* $(KSRC)/drivers/nvme/host */
#include "strom_kmod.h"

#define NVME_PRP_ENTRIES (NVME_CTRL_PAGE_SIZE / sizeof(__le64))

/* ------------------------------------------------------------ file check */
/*
 * With native NVMe multipath (the default on current distributions) the
 * visible nvmeXnY is a bio-based head disk whose private_data is a struct
 * nvme_ns_head, not a namespace; its paths are blk-mq disks.  A blk-mq disk
 * has no ->submit_bio, which tells the two apart.  For a head the first path
 * on its list is used (nvme_find_path() is not exported).  The path is not
 * pinned: one removed while requests are being built fails them, as hot
 * removal fails any I/O in flight.
 */
static struct nvme_ns *disk_nvme_ns(struct gendisk *disk, int *err)
{
	if (!disk->fops->submit_bio)
		return disk->private_data;
#ifdef CONFIG_NVME_MULTIPATH
	{
		struct nvme_ns_head *head = disk->private_data;
		struct nvme_ns *ns;
		int idx = srcu_read_lock(&head->srcu);

		ns = list_first_or_null_rcu(&head->list, struct nvme_ns, siblings);
		srcu_read_unlock(&head->srcu, idx);
		if (ns)
			return ns;
		*err = -ENODEV;
		return NULL;
	}
#else
	*err = -EOPNOTSUPP;
	return NULL;
#endif
}

static struct nvme_ns *file_nvme_ns(struct file *filp, int *err)
{
	struct inode *inode = file_inode(filp);
	struct super_block *sb = inode->i_sb;
	struct block_device *bdev = sb->s_bdev;
	const char *fs = sb->s_type->name;

	*err = -EOPNOTSUPP;
	if (!S_ISREG(inode->i_mode) && !S_ISDIR(inode->i_mode))
		return NULL;
	if (strcmp(fs, "ext4") && strcmp(fs, "xfs"))
		return NULL;
	if (sb->s_blocksize > PAGE_SIZE)
		return NULL;
	if (!bdev || strncmp(bdev->bd_disk->disk_name, "nvme", 4))
		return NULL;   /* md raid0 / others: userspace engine */
	*err = 0;
	return disk_nvme_ns(bdev->bd_disk, err);
}

int strom_check_file(struct strom_check_file *arg)
{
	struct fd f = fdget(arg->fdesc);
	struct nvme_ns *ns;
	int err;

	if (!f.file)
		return -EBADF;
	if (!(f.file->f_mode & FMODE_READ)) {
		fdput(f);
		return -EBADF;
	}
	ns = file_nvme_ns(f.file, &err);
	if (ns) {
		struct device *dev = ns->ctrl->dev;

		arg->numa_node_id = dev_to_node(dev);
		arg->support_dma64 = dma_get_mask(dev) == DMA_BIT_MASK(64);
		if (i_size_read(file_inode(f.file)) < PAGE_SIZE && S_ISREG(file_inode(f.file)->i_mode))
			err = -EOPNOTSUPP;
	}
	fdput(f);
	return err;
}

/* -------------------------------------------------------- PRP pools */
static DEFINE_MUTEX(pool_lock);
static struct {
	struct device *dev;
	struct dma_pool *pool;
} prp_pools[16];

static struct dma_pool *prp_pool(struct device *dev)
{
	struct dma_pool *p = NULL;
	int i;

	mutex_lock(&pool_lock);
	for (i = 0; i < ARRAY_SIZE(prp_pools); i++) {
		if (prp_pools[i].dev == dev) {
			p = prp_pools[i].pool;
			break;
		}
		if (!prp_pools[i].dev) {
			p = dma_pool_create("strom_prp", dev, NVME_CTRL_PAGE_SIZE,
					    NVME_CTRL_PAGE_SIZE, 0);
			if (p) {
				prp_pools[i].dev = dev;
				prp_pools[i].pool = p;
			}
			break;
		}
	}
	mutex_unlock(&pool_lock);
	return p;
}

/* -------------------------------------------------------- request ctx */
struct strom_req {
	struct strom_task *task;
	struct strom_gpumap *gmap;
	struct dma_pool *pool;
	__le64 *prp_list;
	dma_addr_t prp_dma;
	/* SSD2RAM: pages mapped for the device, unmapped on completion */
	struct device *dev;
	dma_addr_t ram_dma[STROM_MAX_REQ / PAGE_SIZE];
	int nram;
	u64 t0;
	/* /proc/diskstats accounting so P2P reads show in iostat, as the
	 * reference's part_stat_* calls did (kmod/nvme_strom.c:1012-1034) */
	struct block_device *acct_bdev;
	unsigned long acct_start;
	unsigned int acct_sectors;
};

static enum rq_end_io_ret strom_end_io(struct request *rq, blk_status_t err)
{
	struct strom_req *r = rq->end_io_data;
	long status = err ? -EIO : 0;
	int i;

	if (!status && nvme_req(rq)->status)
		status = -EIO;
	atomic64_inc(&strom_stats.nr_ssd2gpu);
	atomic64_add(strom_tsc() - r->t0, &strom_stats.clk_ssd2gpu);
	atomic64_dec(&strom_stats.cur_dma_count);
	bdev_end_io_acct(r->acct_bdev, REQ_OP_READ, r->acct_sectors, r->acct_start);
	if (r->prp_list)
		dma_pool_free(r->pool, r->prp_list, r->prp_dma);
	for (i = 0; i < r->nram; i++)
		dma_unmap_page(r->dev, r->ram_dma[i], PAGE_SIZE, DMA_FROM_DEVICE);
	if (r->gmap && atomic_dec_and_test(&r->gmap->inflight))
		wake_up_all(&r->gmap->drain);
	strom_task_put(r->task, status);
	kfree(r);
	return RQ_END_IO_FREE;
}

/* Fill PRP1/PRP2 (+list) for `len` bytes whose bus addresses come from
 * next_addr(); ranges must be NVME_CTRL_PAGE_SIZE aligned and contiguous
 * within each page. */
static int build_prps(struct strom_req *r, struct nvme_command *c, u32 len,
		      int (*next_addr)(void *ctx, u32 off, dma_addr_t *a), void *ctx)
{
	u32 npages = DIV_ROUND_UP(len, NVME_CTRL_PAGE_SIZE), i;
	dma_addr_t a;
	int rc;

	if (npages > NVME_PRP_ENTRIES + 1)
		return -E2BIG;
	rc = next_addr(ctx, 0, &a);
	if (rc)
		return rc;
	c->rw.dptr.prp1 = cpu_to_le64(a);
	if (npages == 1)
		return 0;
	if (npages == 2) {
		rc = next_addr(ctx, NVME_CTRL_PAGE_SIZE, &a);
		c->rw.dptr.prp2 = cpu_to_le64(a);
		return rc;
	}
	r->prp_list = dma_pool_alloc(r->pool, GFP_KERNEL, &r->prp_dma);
	if (!r->prp_list)
		return -ENOMEM;
	for (i = 1; i < npages; i++) {
		rc = next_addr(ctx, i * NVME_CTRL_PAGE_SIZE, &a);
		if (rc)
			return rc;
		r->prp_list[i - 1] = cpu_to_le64(a);
	}
	c->rw.dptr.prp2 = cpu_to_le64(r->prp_dma);
	return 0;
}

struct gpu_addr_ctx {
	struct strom_gpumap *m;
	struct device *dev;
	size_t base;
};

static int gpu_next_addr(void *p, u32 off, dma_addr_t *a)
{
	struct gpu_addr_ctx *g = p;
	size_t contig;

	return strom_gpumap_dma(g->m, g->dev, g->base + off, a, &contig);
}

struct ram_addr_ctx {
	struct strom_req *r;
	struct vm_area_struct *vma;
	unsigned long uaddr;
};

static int ram_next_addr(void *p, u32 off, dma_addr_t *a)
{
	struct ram_addr_ctx *x = p;
	struct page *pg = strom_dma_buffer_page(x->vma, x->uaddr + off - x->vma->vm_start);

	if (!pg)
		return -EFAULT;
	*a = dma_map_page(x->r->dev, pg, 0, PAGE_SIZE, DMA_FROM_DEVICE);
	if (dma_mapping_error(x->r->dev, *a))
		return -EIO;
	x->r->ram_dma[x->r->nram++] = *a;
	return 0;
}

/* submit one merged READ of `len` bytes at 512-B `sect` */
static int submit_read(struct strom_task *t, struct nvme_ns *ns, sector_t sect, u32 len,
		       struct strom_gpumap *gmap, size_t gpu_off, struct vm_area_struct *vma,
		       unsigned long uaddr)
{
	struct device *dev = ns->ctrl->dev;
	struct nvme_command c = {};
	struct strom_req *r;
	struct request *rq;
	u64 t0 = strom_tsc();
	int rc;

	strom_assert_sleepable();
	r = kzalloc(sizeof(*r), GFP_KERNEL);
	if (!r)
		return -ENOMEM;
	r->task = t;
	r->dev = dev;
	r->pool = prp_pool(dev);
	if (!r->pool) {
		kfree(r);
		return -ENOMEM;
	}
	c.rw.opcode = nvme_cmd_read;
	c.rw.nsid = cpu_to_le32(ns->head->ns_id);
	c.rw.slba = cpu_to_le64(nvme_sect_to_lba(ns->head, sect));
	c.rw.length = cpu_to_le16((len >> ns->head->lba_shift) - 1);
	if (gmap) {
		struct gpu_addr_ctx g = { gmap, dev, gpu_off };

		rc = build_prps(r, &c, len, gpu_next_addr, &g);
	} else {
		struct ram_addr_ctx x = { r, vma, uaddr };

		rc = build_prps(r, &c, len, ram_next_addr, &x);
	}
	atomic64_inc(&strom_stats.nr_setup_prps);
	atomic64_add(strom_tsc() - t0, &strom_stats.clk_setup_prps);
	if (rc)
		goto fail;
	rq = blk_mq_alloc_request(ns->queue, nvme_req_op(&c), 0);
	if (IS_ERR(rq)) {
		rc = PTR_ERR(rq);
		goto fail;
	}
	nvme_init_request(rq, &c);
	rq->timeout = 30 * HZ;
	rq->end_io = strom_end_io;
	rq->end_io_data = r;
	strom_task_get(t);
	if (gmap) {
		r->gmap = gmap;
		atomic_inc(&gmap->inflight);
	}
	strom_stat_inflight_inc();
	r->acct_bdev = ns->disk->part0;
	r->acct_sectors = len >> SECTOR_SHIFT;
	r->acct_start = bdev_start_io_acct(r->acct_bdev, REQ_OP_READ, jiffies);
	r->t0 = strom_tsc();
	blk_execute_rq_nowait(rq, false);
	atomic64_inc(&strom_stats.nr_submit_dma);
	atomic64_add(strom_tsc() - r->t0, &strom_stats.clk_submit_dma);
	return 0;
fail:
	if (r->prp_list)
		dma_pool_free(r->pool, r->prp_list, r->prp_dma);
	while (r->nram--)
		dma_unmap_page(dev, r->ram_dma[r->nram], PAGE_SIZE, DMA_FROM_DEVICE);
	kfree(r);
	return rc;
}

/* ---------------------------------------------------------- the planner */
struct pending {
	sector_t sect;
	u32 len;
	size_t dest;         /* gpu offset or DMA-buffer byte offset */
};

struct copy_ctx {
	struct strom_task *t;
	struct nvme_ns *ns;
	struct inode *inode;
	struct strom_gpumap *gmap;
	struct vm_area_struct *vma;
	unsigned long uaddr_base;
	u32 max_req;
	struct pending cur;
	u32 nr_submit, nr_blocks;
};

static int flush_pending(struct copy_ctx *x)
{
	int rc;

	if (!x->cur.len)
		return 0;
	rc = submit_read(x->t, x->ns, x->cur.sect, x->cur.len, x->gmap, x->cur.dest, x->vma,
			 x->uaddr_base + x->cur.dest);
	x->nr_submit++;
	x->nr_blocks += x->cur.len >> SECTOR_SHIFT;
	x->cur.len = 0;
	return rc;
}

/* map chunk pages [fpos, fpos + len) and merge them into NVMe reads */
static int copy_from_ssd(struct copy_ctx *x, loff_t fpos, u32 len, size_t dest)
{
	struct inode *inode = x->inode;
	unsigned int blkbits = inode->i_blkbits;
	u32 off;
	int rc;

	for (off = 0; off < len; off += PAGE_SIZE) {
		sector_t blk = (fpos + off) >> blkbits;
		sector_t sect;

		rc = bmap(inode, &blk);
		if (rc)
			return rc;
		if (!blk)
			return -EIO;    /* hole / unwritten: not DMA-able */
		sect = (blk << (blkbits - SECTOR_SHIFT)) + get_start_sect(inode->i_sb->s_bdev);
		if (x->cur.len && x->cur.sect + (x->cur.len >> SECTOR_SHIFT) == sect &&
		    x->cur.dest + x->cur.len == dest + off && x->cur.len + PAGE_SIZE <= x->max_req) {
			x->cur.len += PAGE_SIZE;
			continue;
		}
		rc = flush_pending(x);
		if (rc)
			return rc;
		x->cur.sect = sect;
		x->cur.len = PAGE_SIZE;
		x->cur.dest = dest + off;
	}
	return 0;
}

/* page-cache majority score; dirty pages count threshold+1 */
static bool chunk_is_cached(struct address_space *map, pgoff_t first, u32 npages)
{
	u32 threshold = npages / 2, score = 0, i;

	for (i = 0; i < npages; i++) {
		struct folio *f = filemap_get_folio(map, first + i);

		if (IS_ERR_OR_NULL(f))
			continue;
		score += folio_test_dirty(f) ? threshold + 1 : 1;
		folio_put(f);
	}
	return score > threshold;
}

/* buffered read of a cached chunk straight into the user destination
 * (reference memcpy_pgcache_to_ubuffer, kmod/nvme_strom.c:1241-1297).  For
 * SSD2RAM the destination is our own DMA buffer, whose pages are resident
 * (VM_IO, populated at allocation), so the copy cannot fault on mmap_lock. */
static int copy_pgcache_to_user(struct file *filp, loff_t fpos, u32 len, char __user *dst)
{
	loff_t pos = fpos;
	ssize_t n = vfs_read(filp, dst, len, &pos);
	if (n < 0)
		return n;
	if (n < len && clear_user(dst + n, len - n))
		return -EFAULT;
	return 0;
}

int strom_memcpy_ssd2gpu(struct strom_session *s, struct strom_memcpy_ssd2gpu __user *uarg)
{
	struct strom_memcpy_ssd2gpu k;
	struct copy_ctx x = {};
	u32 *ids = NULL, *out = NULL, i, nram = 0, nssd = 0;
	struct strom_gpumap *gmap;
	struct file *filp;
	loff_t isize;
	size_t dest;
	int rc, err;

	if (copy_from_user(&k, uarg, sizeof(k)))
		return -EFAULT;
	if (!k.nr_chunks || (k.chunk_sz & (PAGE_SIZE - 1)) || k.chunk_sz < PAGE_SIZE ||
	    k.chunk_sz > STROM_MAX_REQ)
		return -EINVAL;
	gmap = strom_gpumap_get(k.handle);
	if (!gmap)
		return -ENOENT;
	if (k.offset + (size_t)k.nr_chunks * k.chunk_sz > gmap->length) {
		strom_gpumap_put(gmap);
		return -ERANGE;
	}
	filp = fget(k.file_desc);
	if (!filp) {
		strom_gpumap_put(gmap);
		return -EBADF;
	}
	x.ns = file_nvme_ns(filp, &err);
	if (!x.ns) {
		fput(filp);
		strom_gpumap_put(gmap);
		return err;
	}
	ids = kvmalloc_array(k.nr_chunks, 2 * sizeof(u32), GFP_KERNEL);
	if (!ids) {
		fput(filp);
		strom_gpumap_put(gmap);
		return -ENOMEM;
	}
	out = ids + k.nr_chunks;
	if (copy_from_user(ids, k.chunk_ids, k.nr_chunks * sizeof(u32))) {
		rc = -EFAULT;
		goto out_free;
	}
	x.t = strom_task_create(s, filp, gmap);   /* task owns filp + gmap refs */
	if (!x.t) {
		fput(filp);
		strom_gpumap_put(gmap);
		rc = -ENOMEM;
		goto out_free;
	}
	x.inode = file_inode(filp);
	x.gmap = gmap;
	x.max_req = min_t(u32, STROM_MAX_REQ, queue_max_hw_sectors(x.ns->queue) << SECTOR_SHIFT);
	isize = i_size_read(x.inode);
	dest = k.offset;
	rc = 0;
	for (i = 0; i < k.nr_chunks && !rc; i++) {
		u64 cid = ids[i];
		loff_t fpos = (k.relseg_sz ? cid % k.relseg_sz : cid) * (loff_t)k.chunk_sz;

		if (fpos >= isize) {
			rc = -ERANGE;
			break;
		}
		if (chunk_is_cached(filp->f_mapping, fpos >> PAGE_SHIFT, k.chunk_sz >> PAGE_SHIFT)) {
			nram++;
			out[k.nr_chunks - nram] = cid;
			rc = copy_pgcache_to_user(filp, fpos, k.chunk_sz,
						  k.wb_buffer + (size_t)k.chunk_sz * (k.nr_chunks - nram));
		} else {
			out[nssd++] = cid;
			rc = copy_from_ssd(&x, fpos, k.chunk_sz, dest);
			dest += k.chunk_sz;
		}
	}
	if (!rc)
		rc = flush_pending(&x);
	x.t->frozen = true;
	k.dma_task_id = x.t->id;
	strom_task_put(x.t, rc);
	if (rc) {
		long st;

		strom_task_wait_session(s, k.dma_task_id, &st, MAX_SCHEDULE_TIMEOUT);
		goto out_free;
	}
	k.nr_ram2gpu = nram;
	k.nr_ssd2gpu = nssd;
	k.nr_dma_submit = x.nr_submit;
	k.nr_dma_blocks = x.nr_blocks;
	if (copy_to_user(uarg, &k, offsetof(struct strom_memcpy_ssd2gpu, handle)) ||
	    copy_to_user(k.chunk_ids, out, k.nr_chunks * sizeof(u32)))
		rc = -EFAULT;
out_free:
	kvfree(ids);
	return rc;
}

int strom_memcpy_ssd2ram(struct strom_session *s, struct strom_memcpy_ssd2ram __user *uarg)
{
	struct strom_memcpy_ssd2ram k;
	struct copy_ctx x = {};
	struct vm_area_struct *vma;
	u32 *ids = NULL, i, nram = 0, nssd = 0;
	struct file *filp;
	size_t bytes;
	loff_t isize;
	int rc, err;

	if (copy_from_user(&k, uarg, sizeof(k)))
		return -EFAULT;
	if (!k.nr_chunks || (k.chunk_sz & (PAGE_SIZE - 1)) || k.chunk_sz < PAGE_SIZE ||
	    k.chunk_sz > STROM_MAX_REQ || ((unsigned long)k.dest_uaddr & (PAGE_SIZE - 1)))
		return -EINVAL;
	bytes = (size_t)k.nr_chunks * k.chunk_sz;
	mmap_read_lock(current->mm);
	vma = find_vma(current->mm, (unsigned long)k.dest_uaddr);
	if (!vma || !strom_is_dma_buffer(vma) || (unsigned long)k.dest_uaddr < vma->vm_start ||
	    (unsigned long)k.dest_uaddr + bytes > vma->vm_end) {
		mmap_read_unlock(current->mm);
		return -EINVAL;
	}
	filp = fget(k.file_desc);
	if (!filp) {
		mmap_read_unlock(current->mm);
		return -EBADF;
	}
	x.ns = file_nvme_ns(filp, &err);
	if (!x.ns) {
		fput(filp);
		mmap_read_unlock(current->mm);
		return err;
	}
	ids = kvmalloc_array(k.nr_chunks, sizeof(u32), GFP_KERNEL);
	if (!ids || copy_from_user(ids, k.chunk_ids, k.nr_chunks * sizeof(u32))) {
		rc = ids ? -EFAULT : -ENOMEM;
		fput(filp);
		goto out;
	}
	x.t = strom_task_create(s, filp, NULL);
	if (!x.t) {
		fput(filp);
		rc = -ENOMEM;
		goto out;
	}
	/* the buffer's pages must outlive the DMA even if userspace unmaps
	 * and closes it meanwhile (the reference refcounted its buffers) */
	x.t->dbuf_filp = get_file(vma->vm_file);
	x.inode = file_inode(filp);
	x.vma = vma;
	x.uaddr_base = (unsigned long)k.dest_uaddr;
	x.max_req = min_t(u32, STROM_MAX_REQ, queue_max_hw_sectors(x.ns->queue) << SECTOR_SHIFT);
	isize = i_size_read(x.inode);
	rc = 0;
	for (i = 0; i < k.nr_chunks && !rc; i++) {
		u64 cid = ids[i];
		loff_t fpos = (k.relseg_sz ? cid % k.relseg_sz : cid) * (loff_t)k.chunk_sz;
		size_t dest = (size_t)i * k.chunk_sz;   /* SSD2RAM keeps the order */

		if (fpos >= isize) {
			rc = -ERANGE;
			break;
		}
		if (chunk_is_cached(filp->f_mapping, fpos >> PAGE_SHIFT, k.chunk_sz >> PAGE_SHIFT)) {
			nram++;
			rc = flush_pending(&x);
			if (!rc)
				rc = copy_pgcache_to_user(filp, fpos, k.chunk_sz,
							  (char __user *)k.dest_uaddr + dest);
		} else {
			nssd++;
			rc = copy_from_ssd(&x, fpos, k.chunk_sz, dest);
		}
	}
	if (!rc)
		rc = flush_pending(&x);
	x.t->frozen = true;
	k.dma_task_id = x.t->id;
	strom_task_put(x.t, rc);
	if (rc) {
		long st;

		mmap_read_unlock(current->mm);
		strom_task_wait_session(s, k.dma_task_id, &st, MAX_SCHEDULE_TIMEOUT);
		kvfree(ids);
		return rc;
	}
	k.nr_ram2ram = nram;
	k.nr_ssd2ram = nssd;
	k.nr_dma_submit = x.nr_submit;
	k.nr_dma_blocks = x.nr_blocks;
	if (copy_to_user(uarg, &k, offsetof(struct strom_memcpy_ssd2ram, dest_uaddr)))
		rc = -EFAULT;
out:
	mmap_read_unlock(current->mm);
	kvfree(ids);
	return rc;
}
