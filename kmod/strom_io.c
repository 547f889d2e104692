// SPDX-License-Identifier: GPL-2.0
/*
 * strom_io.c — CHECK_FILE, MEMCPY_SSD2GPU / MEMCPY_SSD2RAM, NVMe submission.
 *
 * Every decision is the shared core's (strom_core.c, unit-tested on the CPU
 * by tests/test_kmod_core_cpu.py, and the same code the userspace engine
 * plans with): chunk position + EOF rule, page-cache majority score (dirty
 * pages force the RAM path), landing order (storage chunks from the head,
 * cached chunks from the tail, chunk_ids rewritten), the bmap-extent merge
 * up to the members' max transfer, the raid0 remap, and PRP1/PRP2/list
 * construction from the flattened dma-buf sg table.  Reference:
 * kmod/nvme_strom.c:1299-1981.
 *
 * Submission: one NVMe READ passthrough request per merged range on the
 * member namespace's blk-mq queue, with our own PRPs; a request without a
 * bio keeps the command's data pointers untouched, so the controller DMAs
 * straight into the BAR (SSD2GPU) or the DMA buffer pages (SSD2RAM).  The
 * command lives in the request context until completion (nvme_init_request
 * keeps a pointer to it).  Completion runs in IRQ/softirq context and puts
 * the task.
 *
 * MI355X extension (as the userspace provider): SSD2GPU with wb_buffer ==
 * NULL still lands page-cache chunks at the tail and counts them in
 * nr_ram2gpu, but moves them by DMA after writing their dirty pages back
 * (the device then holds exactly the page cache's bytes).
 */
#include <linux/dmapool.h>
#include <linux/file.h>
#include <linux/highmem.h>
#include <linux/mm.h>
#include <linux/pagemap.h>
#include <linux/slab.h>
#include <linux/uaccess.h>

#include "strom_kmod.h"

#ifndef __LITTLE_ENDIAN
#error "PRP lists are written as host u64: little-endian only"
#endif

#define STROM_MAX_CHUNKS (1u << 24)

/* ------------------------------------------------------------ file check */
static int fs_supported(struct file *filp)
{
	struct inode *inode = file_inode(filp);
	const char *fs = inode->i_sb->s_type->name;

	if (!(filp->f_mode & FMODE_READ))
		return -EBADF;
	if (!S_ISREG(inode->i_mode) && !S_ISDIR(inode->i_mode))
		return -EOPNOTSUPP;
	if (strcmp(fs, "ext4") && strcmp(fs, "xfs"))
		return -EOPNOTSUPP;
	if (inode->i_sb->s_blocksize > PAGE_SIZE)
		return -EOPNOTSUPP;
	if (S_ISREG(inode->i_mode) && i_size_read(inode) < PAGE_SIZE)
		return -EOPNOTSUPP;
	return 0;
}

int strom_check_file(struct strom_check_file *arg)
{
	struct fd f = fdget(arg->fdesc);
	struct strom_volume *v;
	int err, i, node = NUMA_NO_NODE;
	bool dma64 = true;

	if (!fd_file(f))
		return -EBADF;
	err = fs_supported(fd_file(f));
	if (err)
		goto out;
	v = strom_volume_of_file(fd_file(f), &err);
	if (!v)
		goto out;
	/* -1 when the members span NUMA nodes (reference :249-261) */
	for (i = 0; i < v->nmembers; i++) {
		int n = dev_to_node(v->m[i].dma_dev);

		node = i == 0 ? n : (n == node ? node : -1);
		dma64 &= dma_get_mask(v->m[i].dma_dev) == DMA_BIT_MASK(64);
	}
	arg->numa_node_id = node;
	arg->support_dma64 = dma64;
	strom_volume_put(v);
out:
	fdput(f);
	return err;
}

/* -------------------------------------------------------- request ctx */
struct strom_req {
	struct nvme_command cmd;       /* referenced by the request until setup */
	struct strom_task *task;
	struct strom_gpumap *gmap;
	struct strom_member *mbr;
	__le64 *prp_list;
	dma_addr_t prp_dma;
	u64 t0;
	/* /proc/diskstats accounting so P2P reads show in iostat, on the
	 * member namespace AND on the volume the file lives on (md raid0 /
	 * multipath head), as the reference's part_stat_* calls did
	 * (kmod/nvme_strom.c:1012-1034) */
	struct block_device *vol_part;   /* NULL: the file is on the namespace */
	unsigned long acct_start, vol_acct_start;
	unsigned int acct_sectors;
	/* SSD2RAM: the DMA buffer range written (one segment: merges never
	 * cross one), handed back to the CPU on completion */
	const struct strom_dbuf_map *ram_map;
	u64 ram_off;
	u32 ram_len;
};

static void req_release_dma(struct strom_req *r)
{
	if (r->prp_list)
		dma_pool_free(r->mbr->prp_pool, r->prp_list, r->prp_dma);
}

static enum rq_end_io_ret strom_end_io(struct request *rq, blk_status_t err)
{
	struct strom_req *r = rq->end_io_data;
	/* nvme_end_req translated the completion's NVMe status into err */
	long status = err ? blk_status_to_errno(err) : 0;

	atomic64_inc(&strom_stats.nr_ssd2gpu);
	atomic64_add(strom_tsc() - r->t0, &strom_stats.clk_ssd2gpu);
	atomic64_dec(&strom_stats.cur_dma_count);
	bdev_end_io_acct(r->mbr->disk->part0, REQ_OP_READ, r->acct_sectors, r->acct_start);
	if (r->vol_part)
		bdev_end_io_acct(r->vol_part, REQ_OP_READ, r->acct_sectors, r->vol_acct_start);
	if (r->ram_len)          /* the task (not yet put) holds the buffer's file */
		strom_dma_buffer_sync_for_cpu(r->task->dbuf_filp, r->ram_map, r->ram_off, r->ram_len);
	req_release_dma(r);
	if (r->gmap && atomic_dec_and_test(&r->gmap->inflight))
		wake_up_all(&r->gmap->drain);
	strom_task_put(r->task, status);
	kfree(r);
	return RQ_END_IO_FREE;
}

struct copy_ctx {
	struct strom_task *t;
	struct strom_volume *vol;
	struct inode *inode;
	struct strom_gpumap *gmap;       /* SSD2GPU */
	u64 gpu_base;                    /* dma-buf byte offset of destination 0 */
	struct vm_area_struct *vma;      /* SSD2RAM */
	unsigned long uaddr_base;
	u64 ram_base;                    /* SSD2RAM: buffer offset of dest_uaddr; the
					    planner works in buffer offsets so that
					    dest_segment matches the real segments */
	/* SSD2RAM: the buffer's map per route member, resolved on the member's
	 * first request (one lock then, none per request or PRP entry) */
	const struct strom_dbuf_map *ram_maps[STROM_ROUTE_MAX_DISKS];
	struct strom_planner pl;
};

struct ram_addr_ctx {
	struct file *dbuf;
	const struct strom_dbuf_map *map;
	u64 base;                        /* buffer offset of the request */
};

/* the buffer's segments are mapped once per controller (strom_dmabuffer.c) */
static int ram_page_addr(void *p, u64 off, u32 need, u64 *a)
{
	struct ram_addr_ctx *x = p;
	u64 contig;
	int rc = strom_dma_buffer_addr(x->dbuf, x->map, x->base + off, a, &contig);

	if (!rc && contig < need)
		rc = -EINVAL;          /* a merge never crosses a segment (or, mapped
					  page by page, a PRP entry a page) */
	return rc;
}

/* submit one merged READ (the planner's flush callback) */
static int submit_extent(void *p, const struct strom_extent *e)
{
	struct copy_ctx *x = p;
	struct strom_member *mbr = &x->vol->m[e->member < 0 ? 0 : e->member];
	const u32 npages = e->len >> STROM_CORE_PAGE_SHIFT;
	struct strom_prps prps;
	struct strom_req *r;
	struct request *rq;
	u64 t0 = strom_tsc(), slba;
	u32 nlb0;
	int rc;

	strom_assert_sleepable();
	rc = strom_core_nvme_rw(e->sect, e->len, mbr->lba_shift, &slba, &nlb0);
	if (rc)
		return rc;
	r = kzalloc(sizeof(*r), GFP_KERNEL);
	if (!r)
		return -ENOMEM;
	r->task = x->t;
	r->mbr = mbr;
	if (npages > 2) {
		r->prp_list = dma_pool_alloc(mbr->prp_pool, GFP_KERNEL, &r->prp_dma);
		if (!r->prp_list) {
			kfree(r);
			return -ENOMEM;
		}
	}
	if (x->gmap) {
		struct strom_sgmap sg;

		rc = strom_gpumap_sgmap(x->gmap, mbr->dma_dev, &sg);
		if (!rc)
			rc = strom_core_build_prps(strom_core_sg_page_addr, &sg, x->gpu_base + e->dest,
						   e->len, (u64 *)r->prp_list, STROM_CORE_PRP_LIST_MAX,
						   r->prp_dma, &prps);
	} else {
		const int mi = e->member < 0 ? 0 : e->member;
		struct ram_addr_ctx rx = { x->t->dbuf_filp, x->ram_maps[mi], e->dest };

		if (!rx.map)
			rx.map = x->ram_maps[mi] = strom_dma_buffer_map(x->t->dbuf_filp, mbr->dma_dev);
		rc = rx.map ? strom_core_build_prps(ram_page_addr, &rx, 0, e->len, (u64 *)r->prp_list,
						    STROM_CORE_PRP_LIST_MAX, r->prp_dma, &prps)
			    : -EIO;
		if (!rc) {
			r->ram_map = rx.map;
			r->ram_off = e->dest;
			r->ram_len = e->len;
		}
	}
	atomic64_inc(&strom_stats.nr_setup_prps);
	atomic64_add(strom_tsc() - t0, &strom_stats.clk_setup_prps);
	if (rc)
		goto fail;
	r->cmd.rw.opcode = nvme_cmd_read;
	r->cmd.rw.nsid = cpu_to_le32(mbr->nsid);
	r->cmd.rw.slba = cpu_to_le64(slba);
	r->cmd.rw.length = cpu_to_le16(nlb0);
	r->cmd.rw.dptr.prp1 = cpu_to_le64(prps.prp1);
	r->cmd.rw.dptr.prp2 = cpu_to_le64(prps.prp2);
	rq = blk_mq_alloc_request(mbr->q, REQ_OP_DRV_IN, 0);
	if (IS_ERR(rq)) {
		rc = PTR_ERR(rq);
		goto fail;
	}
	nvme_init_request(rq, &r->cmd);
	rq->timeout = 30 * HZ;
	rq->end_io = strom_end_io;
	rq->end_io_data = r;
	strom_task_get(x->t);
	if (x->gmap) {
		r->gmap = x->gmap;
		atomic_inc(&x->gmap->inflight);
	}
	strom_stat_inflight_inc();
	r->acct_sectors = e->len >> SECTOR_SHIFT;
	r->acct_start = bdev_start_io_acct(mbr->disk->part0, REQ_OP_READ, jiffies);
	if (x->vol->registered) {
		r->vol_part = x->inode->i_sb->s_bdev;   /* partition: the disk is accounted too */
		r->vol_acct_start = bdev_start_io_acct(r->vol_part, REQ_OP_READ, jiffies);
	}
	t0 = r->t0 = strom_tsc();
	blk_execute_rq_nowait(rq, false);
	/* r belongs to the completion now (it may already be freed): no r->
	 * past this point (TSAN, kernel-model harness) */
	atomic64_inc(&strom_stats.nr_submit_dma);
	atomic64_add(strom_tsc() - t0, &strom_stats.clk_submit_dma);
	return 0;
fail:
	req_release_dma(r);
	kfree(r);
	return rc;
}

static int ctx_bmap(void *p, u64 fblk, u64 *dblk)
{
	struct copy_ctx *x = p;
	sector_t b = fblk;
	int rc = bmap(x->inode, &b);

	if (rc)
		return rc;
	if (!b)
		return -EIO;     /* hole / unwritten / delalloc: nothing to DMA */
	*dblk = b;
	return 0;
}

static void ctx_init(struct copy_ctx *x, struct file *filp)
{
	struct strom_planner *pl = &x->pl;
	u32 max = STROM_CORE_MAX_REQ;
	int i;

	x->inode = file_inode(filp);
	for (i = 0; i < x->vol->nmembers; i++)
		max = min(max, x->vol->m[i].max_bytes);
	memset(pl, 0, sizeof(*pl));
	pl->max_req = max;
	pl->prp_limited = true;
	pl->blkbits = x->inode->i_blkbits;
	pl->part_start_sect = get_start_sect(x->inode->i_sb->s_bdev);
	pl->raid0 = x->vol->raid0 ? &x->vol->geo : NULL;
	pl->bmap = ctx_bmap;
	pl->bmap_ctx = x;
	pl->submit = submit_extent;
	pl->submit_ctx = x;
	strom_core_planner_init(pl);
}

/* page-cache majority score, one dirty page always wins */
static bool chunk_is_cached(struct address_space *map, pgoff_t first, u32 npages)
{
	const u32 threshold = strom_core_cache_threshold(npages);
	u32 score = 0, i;

	for (i = 0; i < npages; i++) {
		struct folio *f = filemap_get_folio(map, first + i);

		if (IS_ERR_OR_NULL(f))
			continue;
		score = strom_core_cache_add(score, threshold, folio_test_dirty(f));
		folio_put(f);
	}
	return strom_core_cache_wins(score, threshold);
}

/* buffered read of a cached chunk into user memory (SSD2GPU wb_buffer;
 * reference memcpy_pgcache_to_ubuffer, kmod/nvme_strom.c:1241-1297): through
 * one kernel page (kernel_read is exported, vfs_read is not), zero past EOF */
static int copy_pgcache_to_user(struct file *filp, loff_t fpos, u32 len, char __user *dst)
{
	void *bounce = (void *)__get_free_page(GFP_KERNEL);
	int rc = 0;
	u32 off;

	if (!bounce)
		return -ENOMEM;
	for (off = 0; off < len && !rc; off += PAGE_SIZE) {
		loff_t pos = fpos + off;
		ssize_t n = kernel_read(filp, bounce, PAGE_SIZE, &pos);

		if (n < 0) {
			rc = n;
			break;
		}
		if (n < PAGE_SIZE)
			memset((char *)bounce + n, 0, PAGE_SIZE - n);
		if (copy_to_user(dst + off, bounce, PAGE_SIZE))
			rc = -EFAULT;
	}
	free_page((unsigned long)bounce);
	return rc;
}

/* the same into our DMA buffer, through its pages' kernel mappings: no user
 * fault can happen while SSD2RAM holds mmap_lock */
static int copy_pgcache_to_ram(struct file *filp, loff_t fpos, u32 len,
			       struct vm_area_struct *vma, unsigned long uaddr)
{
	u32 off;

	for (off = 0; off < len; off += PAGE_SIZE) {
		struct page *pg = strom_dma_buffer_page(vma, uaddr + off - vma->vm_start);
		loff_t pos = fpos + off;
		ssize_t n;
		void *k;

		if (!pg)
			return -EFAULT;
		k = kmap_local_page(pg);
		n = kernel_read(filp, k, PAGE_SIZE, &pos);
		if (n >= 0 && n < PAGE_SIZE)
			memset((char *)k + n, 0, PAGE_SIZE - n);
		kunmap_local(k);
		if (n < 0)
			return n;
	}
	return 0;
}

/* The part of a chunk that has blocks: whole pages up to EOF.  Pages wholly
 * past EOF are never read (they map to no block); SSD2RAM zero-fills them
 * in the buffer, SSD2GPU leaves them untouched in HBM (libstrom clears the
 * file's tail itself), like the userspace provider's short read. */
static u32 chunk_extent(u64 fpos, u32 chunk_sz, loff_t isize)
{
	return (u32)min_t(u64, chunk_sz, round_up((u64)isize - fpos, PAGE_SIZE));
}

static int zero_ram(struct vm_area_struct *vma, unsigned long uaddr, u32 len)
{
	u32 off;

	for (off = 0; off < len; off += PAGE_SIZE) {
		struct page *pg = strom_dma_buffer_page(vma, uaddr + off - vma->vm_start);
		void *k;

		if (!pg)
			return -EFAULT;
		k = kmap_local_page(pg);
		memset(k, 0, PAGE_SIZE);
		kunmap_local(k);
	}
	return 0;
}

/* resolve file + volume; the task owns the references on success */
static int open_source(int fd, struct file **filp, struct strom_volume **vol)
{
	int err;

	*filp = fget(fd);
	if (!*filp)
		return -EBADF;
	err = fs_supported(*filp);
	if (!err) {
		*vol = strom_volume_of_file(*filp, &err);
		if (*vol)
			return 0;
	}
	fput(*filp);
	return err;
}

int strom_memcpy_ssd2gpu(struct strom_session *s, struct strom_memcpy_ssd2gpu __user *uarg)
{
	struct strom_memcpy_ssd2gpu k;
	struct strom_landing land = {};
	struct copy_ctx x = {};
	u32 *ids = NULL, *out, i;
	struct strom_gpumap *gmap;
	struct file *filp;
	loff_t isize;
	int rc;

	if (copy_from_user(&k, uarg, sizeof(k)))
		return -EFAULT;
	if (!k.nr_chunks || k.nr_chunks > STROM_MAX_CHUNKS || (k.chunk_sz & (PAGE_SIZE - 1)) ||
	    k.chunk_sz < PAGE_SIZE || k.chunk_sz > STROM_CORE_MAX_REQ)
		return -EINVAL;
	gmap = strom_gpumap_get(k.handle);
	if (!gmap)
		return -ENOENT;
	/* overflow-safe range check + 4 KiB destination alignment (PRP rule) */
	rc = strom_core_check_dest(gmap->length, gmap->dmabuf_off, k.offset,
				   (u64)k.nr_chunks * k.chunk_sz);
	if (rc) {
		strom_gpumap_put(gmap);
		return rc;
	}
	rc = open_source(k.file_desc, &filp, &x.vol);
	if (rc) {
		strom_gpumap_put(gmap);
		return rc;
	}
	ids = kvmalloc_array(k.nr_chunks, 2 * sizeof(u32), GFP_KERNEL);
	if (!ids || copy_from_user(ids, k.chunk_ids, k.nr_chunks * sizeof(u32))) {
		rc = ids ? -EFAULT : -ENOMEM;
		fput(filp);
		strom_volume_put(x.vol);
		strom_gpumap_put(gmap);
		goto out_free;
	}
	out = ids + k.nr_chunks;
	x.t = strom_task_create(s, filp, gmap);   /* task owns filp + gmap refs */
	if (!x.t) {
		fput(filp);
		strom_volume_put(x.vol);
		strom_gpumap_put(gmap);
		rc = -ENOMEM;
		goto out_free;
	}
	x.t->vol = x.vol;
	x.gmap = gmap;
	x.gpu_base = gmap->dmabuf_off + k.offset;
	ctx_init(&x, filp);
	isize = i_size_read(x.inode);
	land.nr_chunks = k.nr_chunks;
	land.reorder = true;
	rc = 0;
	for (i = 0; i < k.nr_chunks && !rc; i++) {
		const u32 cid = ids[i];
		u64 fpos;
		bool cached;
		u32 slot;
		size_t dest;

		rc = strom_core_chunk_fpos(cid, k.chunk_sz, k.relseg_sz, isize, &fpos);
		if (rc)
			break;
		cached = chunk_is_cached(filp->f_mapping, fpos >> PAGE_SHIFT, k.chunk_sz >> PAGE_SHIFT);
		slot = strom_core_land(&land, i, cached);
		out[slot] = cid;
		dest = (size_t)slot * k.chunk_sz;
		if (cached && k.wb_buffer) {
			rc = copy_pgcache_to_user(filp, fpos, k.chunk_sz, k.wb_buffer + dest);
		} else {
			/* wb_buffer == NULL: the cached chunk still lands at the
			 * tail, by DMA after its dirty pages reached the device */
			if (cached)
				rc = filemap_write_and_wait_range(filp->f_mapping, fpos,
								  fpos + k.chunk_sz - 1);
			if (!rc)
				rc = strom_core_plan_range(&x.pl, fpos,
							   chunk_extent(fpos, k.chunk_sz, isize), dest);
		}
	}
	if (!rc)
		rc = strom_core_plan_flush(&x.pl);
	x.t->frozen = true;
	k.dma_task_id = x.t->id;
	strom_task_put(x.t, rc);
	if (rc) {
		long st;

		strom_task_wait_session(s, k.dma_task_id, &st, MAX_SCHEDULE_TIMEOUT);
		goto out_free;
	}
	k.nr_ram2gpu = land.nr_ram;
	k.nr_ssd2gpu = land.nr_ssd;
	k.nr_dma_submit = x.pl.nr_submit;
	k.nr_dma_blocks = (u32)x.pl.nr_sectors;
	if (copy_to_user(uarg, &k, offsetof(struct strom_memcpy_ssd2gpu, handle)) ||
	    copy_to_user(k.chunk_ids, out, k.nr_chunks * sizeof(u32)))
		rc = -EFAULT;
out_free:
	kvfree(ids);
	return rc;
}

_Static_assert(sizeof(struct strom_file_extent) == sizeof(struct strom_xfer_extent) &&
	       offsetof(struct strom_file_extent, dst_off) == offsetof(struct strom_xfer_extent, dst_off) &&
	       offsetof(struct strom_file_extent, len) == offsetof(struct strom_xfer_extent, len),
	       "uapi extent == core extent");

/* MEMCPY_SSD2GPU_EXTENTS: exact byte ranges (an Arrow scan's buffers), laid
 * out and merged by the shared core (strom_core_plan_xfer); every byte by
 * NVMe READ into HBM after the span's dirty page-cache pages were written
 * back (the chunk path's coherence rule, without a page-cache leg) */
int strom_memcpy_ssd2gpu_extents(struct strom_session *s,
				 struct strom_memcpy_ssd2gpu_extents __user *uarg)
{
	struct strom_memcpy_ssd2gpu_extents k;
	struct strom_xfer_extent *x = NULL;
	struct strom_gpumap *gmap = NULL;
	struct copy_ctx c = {};
	u64 dst_bytes = 0, read_bytes = 0, want = 0;
	struct file *filp;
	loff_t isize;
	u32 i;
	int rc;

	if (copy_from_user(&k, uarg, sizeof(k)))
		return -EFAULT;
	if (k.nr_extents > STROM_MAX_CHUNKS || (k.flags & ~STROM_EXTENTS_PLAN_ONLY))
		return -EINVAL;
	rc = open_source(k.file_desc, &filp, &c.vol);
	if (rc)
		return rc;
	x = kvmalloc_array(k.nr_extents ? k.nr_extents : 1, sizeof(*x), GFP_KERNEL);
	if (!x || copy_from_user(x, k.extents, (size_t)k.nr_extents * sizeof(*x))) {
		rc = x ? -EFAULT : -ENOMEM;
		goto out_src;
	}
	isize = i_size_read(file_inode(filp));
	/* the layout first: the destination it needs, nothing submitted */
	rc = strom_core_plan_xfer(NULL, x, k.nr_extents, k.gap_max, isize, &dst_bytes, &read_bytes);
	if (rc)
		goto out_src;
	for (i = 0; i < k.nr_extents; i++)
		want += x[i].len;
	k.dst_bytes = dst_bytes;
	k.bytes_read = read_bytes;
	k.gap_bytes = read_bytes - want;
	k.dma_task_id = 0;
	k.nr_dma_submit = k.nr_dma_blocks = 0;
	if (k.flags & STROM_EXTENTS_PLAN_ONLY)
		goto out_copy;
	gmap = strom_gpumap_get(k.handle);
	if (!gmap) {
		rc = -ENOENT;
		goto out_src;
	}
	rc = strom_core_check_dest(gmap->length, gmap->dmabuf_off, k.offset, dst_bytes);
	if (!rc && read_bytes) {
		/* the extents' span: dirty pages reach the device before it is read */
		for (i = 0; i < k.nr_extents && !x[i].len; i++)
			;
		rc = filemap_write_and_wait_range(filp->f_mapping, x[i].file_off,
						  x[k.nr_extents - 1].file_off + x[k.nr_extents - 1].len);
	}
	if (rc) {
		strom_gpumap_put(gmap);
		goto out_src;
	}
	c.t = strom_task_create(s, filp, gmap);   /* task owns filp + gmap refs */
	if (!c.t) {
		strom_gpumap_put(gmap);
		rc = -ENOMEM;
		goto out_src;
	}
	c.t->vol = c.vol;
	c.gmap = gmap;
	c.gpu_base = gmap->dmabuf_off + k.offset;
	ctx_init(&c, filp);
	rc = strom_core_plan_xfer(&c.pl, x, k.nr_extents, k.gap_max, isize, &dst_bytes, &read_bytes);
	if (!rc)
		rc = strom_core_plan_flush(&c.pl);
	c.t->frozen = true;
	k.dma_task_id = c.t->id;
	strom_task_put(c.t, rc);
	if (rc) {
		long st;

		strom_task_wait_session(s, k.dma_task_id, &st, MAX_SCHEDULE_TIMEOUT);
		goto out_free;
	}
	k.nr_dma_submit = c.pl.nr_submit;
	k.nr_dma_blocks = (u32)c.pl.nr_sectors;
	goto out_copy_free;
out_copy:
	fput(filp);
	strom_volume_put(c.vol);
out_copy_free:
	if (copy_to_user(uarg, &k, offsetof(struct strom_memcpy_ssd2gpu_extents, handle)) ||
	    copy_to_user(k.extents, x, (size_t)k.nr_extents * sizeof(*x)))
		rc = -EFAULT;
	goto out_free;
out_src:
	fput(filp);
	strom_volume_put(c.vol);
out_free:
	kvfree(x);
	return rc;
}

int strom_memcpy_ssd2ram(struct strom_session *s, struct strom_memcpy_ssd2ram __user *uarg)
{
	struct strom_memcpy_ssd2ram k;
	struct strom_landing land = {};
	struct copy_ctx x = {};
	struct vm_area_struct *vma;
	u32 *ids = NULL, i;
	struct file *filp;
	size_t bytes;
	loff_t isize;
	int rc;

	if (copy_from_user(&k, uarg, sizeof(k)))
		return -EFAULT;
	if (!k.nr_chunks || k.nr_chunks > STROM_MAX_CHUNKS || (k.chunk_sz & (PAGE_SIZE - 1)) ||
	    k.chunk_sz < PAGE_SIZE || k.chunk_sz > STROM_CORE_MAX_REQ ||
	    ((unsigned long)k.dest_uaddr & (PAGE_SIZE - 1)))
		return -EINVAL;
	bytes = (size_t)k.nr_chunks * k.chunk_sz;
	ids = kvmalloc_array(k.nr_chunks, sizeof(u32), GFP_KERNEL);
	if (!ids)
		return -ENOMEM;
	if (copy_from_user(ids, k.chunk_ids, k.nr_chunks * sizeof(u32))) {
		kvfree(ids);
		return -EFAULT;
	}
	rc = open_source(k.file_desc, &filp, &x.vol);
	if (rc) {
		kvfree(ids);
		return rc;
	}
	mmap_read_lock(current->mm);
	vma = find_vma(current->mm, (unsigned long)k.dest_uaddr);
	if (!vma || !strom_is_dma_buffer(vma) || (unsigned long)k.dest_uaddr < vma->vm_start ||
	    bytes > vma->vm_end - (unsigned long)k.dest_uaddr) {
		mmap_read_unlock(current->mm);
		fput(filp);
		strom_volume_put(x.vol);
		kvfree(ids);
		return -EINVAL;
	}
	x.t = strom_task_create(s, filp, NULL);
	if (!x.t) {
		mmap_read_unlock(current->mm);
		fput(filp);
		strom_volume_put(x.vol);
		kvfree(ids);
		return -ENOMEM;
	}
	x.t->vol = x.vol;
	/* the buffer's pages must outlive the DMA even if userspace unmaps
	 * and closes it meanwhile (the reference refcounted its buffers) */
	x.t->dbuf_filp = get_file(vma->vm_file);
	x.vma = vma;
	x.uaddr_base = (unsigned long)k.dest_uaddr;
	x.ram_base = ((unsigned long)k.dest_uaddr - vma->vm_start) + (vma->vm_pgoff << PAGE_SHIFT);
	ctx_init(&x, filp);
	/* a merged request never crosses a 4 MiB segment of the buffer
	 * (reference dest_segment_sz), where physical contiguity ends */
	x.pl.dest_segment = STROM_DMABUF_SEGMENT;
	isize = i_size_read(x.inode);
	land.nr_chunks = k.nr_chunks;
	land.reorder = false;       /* SSD2RAM: chunk i lands at dest + i * chunk_sz */
	rc = 0;
	for (i = 0; i < k.nr_chunks && !rc; i++) {
		u64 fpos;
		bool cached;
		size_t dest;

		rc = strom_core_chunk_fpos(ids[i], k.chunk_sz, k.relseg_sz, isize, &fpos);
		if (rc)
			break;
		cached = chunk_is_cached(filp->f_mapping, fpos >> PAGE_SHIFT, k.chunk_sz >> PAGE_SHIFT);
		dest = (size_t)strom_core_land(&land, i, cached) * k.chunk_sz;
		if (cached) {
			rc = copy_pgcache_to_ram(filp, fpos, k.chunk_sz, vma, x.uaddr_base + dest);
		} else {
			u32 n = chunk_extent(fpos, k.chunk_sz, isize);

			rc = strom_core_plan_range(&x.pl, fpos, n, x.ram_base + dest);
			if (!rc && n < k.chunk_sz)
				rc = zero_ram(vma, x.uaddr_base + dest + n, k.chunk_sz - n);
		}
	}
	if (!rc)
		rc = strom_core_plan_flush(&x.pl);
	mmap_read_unlock(current->mm);
	x.t->frozen = true;
	k.dma_task_id = x.t->id;
	strom_task_put(x.t, rc);
	if (rc) {
		long st;

		strom_task_wait_session(s, k.dma_task_id, &st, MAX_SCHEDULE_TIMEOUT);
		kvfree(ids);
		return rc;
	}
	k.nr_ram2ram = land.nr_ram;
	k.nr_ssd2ram = land.nr_ssd;
	k.nr_dma_submit = x.pl.nr_submit;
	k.nr_dma_blocks = (u32)x.pl.nr_sectors;
	if (copy_to_user(uarg, &k, offsetof(struct strom_memcpy_ssd2ram, dest_uaddr)))
		rc = -EFAULT;
	kvfree(ids);
	return rc;
}
