// SPDX-License-Identifier: GPL-2.0
/*
 * strom_gpumap.c — HBM mappings imported as dma-bufs.
 *
 * Replaces the reference's nvidia_p2p_get_pages registry (kmod/pmemmap.c:
 * 19-495).  amdgpu exports VRAM buffer objects as dma-bufs; we attach with
 * allow_peer2peer for each NVMe controller that will write into the range,
 * pin the attachment (so the BO cannot migrate out of VRAM while reads are
 * in flight — move_notify is therefore a no-op for pinned attachments) and
 * map it to get bus addresses through the controller's IOMMU domain.
 *
 * Lifetime: handle -> kref'd record; UNMAP removes it from the table and
 * waits until in-flight requests drop to zero before unpinning (fixes
 * reference defect #7: UNMAP neither freed nor waited).
 */
#include <linux/dma-resv.h>
#include <linux/hashtable.h>
#include <linux/slab.h>
#include <linux/uaccess.h>

#include "strom_kmod.h"

static DEFINE_HASHTABLE(gpumap_slots, 6);   /* 64 slots, as in v0.6 */
static DEFINE_SPINLOCK(gpumap_lock);
static unsigned long gpumap_next = 0x5350000000000000UL;

static void strom_move_notify(struct dma_buf_attachment *att)
{
	/* pinned attachments are never moved by the exporter */
}

static const struct dma_buf_attach_ops strom_importer_ops = {
	.allow_peer2peer = true,
	.move_notify = strom_move_notify,
};

static struct workqueue_struct *gpumap_wq;

/* The last reference can drop in an NVMe completion (IRQ context, through
 * the task), but unpin/detach take the reservation lock and sleep: the
 * teardown runs on a workqueue.  Module exit destroys the queue, which
 * waits for a teardown still running. */
static void gpumap_free_work(struct work_struct *w)
{
	struct strom_gpumap *m = container_of(w, struct strom_gpumap, free_work);
	int i;

	for (i = 0; i < m->natt; i++) {
		struct strom_attach *a = &m->att[i];

		dma_resv_lock(m->dmabuf->resv, NULL);
		dma_buf_unmap_attachment(a->att, a->sgt, DMA_BIDIRECTIONAL);
		dma_buf_unpin(a->att);
		dma_resv_unlock(m->dmabuf->resv);
		dma_buf_detach(m->dmabuf, a->att);
		kvfree(a->seg_addr);
	}
	dma_buf_put(m->dmabuf);
	kfree(m);
	module_put(THIS_MODULE);
}

static void gpumap_release(struct kref *ref)
{
	struct strom_gpumap *m = container_of(ref, struct strom_gpumap, ref);

	queue_work(gpumap_wq, &m->free_work);
}

struct strom_gpumap *strom_gpumap_get(unsigned long handle)
{
	struct strom_gpumap *m;

	spin_lock(&gpumap_lock);
	hash_for_each_possible(gpumap_slots, m, node, handle) {
		if (m->handle == handle && uid_eq(m->owner, current_euid())) {
			kref_get(&m->ref);
			spin_unlock(&gpumap_lock);
			return m;
		}
	}
	spin_unlock(&gpumap_lock);
	return NULL;
}

void strom_gpumap_put(struct strom_gpumap *m)
{
	kref_put(&m->ref, gpumap_release);
}

int strom_map_dmabuf(struct strom_map_gpu_dmabuf *arg)
{
	struct strom_gpumap *m;
	struct dma_buf *db;

	if (!arg->length)
		return -EINVAL;
	db = dma_buf_get(arg->dmabuf_fd);
	if (IS_ERR(db))
		return PTR_ERR(db);
	/* userspace exports the whole allocation that holds the range (a
	 * tensor is usually a sub-allocation): the range starts dmabuf_offset
	 * bytes into it */
	if (arg->dmabuf_offset > db->size || arg->length > db->size - arg->dmabuf_offset) {
		dma_buf_put(db);
		return -ERANGE;
	}
	m = kzalloc(sizeof(*m), GFP_KERNEL);
	if (!m) {
		dma_buf_put(db);
		return -ENOMEM;
	}
	m->dmabuf = db;
	m->vaddress = arg->vaddress;
	m->dmabuf_off = arg->dmabuf_offset;
	INIT_WORK(&m->free_work, gpumap_free_work);
	m->length = arg->length;
	m->owner = current_euid();
	mutex_init(&m->att_lock);
	atomic_set(&m->inflight, 0);
	init_waitqueue_head(&m->drain);
	kref_init(&m->ref);
	__module_get(THIS_MODULE);
	spin_lock(&gpumap_lock);
	m->handle = ++gpumap_next;
	hash_add(gpumap_slots, &m->node, m->handle);
	spin_unlock(&gpumap_lock);
	arg->handle = m->handle;
	arg->gpu_page_sz = STROM_GPU_BOUND_SIZE;
	arg->gpu_npages = DIV_ROUND_UP(arg->length, STROM_GPU_BOUND_SIZE);
	prDebug("map dmabuf fd=%d len=%zu handle=%#lx", arg->dmabuf_fd, arg->length, m->handle);
	return 0;
}

/* Only the caller that takes the record out of the table owns the table's
 * reference: a second, concurrent UNMAP of the same handle finds nothing and
 * returns -ENOENT (two callers could both pass a lookup and drop
 * four references against three). */
int strom_unmap_gpu(unsigned long handle)
{
	struct strom_gpumap *m = NULL, *it;

	spin_lock(&gpumap_lock);
	hash_for_each_possible(gpumap_slots, it, node, handle) {
		if (it->handle == handle && uid_eq(it->owner, current_euid())) {
			hash_del(&it->node);
			m = it;
			break;
		}
	}
	spin_unlock(&gpumap_lock);
	if (!m)
		return -ENOENT;
	/* reference v0.6 never waited (defect #7): drain in-flight DMA first */
	wait_event(m->drain, atomic_read(&m->inflight) == 0);
	strom_gpumap_put(m);   /* the table's reference, now ours */
	return 0;
}

/* the sg table flattened into start/len/bus-address arrays once: every
 * later lookup is a binary search (or O(1) for the next page), where v1
 * walked the list from its head for each 4 KiB page */
static int flatten_sgt(struct strom_attach *a)
{
	struct scatterlist *sg;
	u32 n = 0, i = 0;
	u64 off = 0;
	int k;

	for_each_sgtable_dma_sg(a->sgt, sg, k)
		n++;
	a->seg_addr = kvmalloc_array(n, 3 * sizeof(u64), GFP_KERNEL);
	if (!a->seg_addr)
		return -ENOMEM;
	a->seg_len = a->seg_addr + n;
	a->seg_start = a->seg_len + n;
	for_each_sgtable_dma_sg(a->sgt, sg, k) {
		a->seg_addr[i] = sg_dma_address(sg);
		a->seg_len[i] = sg_dma_len(sg);
		a->seg_start[i] = off;
		off += sg_dma_len(sg);
		i++;
	}
	a->nsegs = n;
	return 0;
}

/* attach + pin + map + flatten for `dev` once; caller holds a reference on m */
static struct strom_attach *gpumap_attach(struct strom_gpumap *m, struct device *dev)
{
	struct strom_attach *a = NULL;
	struct dma_buf_attachment *att;
	struct sg_table *sgt;
	int i, rc;

	mutex_lock(&m->att_lock);
	for (i = 0; i < m->natt; i++)
		if (m->att[i].dev == dev) {
			a = &m->att[i];
			goto out;
		}
	if (m->natt == ARRAY_SIZE(m->att))
		goto out;
	att = dma_buf_dynamic_attach(m->dmabuf, dev, &strom_importer_ops, m);
	if (IS_ERR(att))
		goto out;
	if (!att->peer2peer) {
		/* the exporter refused P2P for this device pair */
		dma_buf_detach(m->dmabuf, att);
		goto out;
	}
	dma_resv_lock(m->dmabuf->resv, NULL);
	rc = dma_buf_pin(att);
	if (rc) {
		dma_resv_unlock(m->dmabuf->resv);
		dma_buf_detach(m->dmabuf, att);
		goto out;
	}
	sgt = dma_buf_map_attachment(att, DMA_BIDIRECTIONAL);
	dma_resv_unlock(m->dmabuf->resv);
	if (IS_ERR(sgt))
		goto unpin;
	a = &m->att[m->natt];
	a->dev = dev;
	a->att = att;
	a->sgt = sgt;
	if (flatten_sgt(a)) {
		dma_resv_lock(m->dmabuf->resv, NULL);
		dma_buf_unmap_attachment(att, sgt, DMA_BIDIRECTIONAL);
		dma_resv_unlock(m->dmabuf->resv);
		memset(a, 0, sizeof(*a));
		a = NULL;
		goto unpin;
	}
	m->natt++;
	goto out;
unpin:
	dma_resv_lock(m->dmabuf->resv, NULL);
	dma_buf_unpin(att);
	dma_resv_unlock(m->dmabuf->resv);
	dma_buf_detach(m->dmabuf, att);
out:
	mutex_unlock(&m->att_lock);
	return a;
}

int strom_gpumap_sgmap(struct strom_gpumap *m, struct device *dev, struct strom_sgmap *sg)
{
	struct strom_attach *a = gpumap_attach(m, dev);

	if (!a)
		return -EOPNOTSUPP;
	sg->nsegs = a->nsegs;
	sg->addr = a->seg_addr;
	sg->len = a->seg_len;
	sg->start = a->seg_start;
	sg->hint = 0;          /* per caller: lookups never share a hint */
	return 0;
}

int strom_list_gpu(struct strom_list_gpu_memory __user *uarg)
{
	struct strom_gpumap *m;
	unsigned long *h = NULL;
	u32 nrooms, cap, n = 0;
	int bkt, rc = 0;

	if (get_user(nrooms, &uarg->nrooms))
		return -EFAULT;
	/* copying out may fault and sleep, and a record may be unmapped and
	 * freed once the lock is dropped: snapshot the handles first */
	cap = min_t(u32, nrooms, 4096);
	if (cap) {
		h = kmalloc_array(cap, sizeof(*h), GFP_KERNEL);
		if (!h)
			return -ENOMEM;
	}
	spin_lock(&gpumap_lock);
	hash_for_each(gpumap_slots, bkt, m, node) {
		if (!uid_eq(m->owner, current_euid()))
			continue;
		if (n < cap)
			h[n] = m->handle;
		n++;
	}
	spin_unlock(&gpumap_lock);
	if (cap && copy_to_user(uarg->handles, h, min(n, cap) * sizeof(*h)))
		rc = -EFAULT;
	kfree(h);
	if (!rc && put_user(n, &uarg->nitems))
		rc = -EFAULT;
	return rc;
}

int strom_info_gpu(struct strom_info_gpu_memory __user *uarg)
{
	struct strom_info_gpu_memory k;
	struct strom_gpumap *m;
	u32 i, npages;

	if (copy_from_user(&k, uarg, offsetof(struct strom_info_gpu_memory, paddrs)))
		return -EFAULT;
	m = strom_gpumap_get(k.handle);
	if (!m)
		return -ENOENT;
	npages = DIV_ROUND_UP(m->length, STROM_GPU_BOUND_SIZE);
	k.nitems = npages;
	k.version = 1;
	k.gpu_page_sz = STROM_GPU_BOUND_SIZE;
	k.owner = from_kuid(current_user_ns(), m->owner);
	k.map_offset = m->vaddress & (STROM_GPU_BOUND_SIZE - 1);
	k.map_length = m->length;
	for (i = 0; i < npages && i < k.nrooms; i++) {
		/* bus address as seen by the first attached controller, if any
		 * (natt only grows, and att[0] never changes once set) */
		u64 pa = 0;

		if (m->natt) {
			struct strom_sgmap sg;
			u64 a, c;

			if (!strom_gpumap_sgmap(m, m->att[0].dev, &sg) &&
			    !strom_core_sg_lookup(&sg, m->dmabuf_off + (u64)i * STROM_GPU_BOUND_SIZE, &a, &c))
				pa = a;
		}
		if (put_user(pa, &uarg->paddrs[i])) {
			strom_gpumap_put(m);
			return -EFAULT;
		}
	}
	strom_gpumap_put(m);
	return copy_to_user(uarg, &k, offsetof(struct strom_info_gpu_memory, paddrs)) ? -EFAULT : 0;
}

int strom_gpumap_init(void)
{
	hash_init(gpumap_slots);
	gpumap_wq = alloc_workqueue("strom_gpumap", WQ_UNBOUND, 0);
	return gpumap_wq ? 0 : -ENOMEM;
}

void strom_gpumap_exit(void)
{
	/* live mappings hold module references, so only teardowns queued by
	 * the last puts can remain: destroying the queue drains them */
	destroy_workqueue(gpumap_wq);
}
