// SPDX-License-Identifier: GPL-2.0
/*
 * strom_dmabuffer.c — ALLOC_DMA_BUFFER: NUMA-local host buffers for SSD2RAM.
 *
 * As in the reference (kmod/pmemmap.c:497-717): the buffer is a set of
 * 4 MiB physically contiguous segments allocated on the requested node,
 * wrapped in an anon-inode fd named "dmabuf<node>:<size>" that userspace
 * mmaps MAP_SHARED; pages are served by a fault handler.  The buffer is
 * refcounted by its file, so it outlives the fd while mappings exist.
 * SSD2RAM needs bus addresses (IOMMU-correct; the reference wrote raw
 * physical addresses into PRPs, defect #8): each 4 MiB segment is mapped
 * ONCE per NVMe controller, on first use, with one dma_map_page() of the
 * whole physically contiguous segment, and stays mapped until the buffer is
 * released (the request path does no per-page map/unmap and no allocation).
 * A controller whose DMA layer cannot map 4 MiB at once (swiotlb bouncing
 * caps a mapping at ~256 KiB) gets the segment mapped page by page instead.
 * Any number of controllers may map one buffer (a raid0 route has up to
 * STROM_ROUTE_MAX_DISKS members; a buffer may be reused across volumes).
 * The node is validated before any allocation (reference pmemmap.c:646-650),
 * and an mmap must lie inside the buffer (pmemmap.c:593).
 */
#include <linux/anon_inodes.h>
#include <linux/file.h>
#include <linux/mm.h>
#include <linux/slab.h>

#include "strom_kmod.h"

#define SEG_ORDER (22 - PAGE_SHIFT)          /* 4 MiB segments */
#define SEG_SIZE (PAGE_SIZE << SEG_ORDER)

#define SEG_PAGES (1 << SEG_ORDER)

struct strom_dbuf_map {                  /* the segments as one controller sees them */
	struct device *dev;              /* held (get_device) */
	bool per_page;                   /* dma[] holds one address per page */
	dma_addr_t dma[];                /* per segment, or per page (per_page) */
};

struct strom_dma_buffer {
	size_t length;
	int node;
	int nsegs;
	struct mutex map_lock;           /* guards maps / nmaps / cap_maps */
	int nmaps, cap_maps;
	struct strom_dbuf_map **maps;    /* each map stays put until release */
	struct page *segs[];
};

static vm_fault_t dmabuf_fault(struct vm_fault *vmf)
{
	struct strom_dma_buffer *b = vmf->vma->vm_file->private_data;
	unsigned long off = (vmf->pgoff << PAGE_SHIFT);
	struct page *p;

	if (off >= b->length)
		return VM_FAULT_SIGBUS;
	p = b->segs[off / SEG_SIZE] + ((off % SEG_SIZE) >> PAGE_SHIFT);
	get_page(p);
	vmf->page = p;
	return 0;
}

static const struct vm_operations_struct dmabuf_vm_ops = {
	.fault = dmabuf_fault,
};

static int dmabuf_mmap(struct file *filp, struct vm_area_struct *vma)
{
	struct strom_dma_buffer *b = filp->private_data;

	if (!(vma->vm_flags & VM_SHARED))
		return -EINVAL;
	/* the mapping must lie inside the buffer (reference pmemmap.c:593) */
	if (vma->vm_pgoff > (b->length >> PAGE_SHIFT) ||
	    vma_pages(vma) > (b->length >> PAGE_SHIFT) - vma->vm_pgoff)
		return -EINVAL;
	vm_flags_set(vma, VM_DONTEXPAND | VM_DONTDUMP);
	vma->vm_ops = &dmabuf_vm_ops;
	return 0;
}

static int dmabuf_release(struct inode *inode, struct file *filp)
{
	struct strom_dma_buffer *b = filp->private_data;
	int i, j;

	/* the last reference: no request can still target the buffer (every
	 * SSD2RAM task holds the file until its last completion) */
	for (j = 0; j < b->nmaps; j++) {
		struct strom_dbuf_map *m = b->maps[j];
		const int n = m->per_page ? b->nsegs * SEG_PAGES : b->nsegs;

		for (i = 0; i < n; i++)
			if (m->dma[i])
				dma_unmap_page(m->dev, m->dma[i], m->per_page ? PAGE_SIZE : SEG_SIZE,
					       DMA_FROM_DEVICE);
		put_device(m->dev);
		kfree(m);
	}
	kfree(b->maps);
	for (i = 0; i < b->nsegs; i++) {
		struct page *p = b->segs[i];
		int k;

		for (k = 0; k < (1 << SEG_ORDER); k++)
			__free_page(p + k);
	}
	kfree(b);
	return 0;
}

static const struct file_operations dmabuf_fops = {
	.owner = THIS_MODULE,
	.mmap = dmabuf_mmap,
	.release = dmabuf_release,
};

bool strom_is_dma_buffer(struct vm_area_struct *vma)
{
	return vma->vm_file && vma->vm_file->f_op == &dmabuf_fops;
}

struct page *strom_dma_buffer_page(struct vm_area_struct *vma, unsigned long off)
{
	struct strom_dma_buffer *b = vma->vm_file->private_data;

	off += vma->vm_pgoff << PAGE_SHIFT;
	if (off >= b->length)
		return NULL;
	return b->segs[off / SEG_SIZE] + ((off % SEG_SIZE) >> PAGE_SHIFT);
}

/* map every segment for `dev`: whole segments, or page by page when the
 * DMA layer refuses a 4 MiB mapping; NULL on failure */
static struct strom_dbuf_map *dbuf_map_new(struct strom_dma_buffer *b, struct device *dev,
					   bool per_page)
{
	const int n = per_page ? b->nsegs * SEG_PAGES : b->nsegs;
	struct strom_dbuf_map *m = kzalloc(struct_size(m, dma, n), GFP_KERNEL);
	int i;

	if (!m)
		return NULL;
	m->per_page = per_page;
	for (i = 0; i < n; i++) {
		struct page *pg = per_page ? b->segs[i / SEG_PAGES] + i % SEG_PAGES : b->segs[i];
		const size_t sz = per_page ? PAGE_SIZE : SEG_SIZE;

		m->dma[i] = dma_map_page(dev, pg, 0, sz, DMA_FROM_DEVICE);
		if (dma_mapping_error(dev, m->dma[i])) {
			while (i-- > 0)
				dma_unmap_page(dev, m->dma[i], sz, DMA_FROM_DEVICE);
			kfree(m);
			return NULL;
		}
	}
	m->dev = get_device(dev);
	return m;
}

/* The segment table of the DMA buffer behind `filp` as controller `dev` sees
 * it, mapped on first use.  The result stays valid until the buffer is
 * released (every SSD2RAM task holds the file), so a request resolves it
 * once and then computes its PRP entries without the lock. */
struct strom_dbuf_map *strom_dma_buffer_map(struct file *filp, struct device *dev)
{
	struct strom_dma_buffer *b = filp->private_data;
	struct strom_dbuf_map *m = NULL;
	int j;

	mutex_lock(&b->map_lock);
	for (j = 0; j < b->nmaps; j++)
		if (b->maps[j]->dev == dev) {
			m = b->maps[j];
			goto out;
		}
	if (b->nmaps == b->cap_maps) {
		int cap = b->cap_maps ? 2 * b->cap_maps : 4;
		struct strom_dbuf_map **nm = krealloc_array(b->maps, cap, sizeof(*nm), GFP_KERNEL);

		if (!nm)
			goto out;
		b->maps = nm;
		b->cap_maps = cap;
	}
	m = dbuf_map_new(b, dev, false);
	if (!m) {
		/* Page-by-page maps stay until the buffer is released.  Under
		 * swiotlb every page holds a bounce slot for that long, so the
		 * buffers a controller can serve at once are bounded by the
		 * bounce pool (64 MiB by default): a raid0 route over several
		 * members maps the buffer once per member.  Said in the log,
		 * since SSD2RAM then fails with -EIO, not at allocation. */
		pr_notice("nvme-strom: dma buffer %zu bytes: 4 MiB segment map refused, mapping %d pages one by one\n",
			  (size_t)b->length, b->nsegs * SEG_PAGES);
		m = dbuf_map_new(b, dev, true);
		if (!m)
			pr_warn("nvme-strom: dma buffer %zu bytes: page-by-page map failed (bounce pool exhausted?)\n",
				(size_t)b->length);
	}
	if (m)
		b->maps[b->nmaps++] = m;
out:
	mutex_unlock(&b->map_lock);
	return m;
}

/* Bus address through map `m` of byte `off` of the DMA buffer behind
 * `filp`; *contig = bytes that stay bus-contiguous from there (to the end of
 * the segment, or of the page for a page-by-page map).  No lock. */
int strom_dma_buffer_addr(struct file *filp, const struct strom_dbuf_map *m, u64 off, u64 *addr,
			  u64 *contig)
{
	struct strom_dma_buffer *b = filp->private_data;

	if (off >= b->length)
		return -EFAULT;
	if (m->per_page) {
		*addr = m->dma[off >> PAGE_SHIFT] + (off & (PAGE_SIZE - 1));
		*contig = PAGE_SIZE - (off & (PAGE_SIZE - 1));
	} else {
		*addr = m->dma[off / SEG_SIZE] + off % SEG_SIZE;
		*contig = SEG_SIZE - off % SEG_SIZE;
	}
	return 0;
}

/* hand [off, off+len) back to the CPU after the device wrote it */
void strom_dma_buffer_sync_for_cpu(struct file *filp, const struct strom_dbuf_map *m, u64 off,
				   u64 len)
{
	while (len) {
		u64 a, contig;

		if (strom_dma_buffer_addr(filp, m, off, &a, &contig))
			return;
		if (contig > len)
			contig = len;
		dma_sync_single_for_cpu(m->dev, a, contig, DMA_FROM_DEVICE);
		off += contig;
		len -= contig;
	}
}

int strom_alloc_dma_buffer(struct strom_alloc_dma_buffer *arg)
{
	struct strom_dma_buffer *b;
	char name[48];
	int i, nsegs, fd;

	if (!arg->length)
		return -EINVAL;
	/* a user-chosen node must exist and have memory (alloc_pages_node
	 * indexes node data with it) */
	if (arg->node_id >= 0 && (arg->node_id >= nr_node_ids || !node_online(arg->node_id)))
		return -EINVAL;
	if (arg->length > ((size_t)INT_MAX / 2) * SEG_SIZE)
		return -E2BIG;
	nsegs = DIV_ROUND_UP(arg->length, SEG_SIZE);
	b = kzalloc(struct_size(b, segs, nsegs), GFP_KERNEL);
	if (!b)
		return -ENOMEM;
	b->node = arg->node_id < 0 ? numa_node_id() : arg->node_id;
	b->length = (size_t)nsegs * SEG_SIZE;
	mutex_init(&b->map_lock);
	for (i = 0; i < nsegs; i++) {
		struct page *p = alloc_pages_node(b->node, GFP_KERNEL | __GFP_ZERO, SEG_ORDER);

		if (!p)
			goto nomem;
		split_page(p, SEG_ORDER);
		b->segs[i] = p;
		b->nsegs++;
	}
	snprintf(name, sizeof(name), "dmabuf%d:%zu", b->node, b->length);
	fd = anon_inode_getfd(name, &dmabuf_fops, b, O_RDWR | O_CLOEXEC);
	if (fd < 0) {
		struct file tmp = { .private_data = b };

		dmabuf_release(NULL, &tmp);
		return fd;
	}
	arg->dmabuf_fdesc = fd;
	return 0;
nomem:
	{
		struct file tmp = { .private_data = b };

		dmabuf_release(NULL, &tmp);
	}
	return -ENOMEM;
}
