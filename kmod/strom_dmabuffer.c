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
 * The node is validated before any allocation (reference pmemmap.c:646-650).
 */
#include <linux/anon_inodes.h>
#include <linux/file.h>
#include <linux/mm.h>
#include <linux/slab.h>

#include "strom_kmod.h"

#define SEG_ORDER (22 - PAGE_SHIFT)          /* 4 MiB segments */
#define SEG_SIZE (PAGE_SIZE << SEG_ORDER)

struct strom_dbuf_map {                  /* the segments as one controller sees them */
	struct device *dev;              /* held (get_device) */
	dma_addr_t *seg_dma;
};

struct strom_dma_buffer {
	size_t length;
	int node;
	int nsegs;
	struct mutex map_lock;
	int nmaps;
	struct strom_dbuf_map maps[STROM_MAX_ATTACH];
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
	if (!(vma->vm_flags & VM_SHARED))
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
		struct strom_dbuf_map *m = &b->maps[j];

		for (i = 0; i < b->nsegs; i++)
			if (m->seg_dma[i])
				dma_unmap_page(m->dev, m->seg_dma[i], SEG_SIZE, DMA_FROM_DEVICE);
		kfree(m->seg_dma);
		put_device(m->dev);
	}
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

/* the segment table of `b` as seen by `dev`, mapped on first use */
static struct strom_dbuf_map *dbuf_map_for(struct strom_dma_buffer *b, struct device *dev)
{
	struct strom_dbuf_map *m = NULL;
	dma_addr_t *seg;
	int i, j;

	mutex_lock(&b->map_lock);
	for (j = 0; j < b->nmaps; j++)
		if (b->maps[j].dev == dev) {
			m = &b->maps[j];
			goto out;
		}
	if (b->nmaps == ARRAY_SIZE(b->maps))
		goto out;
	seg = kmalloc_array(b->nsegs, sizeof(*seg), GFP_KERNEL | __GFP_ZERO);
	if (!seg)
		goto out;
	for (i = 0; i < b->nsegs; i++) {
		seg[i] = dma_map_page(dev, b->segs[i], 0, SEG_SIZE, DMA_FROM_DEVICE);
		if (dma_mapping_error(dev, seg[i])) {
			while (i-- > 0)
				dma_unmap_page(dev, seg[i], SEG_SIZE, DMA_FROM_DEVICE);
			kfree(seg);
			goto out;
		}
	}
	m = &b->maps[b->nmaps];
	m->dev = get_device(dev);
	m->seg_dma = seg;
	b->nmaps++;
out:
	mutex_unlock(&b->map_lock);
	return m;
}

/* Bus address, for controller `dev`, of byte `off` of the DMA buffer behind
 * `filp`; *contig = bytes to the end of its segment. */
int strom_dma_buffer_dma(struct file *filp, struct device *dev, u64 off, u64 *addr, u64 *contig)
{
	struct strom_dma_buffer *b = filp->private_data;
	struct strom_dbuf_map *m;

	if (off >= b->length)
		return -EFAULT;
	m = dbuf_map_for(b, dev);
	if (!m)
		return -EIO;
	*addr = m->seg_dma[off / SEG_SIZE] + off % SEG_SIZE;
	*contig = SEG_SIZE - off % SEG_SIZE;
	return 0;
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
