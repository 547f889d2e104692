// SPDX-License-Identifier: GPL-2.0
/*
 * strom_route.c — which NVMe namespaces (queues, DMA devices) serve a file.
 *
 * The reference decoded volumes through private kernel structures: struct
 * nvme_ns for the namespace and md's mddev/r0conf for raid0 members
 * (kmod/nvme_strom.c:185-367, :755-820, vendored headers in
 * kmod/514.6.2.el7/).  Here:
 *   - a plain NVMe namespace disk (blk-mq queue, "nvme*") is used directly;
 *   - an md raid0 array or a native-multipath head (bio-based "nvmeXnY" whose
 *     paths are hidden "nvmeXcYnZ" disks) needs a ROUTE registered by
 *     userspace (STROM_IOCTL__SET_ROUTE, CAP_SYS_ADMIN): the geometry in the
 *     shared core's struct strom_raid0 plus the member namespaces, by dev_t
 *     or, for hidden path disks, by "<pci>/<ctrl>/<disk>" name.  Every member
 *     must be a blk-mq NVMe namespace, and the geometry must be consistent
 *     (strom_core_raid0_check) and fit the members' capacity and the
 *     volume's size.  A single-path alias must be named as a path of the
 *     head ("nvme<S>c<C>n<H>" for head "nvme<S>n<H>": same subsystem and
 *     head instance), answer NVME_IOCTL_ID with the head's nsid and have
 *     exactly the head's capacity.  That md members
 *     really are the array's slaves is NOT verifiable through exported
 *     interfaces (md's rdev list and the holder links are private): it is
 *     asserted by the administrator who registers the route
 *     (CAP_SYS_ADMIN), and a wrong route reads wrong sectors — the same
 *     trust as writing to the member block devices directly.
 * Members are held by their struct device (get_device), and so is each
 * member's PCI function; a member removed while a route exists fails the
 * requests sent to it, like any I/O to a vanished disk.  Unregistered
 * (plain namespace) entries are a cache and are revalidated on every
 * lookup: a disk that went away, or a new disk instance reusing the dev_t
 * (diskseq), drops the stale entry.
 */
#include <linux/blkdev.h>
#include <linux/capability.h>
#include <linux/device.h>
#include <linux/dmapool.h>
#include <linux/log2.h>
#include <linux/pci.h>
#include <linux/slab.h>

#include "strom_kmod.h"

/* Native multipath names a head "nvme<S>n<H>" and each of its paths
 * "nvme<S>c<C>n<H>" (S the subsystem instance, H the head's): a path belongs
 * to a head exactly when S and H agree. */
static bool path_of_head(const char *head, const char *path)
{
	unsigned int s1, h1, s2, c2, h2;
	char tail;

	if (sscanf(head, "nvme%un%u%c", &s1, &h1, &tail) != 2)
		return false;
	if (sscanf(path, "nvme%uc%un%u%c", &s2, &c2, &h2, &tail) != 3)
		return false;
	return s1 == s2 && h1 == h2;
}

static LIST_HEAD(routes);
static DEFINE_MUTEX(routes_lock);

/* nearest PCI ancestor: the NVMe controller function that masters the DMA */
static struct device *pci_ancestor(struct device *d)
{
	for (; d; d = d->parent)
		if (dev_is_pci(d))
			return d;
	return NULL;
}

static int member_from_disk(struct strom_member *m, struct device *disk_dev)
{
	struct gendisk *disk = dev_to_disk(disk_dev);
	struct request_queue *q = disk->queue;
	int nsid;

	if (strncmp(disk->disk_name, "nvme", 4) || !queue_is_mq(q) || !disk->fops->ioctl)
		return -EOPNOTSUPP;
	/* the namespace answers NVME_IOCTL_ID with its nsid (reference CHECK_FILE
	 * used the same ping) */
	nsid = disk->fops->ioctl(disk->part0, BLK_OPEN_READ, NVME_IOCTL_ID, 0);
	if (nsid <= 0)
		return nsid < 0 ? nsid : -EOPNOTSUPP;
	m->dma_dev = pci_ancestor(disk_dev);
	if (!m->dma_dev)
		return -EOPNOTSUPP;
	get_device(m->dma_dev);
	m->disk_dev = get_device(disk_dev);
	m->disk = disk;
	m->q = q;
	m->nsid = nsid;
	m->lba_shift = ilog2(queue_logical_block_size(q));
	m->max_bytes = min_t(u32, queue_max_hw_sectors(q) << SECTOR_SHIFT, STROM_CORE_MAX_REQ);
	m->nr_sects = get_capacity(disk);
	m->prp_pool = dma_pool_create("strom_prp", m->dma_dev, STROM_CORE_PAGE, STROM_CORE_PAGE, 0);
	if (!m->prp_pool) {
		put_device(m->disk_dev);
		put_device(m->dma_dev);
		m->disk_dev = NULL;
		m->dma_dev = NULL;
		return -ENOMEM;
	}
	return 0;
}

static void member_release(struct strom_member *m)
{
	if (m->prp_pool)
		dma_pool_destroy(m->prp_pool);
	if (m->disk_dev)
		put_device(m->disk_dev);
	if (m->dma_dev)
		put_device(m->dma_dev);
	m->prp_pool = NULL;
	m->disk_dev = NULL;
	m->dma_dev = NULL;
}

/* "<pci>/<ctrl>/<disk>": PCI function -> controller device -> path disk */
static struct device *find_named_disk(const char *name)
{
	char buf[40], *ctrl, *disk;
	struct device *pdev, *cdev, *ddev = NULL;

	if (strscpy(buf, name, sizeof(buf)) < 0)
		return NULL;
	ctrl = strchr(buf, '/');
	if (!ctrl)
		return NULL;
	*ctrl++ = 0;
	disk = strchr(ctrl, '/');
	if (!disk)
		return NULL;
	*disk++ = 0;
	pdev = bus_find_device_by_name(&pci_bus_type, NULL, buf);
	if (!pdev)
		return NULL;
	cdev = device_find_child_by_name(pdev, ctrl);
	put_device(pdev);
	if (!cdev)
		return NULL;
	ddev = device_find_child_by_name(cdev, disk);
	put_device(cdev);
	if (ddev && (!ddev->class || strcmp(ddev->class->name, "block"))) {
		put_device(ddev);
		ddev = NULL;
	}
	return ddev;
}

static struct device *find_disk_by_devt(dev_t devt)
{
	/* the disk is registered: open it by number for the lookup only */
#if LINUX_VERSION_CODE >= KERNEL_VERSION(6, 9, 0)
	struct file *f = bdev_file_open_by_dev(devt, BLK_OPEN_READ, NULL, NULL);
	struct device *d;

	if (IS_ERR(f))
		return NULL;
	d = get_device(disk_to_dev(file_bdev(f)->bd_disk));
	fput(f);
	return d;
#else
	struct bdev_handle *h = bdev_open_by_dev(devt, BLK_OPEN_READ, NULL, NULL);
	struct device *d;

	if (IS_ERR(h))
		return NULL;
	d = get_device(disk_to_dev(h->bdev->bd_disk));
	bdev_release(h);
	return d;
#endif
}

static struct workqueue_struct *route_wq;

/* the last reference can drop in an NVMe completion (IRQ context, through
 * the task), but dma_pool_destroy and put_device may sleep */
static void volume_free_work(struct work_struct *w)
{
	struct strom_volume *v = container_of(w, struct strom_volume, free_work);
	int i;

	for (i = 0; i < v->nmembers; i++)
		member_release(&v->m[i]);
	kfree(v);
}

static void volume_free(struct kref *ref)
{
	struct strom_volume *v = container_of(ref, struct strom_volume, ref);

	queue_work(route_wq, &v->free_work);
}

static struct strom_volume *volume_alloc(dev_t devt)
{
	struct strom_volume *v = kzalloc(sizeof(*v), GFP_KERNEL);

	if (!v)
		return NULL;
	kref_init(&v->ref);
	INIT_WORK(&v->free_work, volume_free_work);
	v->devt = devt;
	return v;
}

void strom_volume_put(struct strom_volume *v)
{
	if (v)
		kref_put(&v->ref, volume_free);
}

/* an unregistered entry describes the disk instance it was built from */
static bool volume_stale(const struct strom_volume *v, struct gendisk *disk)
{
	return !v->registered &&
	       (v->m[0].disk != disk || v->diskseq != disk->diskseq || !disk_live(disk));
}

/* under routes_lock: the entry for devt, a stale cached one unlinked into *stale */
static struct strom_volume *route_lookup(dev_t devt, struct gendisk *disk,
					 struct strom_volume **stale)
{
	struct strom_volume *v;

	list_for_each_entry(v, &routes, node) {
		if (v->devt != devt)
			continue;
		if (volume_stale(v, disk)) {
			list_del(&v->node);
			*stale = v;          /* the list's reference, dropped by the caller */
			return NULL;
		}
		kref_get(&v->ref);
		return v;
	}
	return NULL;
}

struct strom_volume *strom_volume_of_file(struct file *filp, int *err)
{
	struct inode *inode = file_inode(filp);
	struct super_block *sb = inode->i_sb;
	struct block_device *bdev = sb->s_bdev;
	struct strom_volume *v, *stale = NULL, *o;
	struct gendisk *disk;
	dev_t devt;
	int rc;

	*err = -EOPNOTSUPP;
	if (!bdev)
		return NULL;
	disk = bdev->bd_disk;
	devt = disk_devt(disk);
	mutex_lock(&routes_lock);
	v = route_lookup(devt, disk, &stale);
	mutex_unlock(&routes_lock);
	strom_volume_put(stale);                      /* in-flight tasks hold their own */
	if (v) {
		*err = 0;
		return v;
	}
	/* unregistered: only a plain blk-mq namespace can be served */
	v = volume_alloc(devt);
	if (!v) {
		*err = -ENOMEM;
		return NULL;
	}
	rc = member_from_disk(&v->m[0], disk_to_dev(disk));
	if (rc) {
		kfree(v);
		if (!queue_is_mq(disk->queue))
			prDebug("%s: bio-based volume (md / nvme multipath head): register a route",
				disk->disk_name);
		*err = rc;
		return NULL;
	}
	v->nmembers = 1;
	v->diskseq = disk->diskseq;
	/* cache it (unregistered entries live until a route replaces them, the
	 * disk goes away, or the module unloads) */
	stale = NULL;
	mutex_lock(&routes_lock);
	o = route_lookup(devt, disk, &stale);
	if (o) {                                      /* lost a race: use theirs */
		mutex_unlock(&routes_lock);
		strom_volume_put(stale);
		strom_volume_put(v);
		*err = 0;
		return o;
	}
	kref_get(&v->ref);                            /* the list's reference */
	list_add_tail(&v->node, &routes);
	mutex_unlock(&routes_lock);
	strom_volume_put(stale);
	*err = 0;
	return v;
}

int strom_set_route(const struct strom_set_route *r)
{
	const dev_t vdev = MKDEV(r->volume_major, r->volume_minor);
	struct strom_volume *v, *old = NULL;
	struct device *vd;
	sector_t vol_sects;
	u32 i, z;
	int rc;

	if (!capable(CAP_SYS_ADMIN))
		return -EPERM;
	if (r->nmembers > STROM_ROUTE_MAX_DISKS || r->nzones > STROM_ROUTE_MAX_ZONES)
		return -EINVAL;
	vd = find_disk_by_devt(vdev);
	if (!vd)
		return -ENODEV;
	vol_sects = get_capacity(dev_to_disk(vd));
	put_device(vd);
	if (!r->nmembers) {
		mutex_lock(&routes_lock);
		list_for_each_entry(v, &routes, node)
			if (v->devt == vdev) {
				list_del(&v->node);
				old = v;
				break;
			}
		mutex_unlock(&routes_lock);
		strom_volume_put(old);          /* in-flight tasks keep their own ref */
		return old ? 0 : -ENOENT;
	}
	v = volume_alloc(vdev);
	if (!v)
		return -ENOMEM;
	v->registered = true;
	for (i = 0; i < r->nmembers; i++) {
		struct device *md;

		if (r->member_major[i])
			md = find_disk_by_devt(MKDEV(r->member_major[i], r->member_minor[i]));
		else
			md = find_named_disk(r->member_name[i]);
		if (!md) {
			rc = -ENODEV;
			goto fail;
		}
		rc = member_from_disk(&v->m[i], md);
		put_device(md);                 /* member_from_disk took its own */
		if (rc)
			goto fail;
		v->nmembers++;
	}
	if (r->chunk_sects) {
		struct strom_raid0 *g = &v->geo;

		v->raid0 = true;
		g->chunk_sects = r->chunk_sects;
		g->nzones = r->nzones;
		g->ndisks = r->nmembers;
		for (z = 0; z < r->nzones; z++) {
			g->zone_end[z] = r->zone_end[z];
			g->zone_dev_start[z] = r->zone_dev_start[z];
			g->zone_nb_dev[z] = r->zone_nb_dev[z];
			memcpy(g->zone_devs[z], r->zone_devs[z], STROM_ROUTE_MAX_DISKS);
		}
		for (i = 0; i < r->nmembers; i++)
			g->data_offset[i] = r->data_offset[i];
		rc = strom_core_raid0_check(g);
		if (rc)
			goto fail;
		/* the array is no larger than the volume, and every zone's rows
		 * stay inside every member it stripes over */
		rc = -EINVAL;
		if (g->zone_end[g->nzones - 1] > vol_sects)
			goto fail;
		for (z = 0; z < g->nzones; z++) {
			const u64 zs = z ? g->zone_end[z - 1] : 0;
			const u64 rows = (g->zone_end[z] - zs) / ((u64)g->zone_nb_dev[z] * g->chunk_sects);
			const u64 dev_end = g->zone_dev_start[z] + rows * g->chunk_sects;
			u32 k;

			for (k = 0; k < g->zone_nb_dev[z]; k++) {
				const u32 mbr = g->zone_devs[z][k];

				if (dev_end + g->data_offset[mbr] > v->m[mbr].nr_sects)
					goto fail;
			}
		}
	} else {
		/* a path alias of a multipath head: one member that is a path of
		 * THIS head by name (same subsystem and head instance), answers
		 * the head's nsid and has exactly its capacity */
		int head_nsid = -1;

		rc = -EINVAL;
		if (r->nmembers != 1 || v->m[0].nr_sects != vol_sects)
			goto fail;
		vd = find_disk_by_devt(vdev);
		if (vd) {
			struct gendisk *hd = dev_to_disk(vd);

			/* only an NVMe head is asked NVME_IOCTL_ID (never another
			 * driver's ioctl, e.g. dm passing it through) */
			if (path_of_head(hd->disk_name, v->m[0].disk->disk_name) && hd->fops &&
			    hd->fops->ioctl)
				head_nsid = hd->fops->ioctl(hd->part0, BLK_OPEN_READ, NVME_IOCTL_ID, 0);
			put_device(vd);
		}
		if (head_nsid <= 0 || (u32)head_nsid != v->m[0].nsid)
			goto fail;
	}
	mutex_lock(&routes_lock);
	list_for_each_entry(old, &routes, node)
		if (old->devt == vdev) {
			list_del(&old->node);
			break;
		}
	if (&old->node == &routes)
		old = NULL;
	list_add(&v->node, &routes);
	mutex_unlock(&routes_lock);
	strom_volume_put(old);
	prDebug("route %u:%u -> %d member(s)%s", r->volume_major, r->volume_minor, v->nmembers,
		v->raid0 ? " raid0" : "");
	return 0;
fail:
	strom_volume_put(v);
	return rc;
}

int strom_route_init(void)
{
	route_wq = alloc_workqueue("strom_route", WQ_UNBOUND, 0);
	return route_wq ? 0 : -ENOMEM;
}

void strom_route_exit(void)
{
	struct strom_volume *v, *n;

	mutex_lock(&routes_lock);
	list_for_each_entry_safe(v, n, &routes, node) {
		list_del(&v->node);
		strom_volume_put(v);
	}
	mutex_unlock(&routes_lock);
	/* live tasks hold module references, so only queued frees remain */
	destroy_workqueue(route_wq);
}
