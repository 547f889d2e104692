// SPDX-License-Identifier: GPL-2.0
/*
 * strom_main.c — module lifecycle, /dev + /proc entry points, ioctl dispatch.
 *
 * Mirrors the reference's /proc/nvme-strom fops (kmod/nvme_strom.c:2030-2157)
 * and init/exit (:2159-2217) with modern registration: a misc device
 * (/dev/nvme-strom, mode 0444) plus the legacy /proc entry for old binaries.
 * read() returns the version signature; release() reclaims failed tasks the
 * opener never waited for.  SET_ROUTE (admin) registers the namespaces behind
 * an md raid0 array or an NVMe multipath head.  MAP_GPU_MEMORY (VA only) is
 * answered -EOPNOTSUPP:
 * the kernel cannot resolve an amdgpu VA to its buffer object, so libstrom
 * exports the range as a dma-buf and calls MAP_GPU_DMABUF instead.
 */
#include <linux/miscdevice.h>
#include <linux/module.h>
#include <linux/proc_fs.h>
#include <linux/slab.h>
#include <linux/string.h>
#include <linux/uaccess.h>

#include "strom_kmod.h"

int strom_verbose;
module_param_named(verbose, strom_verbose, int, 0644);
MODULE_PARM_DESC(verbose, "0 quiet, 1 events, 2 with function:line");
int strom_stat_level = 1;
module_param_named(stat_info, strom_stat_level, int, 0644);
MODULE_PARM_DESC(stat_info, "0 off, 1 on, 2 with debug counters");

static const char strom_signature[] =
	"version: 0.1.0-mi355x\ntarget: " UTS_RELEASE "\nbuild: " __DATE__ " " __TIME__ "\n";

static int strom_open(struct inode *inode, struct file *filp)
{
	struct strom_session *s = kzalloc(sizeof(*s), GFP_KERNEL);

	if (!s)
		return -ENOMEM;
	INIT_LIST_HEAD(&s->failed);
	spin_lock_init(&s->lock);
	s->filp = filp;
	filp->private_data = s;
	return 0;
}

static int strom_release(struct inode *inode, struct file *filp)
{
	struct strom_session *s = filp->private_data;
	int n = strom_session_reclaim(s);

	if (n)
		pr_notice("nvme-strom: %d failed task(s) reclaimed on close\n", n);
	kfree(s);
	return 0;
}

static ssize_t strom_read(struct file *filp, char __user *buf, size_t len, loff_t *pos)
{
	return simple_read_from_buffer(buf, len, pos, strom_signature,
				       sizeof(strom_signature) - 1);
}

#define COPY_IN(type)                                                     \
	type karg;                                                        \
	if (copy_from_user(&karg, uarg, sizeof(karg)))                    \
		return -EFAULT

static long strom_ioctl(struct file *filp, unsigned int cmd, unsigned long arg)
{
	struct strom_session *s = filp->private_data;
	void __user *uarg = (void __user *)arg;
	long rc;

	switch (cmd) {
	case STROM_IOCTL__CHECK_FILE: {
		COPY_IN(struct strom_check_file);
		rc = strom_check_file(&karg);
		if (!rc && copy_to_user(uarg, &karg, sizeof(karg)))
			rc = -EFAULT;
		return rc;
	}
	case STROM_IOCTL__MAP_GPU_MEMORY:
		return -EOPNOTSUPP;   /* libstrom translates to MAP_GPU_DMABUF */
	case STROM_IOCTL__MAP_GPU_DMABUF: {
		COPY_IN(struct strom_map_gpu_dmabuf);
		rc = strom_map_dmabuf(&karg);
		if (!rc && copy_to_user(uarg, &karg, sizeof(karg)))
			rc = -EFAULT;
		return rc;
	}
	case STROM_IOCTL__UNMAP_GPU_MEMORY: {
		COPY_IN(struct strom_unmap_gpu_memory);
		return strom_unmap_gpu(karg.handle);
	}
	case STROM_IOCTL__LIST_GPU_MEMORY:
		return strom_list_gpu(uarg);
	case STROM_IOCTL__INFO_GPU_MEMORY:
		return strom_info_gpu(uarg);
	case STROM_IOCTL__ALLOC_DMA_BUFFER: {
		COPY_IN(struct strom_alloc_dma_buffer);
		rc = strom_alloc_dma_buffer(&karg);
		if (!rc && copy_to_user(uarg, &karg, sizeof(karg)))
			rc = -EFAULT;
		return rc;
	}
	case STROM_IOCTL__MEMCPY_SSD2GPU:
		return strom_memcpy_ssd2gpu(s, uarg);
	case STROM_IOCTL__MEMCPY_SSD2RAM:
		return strom_memcpy_ssd2ram(s, uarg);
	case STROM_IOCTL__MEMCPY_SSD2GPU_EXTENTS:
		return strom_memcpy_ssd2gpu_extents(s, uarg);
	case STROM_IOCTL__MEMCPY_WAIT: {
		COPY_IN(struct strom_memcpy_wait);
		rc = strom_task_wait_session(s, karg.dma_task_id, &karg.status,
					     MAX_SCHEDULE_TIMEOUT);
		if (copy_to_user(uarg, &karg, sizeof(karg)))
			rc = -EFAULT;
		return rc;
	}
	case STROM_IOCTL__MEMCPY_WAIT_TIMED: {
		COPY_IN(struct strom_memcpy_wait_timed);
		rc = strom_task_wait_session(s, karg.dma_task_id, &karg.status,
					     nsecs_to_jiffies(karg.timeout_ns));
		if (copy_to_user(uarg, &karg, sizeof(karg)))
			rc = -EFAULT;
		return rc;
	}
	case STROM_IOCTL__SET_ROUTE: {
		struct strom_set_route *r = memdup_user(uarg, sizeof(*r));

		if (IS_ERR(r))
			return PTR_ERR(r);
		rc = strom_set_route(r);
		kfree(r);
		return rc;
	}
	case STROM_IOCTL__STAT_INFO: {
		COPY_IN(struct strom_stat_info);
		rc = strom_stat_info(&karg);
		if (!rc && copy_to_user(uarg, &karg, sizeof(karg)))
			rc = -EFAULT;
		return rc;
	}
	default:
		return -EINVAL;
	}
}

static const struct file_operations strom_fops = {
	.owner = THIS_MODULE,
	.open = strom_open,
	.release = strom_release,
	.read = strom_read,
	.unlocked_ioctl = strom_ioctl,
	.compat_ioctl = compat_ptr_ioctl,
};

static const struct proc_ops strom_proc_ops = {
	.proc_open = strom_open,
	.proc_release = strom_release,
	.proc_read = strom_read,
	.proc_ioctl = strom_ioctl,
};

static struct miscdevice strom_misc = {
	.minor = MISC_DYNAMIC_MINOR,
	.name = STROM_NAME,
	.fops = &strom_fops,
	.mode = 0444,
};

static struct proc_dir_entry *strom_proc;

static int __init nvme_strom_init(void)
{
	int rc;

	strom_task_init();
	rc = strom_gpumap_init();
	if (rc)
		return rc;
	rc = strom_route_init();
	if (rc)
		goto out_map;
	rc = misc_register(&strom_misc);
	if (rc)
		goto out_route;
	strom_proc = proc_create(STROM_NAME, 0444, NULL, &strom_proc_ops);
	if (!strom_proc) {
		rc = -ENOMEM;
		goto out_misc;
	}
	pr_info("nvme-strom: MI355X provider loaded (/dev/%s, /proc/%s)\n", STROM_NAME,
		STROM_NAME);
	return 0;
out_misc:
	misc_deregister(&strom_misc);
out_route:
	strom_route_exit();
out_map:
	strom_gpumap_exit();
	return rc;
}

static void __exit nvme_strom_exit(void)
{
	proc_remove(strom_proc);
	misc_deregister(&strom_misc);
	strom_route_exit();
	strom_gpumap_exit();
	pr_info("nvme-strom: unloaded\n");
}

module_init(nvme_strom_init);
module_exit(nvme_strom_exit);
MODULE_AUTHOR("strom-mi355x");
MODULE_DESCRIPTION("SSD-to-GPU direct DMA for AMD Instinct MI355X (dma-buf P2P)");
MODULE_VERSION("0.1.0");
MODULE_LICENSE("GPL v2");
#if LINUX_VERSION_CODE >= KERNEL_VERSION(6, 13, 0)
MODULE_IMPORT_NS("DMA_BUF");        /* namespaces are string literals since 6.13 */
#else
MODULE_IMPORT_NS(DMA_BUF);
#endif
