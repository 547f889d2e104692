// SPDX-License-Identifier: GPL-2.0
/*
 * strom_task.c — DMA task table, WAIT, statistics.
 *
 * Semantics of the reference's strom_dma_task (kmod/nvme_strom.c:504-731,
 * 1123-1235, 1983-2028): refcount = 1 submitter + 1 per NVMe command, the
 * first error wins, a failed task outlives its last put on the session's
 * failed list until WAIT consumes it or the fd closes.  Ids are a 64-bit
 * counter, not kernel pointers; WAIT on an id that was never issued returns
 * -ENOENT (the reference returned success); WAIT can carry a timeout.
 */
#include <linux/hashtable.h>
#include <linux/sched/signal.h>
#include <linux/slab.h>

#include "strom_kmod.h"

struct strom_stats strom_stats;

static struct {
	spinlock_t lock;
	wait_queue_head_t wq;
	struct hlist_head running;
} slots[STROM_NR_TASK_SLOTS];

static atomic64_t next_id = ATOMIC64_INIT(0);

static inline unsigned int slot_of(unsigned long id)
{
	return hash_long(id, 9);
}

void strom_task_init(void)
{
	int i;

	for (i = 0; i < STROM_NR_TASK_SLOTS; i++) {
		spin_lock_init(&slots[i].lock);
		init_waitqueue_head(&slots[i].wq);
		INIT_HLIST_HEAD(&slots[i].running);
	}
}

struct strom_task *strom_task_create(struct strom_session *s, struct file *filp,
				     struct strom_gpumap *gmap)
{
	struct strom_task *t = kzalloc(sizeof(*t), GFP_KERNEL);
	unsigned long flags;
	unsigned int k;

	if (!t)
		return NULL;
	t->id = atomic64_inc_return(&next_id);
	t->sess = s;
	get_file(s->filp);      /* the session outlives its tasks */
	atomic_set(&t->refcnt, 1);
	t->gmap = gmap;
	t->filp = filp;
	t->t_start = strom_tsc();
	INIT_LIST_HEAD(&t->failed_node);
	k = slot_of(t->id);
	spin_lock_irqsave(&slots[k].lock, flags);
	hlist_add_head(&t->node, &slots[k].running);
	spin_unlock_irqrestore(&slots[k].lock, flags);
	return t;
}

void strom_task_get(struct strom_task *t)
{
	STROM_ASSERT(!t->frozen);
	STROM_ASSERT(atomic_read(&t->refcnt) > 0);
	atomic_inc(&t->refcnt);
}

/* may run in IRQ context (NVMe completion) */
void strom_task_put(struct strom_task *t, long status)
{
	unsigned int k = slot_of(t->id);
	struct strom_gpumap *gmap;
	struct strom_volume *vol;
	struct file *filp, *dbuf, *sfilp;
	unsigned long flags;
	bool failed;

	if (status)
		cmpxchg(&t->status, 0, status);
	if (!atomic_dec_and_test(&t->refcnt))
		return;
	/* The last reference.  Everything the record holds is taken out BEFORE
	 * it becomes visible on the failed list: from that moment a WAIT on
	 * another CPU may consume and kfree it (found by the TSAN run of the
	 * kernel-model harness, kmod/testshim/kmod_exec.c). */
	gmap = t->gmap;
	filp = t->filp;
	dbuf = t->dbuf_filp;
	vol = t->vol;
	sfilp = t->sess->filp;
	t->gmap = NULL;
	t->filp = NULL;
	t->dbuf_filp = NULL;
	t->vol = NULL;
	failed = t->status != 0;
	spin_lock_irqsave(&slots[k].lock, flags);
	hlist_del(&t->node);
	if (failed) {
		spin_lock(&t->sess->lock);
		list_add_tail(&t->failed_node, &t->sess->failed);
		spin_unlock(&t->sess->lock);
	}
	spin_unlock_irqrestore(&slots[k].lock, flags);
	wake_up_all(&slots[k].wq);
	if (!failed)
		kfree(t);
	/* t may be gone now */
	if (gmap)
		strom_gpumap_put(gmap);      /* teardown runs on a workqueue */
	if (filp)
		fput(filp);
	if (dbuf)
		fput(dbuf);
	strom_volume_put(vol);              /* frees on a workqueue if last */
	/* last: the session (and a failed record on its list) lives until WAIT
	 * or release(), which this reference holds off */
	fput(sfilp);
}

static bool task_running(unsigned long id)
{
	unsigned int k = slot_of(id);
	struct strom_task *t;
	unsigned long flags;
	bool found = false;

	spin_lock_irqsave(&slots[k].lock, flags);
	hlist_for_each_entry(t, &slots[k].running, node)
		if (t->id == id) {
			found = true;
			break;
		}
	spin_unlock_irqrestore(&slots[k].lock, flags);
	return found;
}

static struct strom_task *take_failed(struct strom_session *s, unsigned long id)
{
	struct strom_task *t, *n;

	spin_lock_irq(&s->lock);
	list_for_each_entry_safe(t, n, &s->failed, failed_node)
		if (t->id == id) {
			list_del(&t->failed_node);
			spin_unlock_irq(&s->lock);
			return t;
		}
	spin_unlock_irq(&s->lock);
	return NULL;
}

int strom_task_wait(unsigned long id, long *status, long timeout)
{
	unsigned int k = slot_of(id);
	u64 t0 = strom_tsc();
	long left;

	*status = 0;
	if (!id || id > (unsigned long)atomic64_read(&next_id))
		return -ENOENT;
	left = wait_event_interruptible_timeout(slots[k].wq, !task_running(id), timeout);
	atomic64_inc(&strom_stats.nr_wait_dtask);
	atomic64_add(strom_tsc() - t0, &strom_stats.clk_wait_dtask);
	if (left == -ERESTARTSYS)
		return -EINTR;
	if (left == 0 && task_running(id))
		return -ETIME;
	return 0;   /* finished; failures are consumed by strom_task_wait_session */
}

int strom_session_reclaim(struct strom_session *s)
{
	struct strom_task *t, *n;
	int cnt = 0;

	spin_lock_irq(&s->lock);
	list_for_each_entry_safe(t, n, &s->failed, failed_node) {
		list_del(&t->failed_node);
		kfree(t);
		cnt++;
	}
	spin_unlock_irq(&s->lock);
	return cnt;
}

/* WAIT variant that also consumes a failed record from the caller's session */
int strom_task_wait_session(struct strom_session *s, unsigned long id, long *status,
			    long timeout)
{
	int rc = strom_task_wait(id, status, timeout);
	struct strom_task *t;

	if (rc)
		return rc;
	t = take_failed(s, id);
	if (t) {
		*status = t->status;
		kfree(t);
		return -EIO;
	}
	return 0;
}

void strom_stat_inflight_inc(void)
{
	s64 cur = atomic64_inc_return(&strom_stats.cur_dma_count);
	s64 mx = atomic64_read(&strom_stats.max_dma_count);

	while (cur > mx) {
		s64 old = atomic64_cmpxchg(&strom_stats.max_dma_count, mx, cur);

		if (old == mx)
			break;
		mx = old;
	}
}

int strom_stat_info(struct strom_stat_info *a)
{
	int i;

	if (a->version != 1)
		return -EINVAL;
	if (!strom_stat_level)
		return -ENODATA;
	a->has_debug = strom_stat_level >= 2;
	a->tsc = strom_tsc();
	a->nr_ssd2gpu = atomic64_read(&strom_stats.nr_ssd2gpu);
	a->clk_ssd2gpu = atomic64_read(&strom_stats.clk_ssd2gpu);
	a->nr_setup_prps = atomic64_read(&strom_stats.nr_setup_prps);
	a->clk_setup_prps = atomic64_read(&strom_stats.clk_setup_prps);
	a->nr_submit_dma = atomic64_read(&strom_stats.nr_submit_dma);
	a->clk_submit_dma = atomic64_read(&strom_stats.clk_submit_dma);
	a->nr_wait_dtask = atomic64_read(&strom_stats.nr_wait_dtask);
	a->clk_wait_dtask = atomic64_read(&strom_stats.clk_wait_dtask);
	a->nr_wrong_wakeup = atomic64_read(&strom_stats.nr_wrong_wakeup);
	a->cur_dma_count = atomic64_read(&strom_stats.cur_dma_count);
	a->max_dma_count = atomic64_xchg(&strom_stats.max_dma_count, a->cur_dma_count);
	for (i = 0; i < 4; i++) {
		u64 *nr = &a->nr_debug1 + 2 * i, *clk = &a->clk_debug1 + 2 * i;

		*nr = a->has_debug ? atomic64_read(&strom_stats.nr_debug[i]) : 0;
		*clk = a->has_debug ? atomic64_read(&strom_stats.clk_debug[i]) : 0;
	}
	return 0;
}
