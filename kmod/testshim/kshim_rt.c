/* kshim_rt.c — userspace implementation of the kernel model in kshim.h.
 *
 * The real kmod/strom_*.c sources are linked against this file and driven
 * through their misc-device fops (open / ioctl / read / release), so the
 * kernel provider's submission, completion, task lifetime, dma-buf import,
 * page-cache and error paths EXECUTE on the CPU ("the P2P
 * provider's kernel glue has never run").  The world it provides:
 *
 *  - NVMe controllers (a PCI function with its own IOMMU domain, a thread
 *    that fetches queued requests — optionally out of order or held — and
 *    validates each READ against the NVMe spec before moving bytes:
 *    opcode, nsid, slba/nlb against capacity, PRP1 dword alignment, PRP2 as
 *    page pointer or list pointer, list entries page aligned, every address
 *    translated through the issuing controller's IOMMU).  Completions run
 *    the request's end_io in "IRQ context".
 *  - namespaces, md raid0 arrays (own striping model, not strom_core's),
 *    NVMe multipath heads with hidden path disks, partitions, per-bdev
 *    diskstats.
 *  - an ext4-like filesystem: per-file block map (holes allowed), a page
 *    cache with clean and dirty pages over a logical content that differs
 *    from the device blocks until written back.
 *  - a dma-buf exporter ("VRAM" split into several segments placed at
 *    scattered bus addresses), whose pin/map/unmap/unpin assert the
 *    reservation lock like dma_resv_assert_held.
 *  - files with refcounts and deferred release (fput from IRQ context),
 *    an fd table, anon inodes, VMAs with fault handlers, workqueues.
 *
 * Contract checks (counted as violations, reported by ksim_counters()):
 * sleeping (mutex, wait, GFP_KERNEL, copy_*_user, resv lock) in IRQ context
 * or under a spinlock; dma-buf pin/map without the resv lock; DMA to bus
 * addresses not mapped for the controller; unmap of unmapped ranges;
 * dma_pool_destroy with live blocks; put_device underflow; alloc on an
 * invalid NUMA node; and leak counters for allocations, pages, IOMMU
 * mappings, requests, device and module references.
 */
#define _GNU_SOURCE
#include "kshim.h"

#include <pthread.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "kshim_sim.h"

/* ------------------------------------------------------------ context */
static __thread int t_in_irq;
static __thread int t_spin_depth;
static __thread int t_resv_held;
static __thread unsigned int t_euid = 1000;
static int g_admin;
static volatile int g_signal;
static int g_verbose;

static pthread_mutex_t g_viol_m = PTHREAD_MUTEX_INITIALIZER;
static char g_viol_msg[512];
static struct ksim_counters g_cnt;          /* updated with __atomic ops */

#define CNT_ADD(f, v) __atomic_add_fetch(&g_cnt.f, (v), __ATOMIC_SEQ_CST)

static void violation(const char *fmt, ...)
{
	va_list ap;

	pthread_mutex_lock(&g_viol_m);
	va_start(ap, fmt);
	vsnprintf(g_viol_msg, sizeof(g_viol_msg), fmt, ap);
	va_end(ap);
	fprintf(stderr, "kshim VIOLATION: %s\n", g_viol_msg);
	pthread_mutex_unlock(&g_viol_m);
	CNT_ADD(violations, 1);
}

void kshim_bug(const char *what, const char *file, int line)
{
	fprintf(stderr, "kshim BUG: %s at %s:%d\n", what, file, line);
	abort();
}

void kshim_warn(const char *what, const char *file, int line)
{
	violation("WARN_ON(%s) at %s:%d", what, file, line);
}

static void check_sleepable(const char *what, const char *file, int line)
{
	if (t_in_irq)
		violation("%s in IRQ context (%s:%d)", what, file ? file : "?", line);
	if (t_spin_depth)
		violation("%s under a spinlock (%s:%d)", what, file ? file : "?", line);
}

void kshim_might_sleep(const char *file, int line)
{
	check_sleepable("might_sleep", file, line);
}

void kshim_printk(const char *fmt, ...)
{
	va_list ap;

	CNT_ADD(printk, 1);
	if (!g_verbose)
		return;
	va_start(ap, fmt);
	vfprintf(stderr, fmt, ap);
	va_end(ap);
}

u64 kshim_now_ns(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (u64)ts.tv_sec * 1000000000ull + ts.tv_nsec;
}

bool kshim_signal_pending(void)
{
	return __atomic_load_n(&g_signal, __ATOMIC_SEQ_CST);
}

/* the kernel reads jiffies racily by design; the model keeps it constant
 * (accounting start times only) so TSAN sees no artificial race */
unsigned long jiffies;

unsigned long nsecs_to_jiffies(u64 n)
{
	return n / (1000000000ull / HZ);
}

u64 rdtsc_ordered(void)
{
	return __builtin_ia32_rdtsc();
}

/* ------------------------------------------------------------ user memory */
static pthread_mutex_t g_poison_m = PTHREAD_MUTEX_INITIALIZER;
static struct { const char *p; size_t n; } g_poison[8];
static int g_npoison;

bool kshim_uaccess_ok(const void *p, size_t n)
{
	bool ok = (uintptr_t)p >= 4096;
	int i;

	pthread_mutex_lock(&g_poison_m);
	for (i = 0; ok && i < g_npoison; i++)
		if ((const char *)p < g_poison[i].p + g_poison[i].n && g_poison[i].p < (const char *)p + n)
			ok = false;
	pthread_mutex_unlock(&g_poison_m);
	return ok;
}

void ksim_poison_user(const void *p, size_t n)
{
	pthread_mutex_lock(&g_poison_m);
	if (p == NULL)
		g_npoison = 0;
	else if (g_npoison < 8)
		g_poison[g_npoison].p = p, g_poison[g_npoison++].n = n;
	pthread_mutex_unlock(&g_poison_m);
}

unsigned long copy_from_user(void *to, const void __user *from, unsigned long n)
{
	check_sleepable("copy_from_user", NULL, 0);
	if (!kshim_uaccess_ok(from, n))
		return n;
	memcpy(to, from, n);
	return 0;
}

unsigned long copy_to_user(void __user *to, const void *from, unsigned long n)
{
	check_sleepable("copy_to_user", NULL, 0);
	if (!kshim_uaccess_ok(to, n))
		return n;
	memcpy(to, from, n);
	return 0;
}

unsigned long clear_user(void __user *to, unsigned long n)
{
	if (!kshim_uaccess_ok(to, n))
		return n;
	memset(to, 0, n);
	return 0;
}

#define KSIM_MD_MAX 32   /* md members (the route ABI allows STROM_ROUTE_MAX_DISKS) */

/* ------------------------------------------------------------ allocations */
static void *kalloc(size_t n, gfp_t gfp, bool zero)
{
	void *p;

	if (!(gfp & GFP_ATOMIC))
		check_sleepable("GFP_KERNEL allocation", NULL, 0);
	p = zero ? calloc(1, n ? n : 1) : malloc(n ? n : 1);
	if (p)
		CNT_ADD(kmallocs_live, 1);
	return p;
}

void *kzalloc(size_t n, gfp_t gfp)
{
	return kalloc(n, gfp, true);
}

void *kmalloc_array(size_t n, size_t size, gfp_t gfp)
{
	if (size && n > SIZE_MAX / size)
		return NULL;
	return kalloc(n * size, gfp, gfp & __GFP_ZERO);
}

void *krealloc_array(void *p, size_t n, size_t size, gfp_t gfp)
{
	void *q;

	if (size && n > SIZE_MAX / size)
		return NULL;
	if (!(gfp & GFP_ATOMIC))
		check_sleepable("GFP_KERNEL allocation", NULL, 0);
	q = realloc(p, n * size ? n * size : 1);
	if (q && !p)
		CNT_ADD(kmallocs_live, 1);
	return q;
}

void *kvmalloc_array(size_t n, size_t size, gfp_t gfp)
{
	return kmalloc_array(n, size, gfp);
}

void kfree(const void *p)
{
	if (!p)
		return;
	CNT_ADD(kmallocs_live, -1);
	free((void *)p);
}

void kvfree(const void *p)
{
	kfree(p);
}

void *memdup_user(const void __user *src, size_t n)
{
	void *p;

	if (!kshim_uaccess_ok(src, n))
		return ERR_PTR(-EFAULT);
	p = kalloc(n, GFP_KERNEL, false);
	if (!p)
		return ERR_PTR(-ENOMEM);
	memcpy(p, src, n);
	return p;
}

long strscpy(char *dst, const char *src, size_t count)
{
	size_t n = strnlen(src, count);

	if (!count)
		return -E2BIG;
	if (n == count) {
		memcpy(dst, src, count - 1);
		dst[count - 1] = 0;
		return -E2BIG;
	}
	memcpy(dst, src, n + 1);
	return (long)n;
}

ssize_t simple_read_from_buffer(void __user *to, size_t count, loff_t *ppos, const void *from,
				size_t available)
{
	loff_t pos = *ppos;
	size_t n;

	if (pos < 0)
		return -EINVAL;
	if ((size_t)pos >= available || !count)
		return 0;
	n = min(count, available - (size_t)pos);
	if (copy_to_user(to, (const char *)from + pos, n))
		return -EFAULT;
	*ppos = pos + n;
	return (ssize_t)n;
}

long compat_ptr_ioctl(struct file *file, unsigned int cmd, unsigned long arg)
{
	return -ENOIOCTLCMD;
}

unsigned int hash_long(unsigned long v, unsigned int bits)
{
	return bits ? (unsigned int)((v * 0x61C8864680B583EBull) >> (64 - bits)) : 0;
}

/* ------------------------------------------------------------ sync */
void spin_lock_init(spinlock_t *l)
{
	__atomic_store_n(&l->locked, 0, __ATOMIC_RELEASE);
}

void spin_lock(spinlock_t *l)
{
	while (__atomic_exchange_n(&l->locked, 1, __ATOMIC_ACQUIRE))
		sched_yield();
	t_spin_depth++;
}

void spin_unlock(spinlock_t *l)
{
	t_spin_depth--;
	__atomic_store_n(&l->locked, 0, __ATOMIC_RELEASE);
}

void spin_lock_irq(spinlock_t *l)
{
	spin_lock(l);
}

void spin_unlock_irq(spinlock_t *l)
{
	spin_unlock(l);
}

void mutex_init(struct mutex *m)
{
	__atomic_store_n(&m->locked, 0, __ATOMIC_RELEASE);
}

void mutex_lock(struct mutex *m)
{
	check_sleepable("mutex_lock", NULL, 0);
	while (__atomic_exchange_n(&m->locked, 1, __ATOMIC_ACQUIRE))
		usleep(20);
}

void mutex_unlock(struct mutex *m)
{
	__atomic_store_n(&m->locked, 0, __ATOMIC_RELEASE);
}

static pthread_mutex_t g_wq_m = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_wq_c = PTHREAD_COND_INITIALIZER;

void init_waitqueue_head(wait_queue_head_t *wq)
{
	wq->x = 0;
}

void wake_up_all(wait_queue_head_t *wq)
{
	(void)wq;
	pthread_mutex_lock(&g_wq_m);
	pthread_cond_broadcast(&g_wq_c);
	pthread_mutex_unlock(&g_wq_m);
}

void kshim_wait_slice(wait_queue_head_t *wq, const char *file, int line)
{
	struct timespec ts;

	(void)wq;
	check_sleepable("wait", file, line);
	clock_gettime(CLOCK_REALTIME, &ts);
	ts.tv_nsec += 200000;
	if (ts.tv_nsec >= 1000000000) {
		ts.tv_sec++;
		ts.tv_nsec -= 1000000000;
	}
	pthread_mutex_lock(&g_wq_m);
	pthread_cond_timedwait(&g_wq_c, &g_wq_m, &ts);
	pthread_mutex_unlock(&g_wq_m);
}

void kref_init(struct kref *k)
{
	__atomic_store_n(&k->refcount.counter, 1, __ATOMIC_SEQ_CST);
}

void kref_get(struct kref *k)
{
	if (__atomic_fetch_add(&k->refcount.counter, 1, __ATOMIC_SEQ_CST) <= 0)
		violation("kref_get on a dead object");
}

int kref_put(struct kref *k, void (*release)(struct kref *))
{
	int v = __atomic_sub_fetch(&k->refcount.counter, 1, __ATOMIC_SEQ_CST);

	if (v < 0)
		violation("kref underflow");
	if (v == 0) {
		release(k);
		return 1;
	}
	return 0;
}

void atomic_set(atomic_t *a, int v) { __atomic_store_n(&a->counter, v, __ATOMIC_SEQ_CST); }
int atomic_read(const atomic_t *a) { return __atomic_load_n(&a->counter, __ATOMIC_SEQ_CST); }
void atomic_inc(atomic_t *a) { __atomic_add_fetch(&a->counter, 1, __ATOMIC_SEQ_CST); }
bool atomic_dec_and_test(atomic_t *a) { return __atomic_sub_fetch(&a->counter, 1, __ATOMIC_SEQ_CST) == 0; }
s64 atomic64_read(const atomic64_t *a) { return __atomic_load_n(&a->counter, __ATOMIC_SEQ_CST); }
void atomic64_inc(atomic64_t *a) { __atomic_add_fetch(&a->counter, 1, __ATOMIC_SEQ_CST); }
void atomic64_dec(atomic64_t *a) { __atomic_sub_fetch(&a->counter, 1, __ATOMIC_SEQ_CST); }
void atomic64_add(s64 v, atomic64_t *a) { __atomic_add_fetch(&a->counter, v, __ATOMIC_SEQ_CST); }
s64 atomic64_inc_return(atomic64_t *a) { return __atomic_add_fetch(&a->counter, 1, __ATOMIC_SEQ_CST); }
s64 atomic64_cmpxchg(atomic64_t *a, s64 o, s64 n)
{
	__atomic_compare_exchange_n(&a->counter, &o, n, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
	return o;
}
s64 atomic64_xchg(atomic64_t *a, s64 v) { return __atomic_exchange_n(&a->counter, v, __ATOMIC_SEQ_CST); }

/* lists */
void list_add(struct list_head *n, struct list_head *h)
{
	n->next = h->next;
	n->prev = h;
	h->next->prev = n;
	h->next = n;
}

void list_add_tail(struct list_head *n, struct list_head *h)
{
	n->prev = h->prev;
	n->next = h;
	h->prev->next = n;
	h->prev = n;
}

void list_del(struct list_head *e)
{
	e->prev->next = e->next;
	e->next->prev = e->prev;
	e->next = e->prev = NULL;
}

void hlist_add_head(struct hlist_node *n, struct hlist_head *h)
{
	n->next = h->first;
	if (h->first)
		h->first->pprev = &n->next;
	h->first = n;
	n->pprev = &h->first;
}

void hlist_del(struct hlist_node *n)
{
	*n->pprev = n->next;
	if (n->next)
		n->next->pprev = n->pprev;
	n->next = NULL;
	n->pprev = NULL;
}

/* ------------------------------------------------------------ workqueues */
struct workqueue_struct {
	pthread_t th;
	pthread_mutex_t m;
	pthread_cond_t c;
	struct work_struct *head, *tail;
	int running;
	bool stop;
	char name[32];
};

static void *wq_thread(void *p)
{
	struct workqueue_struct *wq = p;

	pthread_mutex_lock(&wq->m);
	for (;;) {
		struct work_struct *w;

		while (!wq->head && !wq->stop)
			pthread_cond_wait(&wq->c, &wq->m);
		if (!wq->head && wq->stop)
			break;
		w = wq->head;
		wq->head = w->next;
		if (!wq->head)
			wq->tail = NULL;
		w->next = NULL;
		w->pending = 0;         /* cleared before the call: the work may free itself */
		wq->running++;
		pthread_mutex_unlock(&wq->m);
		w->func(w);
		pthread_mutex_lock(&wq->m);
		wq->running--;
		pthread_cond_broadcast(&wq->c);
	}
	pthread_mutex_unlock(&wq->m);
	return NULL;
}

struct workqueue_struct *alloc_workqueue(const char *fmt, unsigned int flags, int max_active, ...)
{
	struct workqueue_struct *wq = calloc(1, sizeof(*wq));

	(void)flags;
	(void)max_active;
	if (!wq)
		return NULL;
	snprintf(wq->name, sizeof(wq->name), "%s", fmt);
	pthread_mutex_init(&wq->m, NULL);
	pthread_cond_init(&wq->c, NULL);
	if (pthread_create(&wq->th, NULL, wq_thread, wq)) {
		free(wq);
		return NULL;
	}
	return wq;
}

bool queue_work(struct workqueue_struct *wq, struct work_struct *w)
{
	bool queued = false;

	pthread_mutex_lock(&wq->m);
	if (!w->pending) {
		w->pending = 1;
		w->next = NULL;
		if (wq->tail)
			wq->tail->next = w;
		else
			wq->head = w;
		wq->tail = w;
		queued = true;
		pthread_cond_broadcast(&wq->c);
	}
	pthread_mutex_unlock(&wq->m);
	return queued;
}

static void wq_drain(struct workqueue_struct *wq)
{
	pthread_mutex_lock(&wq->m);
	while (wq->head || wq->running)
		pthread_cond_wait(&wq->c, &wq->m);
	pthread_mutex_unlock(&wq->m);
}

void destroy_workqueue(struct workqueue_struct *wq)
{
	check_sleepable("destroy_workqueue", NULL, 0);
	wq_drain(wq);
	pthread_mutex_lock(&wq->m);
	wq->stop = true;
	pthread_cond_broadcast(&wq->c);
	pthread_mutex_unlock(&wq->m);
	pthread_join(wq->th, NULL);
	pthread_mutex_destroy(&wq->m);
	pthread_cond_destroy(&wq->c);
	free(wq);
}

/* ------------------------------------------------------------ module, creds */
void __module_get(struct module *m) { (void)m; CNT_ADD(module_refs, 1); }
void module_put(struct module *m)
{
	(void)m;
	if (CNT_ADD(module_refs, -1) < 0)
		violation("module_put underflow");
}
kuid_t current_euid(void) { kuid_t k = { t_euid }; return k; }
unsigned int from_kuid(void *ns, kuid_t uid) { (void)ns; return uid.val; }
void *current_user_ns(void) { return NULL; }
bool capable(int cap) { return cap == CAP_SYS_ADMIN && g_admin; }
void ksim_set_euid(unsigned int uid) { t_euid = uid; }
void ksim_set_admin(int on) { g_admin = on; }
void ksim_set_signal(int on) { __atomic_store_n(&g_signal, on, __ATOMIC_SEQ_CST); }
void ksim_set_verbose(int v) { g_verbose = v; }

/* ------------------------------------------------------------ IOMMU domains */
struct iommu_ent { u64 key; char *host; int state; };   /* 0 empty, 1 used, 2 tomb */
struct kshim_iommu {
	pthread_mutex_t m;
	u64 next_iova;
	struct iommu_ent *tab;
	size_t cap, used, tombs;
};

static struct kshim_iommu *iommu_new(int idx)
{
	struct kshim_iommu *d = calloc(1, sizeof(*d));

	pthread_mutex_init(&d->m, NULL);
	/* every controller has its own IOVA space: a bus address mapped for
	 * one controller means nothing to another */
	d->next_iova = 0x100000000000ull + ((u64)idx << 40);
	d->cap = 1 << 12;
	d->tab = calloc(d->cap, sizeof(*d->tab));
	return d;
}

static void iommu_free(struct kshim_iommu *d)
{
	free(d->tab);
	pthread_mutex_destroy(&d->m);
	free(d);
}

static size_t ihash(u64 k, size_t cap)
{
	return (size_t)((k * 0x9E3779B97F4A7C15ull) >> 20) & (cap - 1);
}

static void iommu_put_locked(struct kshim_iommu *d, u64 key, char *host);

static void iommu_grow(struct kshim_iommu *d)
{
	struct iommu_ent *old = d->tab;
	size_t oc = d->cap, i;

	d->cap = d->used * 4 > oc ? oc * 2 : oc;
	d->tab = calloc(d->cap, sizeof(*d->tab));
	d->used = d->tombs = 0;
	for (i = 0; i < oc; i++)
		if (old[i].state == 1)
			iommu_put_locked(d, old[i].key, old[i].host);
	free(old);
}

static void iommu_put_locked(struct kshim_iommu *d, u64 key, char *host)
{
	size_t i;

	if ((d->used + d->tombs + 1) * 2 > d->cap)
		iommu_grow(d);
	for (i = ihash(key, d->cap);; i = (i + 1) & (d->cap - 1)) {
		if (d->tab[i].state != 1) {
			if (d->tab[i].state == 2)
				d->tombs--;
			d->tab[i].key = key;
			d->tab[i].host = host;
			d->tab[i].state = 1;
			d->used++;
			return;
		}
		if (d->tab[i].key == key) {
			violation("IOMMU: bus page %#llx mapped twice", (unsigned long long)key << 12);
			return;
		}
	}
}

static struct iommu_ent *iommu_find_locked(struct kshim_iommu *d, u64 key)
{
	size_t i;

	for (i = ihash(key, d->cap);; i = (i + 1) & (d->cap - 1)) {
		if (d->tab[i].state == 0)
			return NULL;
		if (d->tab[i].state == 1 && d->tab[i].key == key)
			return &d->tab[i];
	}
}

/* map [host, host+len) (host page aligned + off) -> returns bus address */
static u64 iommu_map(struct kshim_iommu *d, char *host, size_t len)
{
	size_t off = (uintptr_t)host & (PAGE_SIZE - 1), npg, i;
	char *base = host - off;
	u64 iova;

	npg = (off + len + PAGE_SIZE - 1) >> PAGE_SHIFT;
	pthread_mutex_lock(&d->m);
	iova = d->next_iova;
	d->next_iova += (npg + 1) << PAGE_SHIFT;       /* one guard page */
	for (i = 0; i < npg; i++)
		iommu_put_locked(d, (iova >> PAGE_SHIFT) + i, base + (i << PAGE_SHIFT));
	pthread_mutex_unlock(&d->m);
	CNT_ADD(iommu_pages_live, (s64)npg);
	return iova + off;
}

static void iommu_unmap(struct kshim_iommu *d, u64 iova, size_t len)
{
	size_t off = iova & (PAGE_SIZE - 1), npg, i;
	u64 k0 = iova >> PAGE_SHIFT;

	npg = (off + len + PAGE_SIZE - 1) >> PAGE_SHIFT;
	pthread_mutex_lock(&d->m);
	for (i = 0; i < npg; i++) {
		struct iommu_ent *e = iommu_find_locked(d, k0 + i);

		if (!e) {
			pthread_mutex_unlock(&d->m);
			violation("IOMMU: unmap of unmapped bus page %#llx", (unsigned long long)(k0 + i) << 12);
			return;
		}
		e->state = 2;
		d->used--;
		d->tombs++;
	}
	pthread_mutex_unlock(&d->m);
	CNT_ADD(iommu_pages_live, -(s64)npg);
}

/* host address of bus byte `iova` with `need` bytes contiguous in one page */
static char *iommu_xlate(struct kshim_iommu *d, u64 iova)
{
	struct iommu_ent *e;
	char *h = NULL;

	pthread_mutex_lock(&d->m);
	e = iommu_find_locked(d, iova >> PAGE_SHIFT);
	if (e)
		h = e->host + (iova & (PAGE_SIZE - 1));
	pthread_mutex_unlock(&d->m);
	return h;
}

static bool iommu_mapped(struct kshim_iommu *d, u64 iova, size_t len)
{
	u64 p;

	for (p = iova & ~(u64)(PAGE_SIZE - 1); p < iova + len; p += PAGE_SIZE)
		if (!iommu_xlate(d, p))
			return false;
	return true;
}

/* ------------------------------------------------------------ devices */
const struct bus_type pci_bus_type = { "pci" };
static const struct class block_class = { "block" };
static const struct bus_type nvme_bus = { "nvme-ctrl" };

#define MAX_DEVS 256
static pthread_mutex_t g_dev_m = PTHREAD_MUTEX_INITIALIZER;
static struct device *g_devs[MAX_DEVS];
static int g_ndevs;

static void dev_register(struct device *d, struct device *parent, const struct bus_type *bus,
			 const struct class *cls, const char *name)
{
	d->parent = parent;
	d->bus = bus;
	d->class = cls;
	snprintf(d->kname, sizeof(d->kname), "%s", name);
	d->dma_mask = DMA_BIT_MASK(64);
	pthread_mutex_lock(&g_dev_m);
	g_devs[g_ndevs++] = d;
	pthread_mutex_unlock(&g_dev_m);
}

static void dev_unregister(struct device *d)
{
	int i;

	pthread_mutex_lock(&g_dev_m);
	for (i = 0; i < g_ndevs; i++)
		if (g_devs[i] == d) {
			g_devs[i] = g_devs[--g_ndevs];
			break;
		}
	pthread_mutex_unlock(&g_dev_m);
}

struct device *get_device(struct device *d)
{
	if (d)
		__atomic_add_fetch(&d->krefs, 1, __ATOMIC_SEQ_CST);
	return d;
}

void put_device(struct device *d)
{
	if (d && __atomic_sub_fetch(&d->krefs, 1, __ATOMIC_SEQ_CST) < 0)
		violation("put_device underflow on %s", d->kname);
}

struct device *bus_find_device_by_name(const struct bus_type *bus, struct device *start,
				       const char *name)
{
	struct device *r = NULL;
	int i;

	(void)start;
	check_sleepable("bus_find_device_by_name", NULL, 0);
	pthread_mutex_lock(&g_dev_m);
	for (i = 0; i < g_ndevs; i++)
		if (g_devs[i]->bus == bus && !strcmp(g_devs[i]->kname, name)) {
			r = get_device(g_devs[i]);
			break;
		}
	pthread_mutex_unlock(&g_dev_m);
	return r;
}

struct device *device_find_child_by_name(struct device *parent, const char *name)
{
	struct device *r = NULL;
	int i;

	pthread_mutex_lock(&g_dev_m);
	for (i = 0; i < g_ndevs; i++)
		if (g_devs[i]->parent == parent && !strcmp(g_devs[i]->kname, name)) {
			r = get_device(g_devs[i]);
			break;
		}
	pthread_mutex_unlock(&g_dev_m);
	return r;
}

u64 dma_get_mask(struct device *d) { return d->dma_mask; }
int dev_to_node(struct device *d) { return d->numa_node; }

/* ------------------------------------------------------------ pages */
struct kshim_pblock { char *mem; struct page *pages; int npages; int live; };
unsigned int nr_node_ids = 2;

bool node_online(int nid)
{
	return nid == 0 || nid == 1;
}

int numa_node_id(void)
{
	return 0;
}

struct page *alloc_pages_node(int nid, gfp_t gfp, unsigned int order)
{
	struct kshim_pblock *b;
	int n = 1 << order, i;

	if (!(gfp & GFP_ATOMIC))
		check_sleepable("alloc_pages_node", NULL, 0);
	if (nid < 0 || (unsigned int)nid >= nr_node_ids || !node_online(nid)) {
		violation("alloc_pages_node on invalid node %d", nid);
		return NULL;
	}
	b = calloc(1, sizeof(*b));
	b->mem = aligned_alloc(PAGE_SIZE, (size_t)n << PAGE_SHIFT);
	b->pages = calloc(n, sizeof(struct page));
	if (!b->mem || !b->pages) {
		free(b->mem);
		free(b->pages);
		free(b);
		return NULL;
	}
	if (gfp & __GFP_ZERO)
		memset(b->mem, 0, (size_t)n << PAGE_SHIFT);
	else
		memset(b->mem, 0xa5, (size_t)n << PAGE_SHIFT);
	b->npages = n;
	b->live = 1;
	for (i = 0; i < n; i++) {
		b->pages[i].kaddr = b->mem + ((size_t)i << PAGE_SHIFT);
		b->pages[i].blk = b;
	}
	b->pages[0].refcount = 1;
	CNT_ADD(pages_live, n);
	return b->pages;
}

void split_page(struct page *p, unsigned int order)
{
	int i;

	for (i = 1; i < (1 << order); i++) {
		p[i].refcount = 1;
		p->blk->live++;
	}
}

void get_page(struct page *p)
{
	__atomic_add_fetch(&p->refcount, 1, __ATOMIC_SEQ_CST);
}

void __free_page(struct page *p)
{
	struct kshim_pblock *b = p->blk;
	int r = __atomic_sub_fetch(&p->refcount, 1, __ATOMIC_SEQ_CST);

	if (r < 0) {
		violation("page freed twice");
		return;
	}
	if (r)
		return;
	CNT_ADD(pages_live, -1);
	if (__atomic_sub_fetch(&b->live, 1, __ATOMIC_SEQ_CST) == 0) {
		/* an unsplit high-order block frees all its pages with page 0 */
		if (b->npages > 1 && p == b->pages && b->pages[1].refcount == 0)
			CNT_ADD(pages_live, -(b->npages - 1));
		free(b->mem);
		free(b->pages);
		free(b);
	}
}

unsigned long __get_free_page(gfp_t gfp)
{
	void *p;

	if (!(gfp & GFP_ATOMIC))
		check_sleepable("__get_free_page", NULL, 0);
	p = aligned_alloc(PAGE_SIZE, PAGE_SIZE);
	if (p)
		CNT_ADD(kmallocs_live, 1);
	return (unsigned long)p;
}

void free_page(unsigned long p)
{
	if (p) {
		CNT_ADD(kmallocs_live, -1);
		free((void *)p);
	}
}

void *kmap_local_page(struct page *p) { return p->kaddr; }
void kunmap_local(const void *p) { (void)p; }

/* ------------------------------------------------------------ DMA API */
static int g_fail_map_at;                 /* fail the Nth dma_map_page (1-based) */
static int g_nmaps;
static size_t g_max_mapping;              /* swiotlb-like cap on one mapping (0: none) */

void ksim_dma_max_mapping(size_t bytes)
{
	__atomic_store_n(&g_max_mapping, bytes, __ATOMIC_SEQ_CST);
}

void ksim_fail_map(int nth)
{
	__atomic_store_n(&g_fail_map_at, nth, __ATOMIC_SEQ_CST);
	__atomic_store_n(&g_nmaps, 0, __ATOMIC_SEQ_CST);
}

dma_addr_t dma_map_page(struct device *dev, struct page *pg, size_t off, size_t sz,
			enum dma_data_direction dir)
{
	int n = __atomic_add_fetch(&g_nmaps, 1, __ATOMIC_SEQ_CST);
	int f = __atomic_load_n(&g_fail_map_at, __ATOMIC_SEQ_CST);

	(void)dir;
	CNT_ADD(dma_map_calls, 1);
	if (!dev || !dev->iommu) {
		violation("dma_map_page for a device without a DMA domain");
		return DMA_MAPPING_ERROR;
	}
	if (f && n == f)
		return DMA_MAPPING_ERROR;
	{
		size_t cap = __atomic_load_n(&g_max_mapping, __ATOMIC_SEQ_CST);

		if (cap && sz > cap)
			return DMA_MAPPING_ERROR;   /* what a bounce-buffered device does */
	}
	return iommu_map(dev->iommu, (char *)pg->kaddr + off, sz);
}

void dma_unmap_page(struct device *dev, dma_addr_t a, size_t sz, enum dma_data_direction dir)
{
	(void)dir;
	iommu_unmap(dev->iommu, a, sz);
}

void dma_sync_single_for_cpu(struct device *dev, dma_addr_t a, size_t sz,
			     enum dma_data_direction dir)
{
	(void)dir;
	if (!iommu_mapped(dev->iommu, a, sz))
		violation("dma_sync_single_for_cpu on an unmapped range %#llx+%zu",
			  (unsigned long long)a, sz);
}

int dma_mapping_error(struct device *dev, dma_addr_t a)
{
	(void)dev;
	return a == DMA_MAPPING_ERROR;
}

struct dma_pool { struct device *dev; size_t size; int live; char name[32]; };

struct dma_pool *dma_pool_create(const char *name, struct device *dev, size_t size, size_t align,
				 size_t boundary)
{
	struct dma_pool *p = kzalloc(sizeof(*p), GFP_KERNEL);

	(void)align;
	(void)boundary;
	if (!p)
		return NULL;
	p->dev = dev;
	p->size = size;
	snprintf(p->name, sizeof(p->name), "%s", name);
	return p;
}

void dma_pool_destroy(struct dma_pool *p)
{
	if (!p)
		return;
	if (p->live)
		violation("dma_pool_destroy(%s) with %d live blocks", p->name, p->live);
	kfree(p);
}

void *dma_pool_alloc(struct dma_pool *p, gfp_t gfp, dma_addr_t *dma)
{
	void *v;

	if (!(gfp & GFP_ATOMIC))
		check_sleepable("dma_pool_alloc", NULL, 0);
	v = aligned_alloc(PAGE_SIZE, (p->size + PAGE_SIZE - 1) & ~(PAGE_SIZE - 1));
	if (!v)
		return NULL;
	memset(v, 0xcc, p->size);
	*dma = iommu_map(p->dev->iommu, v, p->size);
	__atomic_add_fetch(&p->live, 1, __ATOMIC_SEQ_CST);
	return v;
}

void dma_pool_free(struct dma_pool *p, void *v, dma_addr_t dma)
{
	if (iommu_xlate(p->dev->iommu, dma) != v)
		violation("dma_pool_free: bus address does not map the block");
	iommu_unmap(p->dev->iommu, dma, p->size);
	__atomic_sub_fetch(&p->live, 1, __ATOMIC_SEQ_CST);
	free(v);
}

/* ------------------------------------------------------------ files */
enum { KF_PLAIN, KF_FS, KF_BDEV, KF_DMABUF, KF_DEV };

struct ksim_file {
	struct file f;
	int refs;
	int kind;
	struct inode *inode;
	struct inode own_inode;
	struct block_device *bdev;          /* KF_BDEV */
	void *obj;                          /* KF_FS: fsfile; KF_DMABUF: dmabuf */
	char name[64];
};

#define MAX_FDS 1024
static pthread_mutex_t g_fd_m = PTHREAD_MUTEX_INITIALIZER;
static struct ksim_file *g_fds[MAX_FDS];

static struct ksim_file *kf_of(const struct file *f)
{
	return container_of(f, struct ksim_file, f);
}

static struct ksim_file *kf_new(int kind)
{
	struct ksim_file *kf = calloc(1, sizeof(*kf));

	kf->refs = 1;
	kf->kind = kind;
	kf->inode = &kf->own_inode;
	kf->f.f_mode = FMODE_READ;
	CNT_ADD(files_live, 1);
	return kf;
}

static int fd_install(struct ksim_file *kf)
{
	int i;

	pthread_mutex_lock(&g_fd_m);
	for (i = 3; i < MAX_FDS; i++)
		if (!g_fds[i]) {
			g_fds[i] = kf;
			pthread_mutex_unlock(&g_fd_m);
			return i;
		}
	pthread_mutex_unlock(&g_fd_m);
	return -1;
}

struct file *fget(unsigned int fd)
{
	struct ksim_file *kf = NULL;

	pthread_mutex_lock(&g_fd_m);
	if (fd < MAX_FDS)
		kf = g_fds[fd];
	if (kf)
		__atomic_add_fetch(&kf->refs, 1, __ATOMIC_SEQ_CST);
	pthread_mutex_unlock(&g_fd_m);
	return kf ? &kf->f : NULL;
}

struct file *get_file(struct file *f)
{
	if (__atomic_fetch_add(&kf_of(f)->refs, 1, __ATOMIC_SEQ_CST) <= 0)
		violation("get_file on a released file");
	return f;
}

static void dmabuf_file_release(struct ksim_file *kf);
static struct workqueue_struct *g_fput_wq;

struct fput_work { struct work_struct w; struct ksim_file *kf; };

static void file_release(struct ksim_file *kf)
{
	if (kf->f.f_op && kf->f.f_op->release)
		kf->f.f_op->release(kf->inode, &kf->f);
	if (kf->kind == KF_DMABUF)
		dmabuf_file_release(kf);
	if (kf->kind == KF_BDEV)
		put_device(&kf->bdev->bd_device);
	CNT_ADD(files_live, -1);
	free(kf);
}

static void fput_work_fn(struct work_struct *w)
{
	struct fput_work *fw = container_of(w, struct fput_work, w);

	file_release(fw->kf);
	free(fw);
}

void fput(struct file *f)
{
	struct ksim_file *kf = kf_of(f);
	int r = __atomic_sub_fetch(&kf->refs, 1, __ATOMIC_SEQ_CST);

	if (r < 0) {
		violation("fput underflow");
		return;
	}
	if (r)
		return;
	if (t_in_irq || t_spin_depth) {
		/* as the kernel's delayed_fput: ->release runs in process context */
		struct fput_work *fw = calloc(1, sizeof(*fw));

		INIT_WORK(&fw->w, fput_work_fn);
		fw->kf = kf;
		CNT_ADD(deferred_fputs, 1);
		queue_work(g_fput_wq, &fw->w);
		return;
	}
	file_release(kf);
}

struct fd fdget(unsigned int fd)
{
	struct fd r = { fget(fd) };

	return r;
}

void fdput(struct fd fd)
{
	if (fd.file)
		fput(fd.file);
}

struct inode *file_inode(const struct file *f)
{
	return kf_of(f)->inode;
}

loff_t i_size_read(const struct inode *inode)
{
	return __atomic_load_n(&inode->i_size, __ATOMIC_SEQ_CST);
}

int ksim_close(int fd)
{
	struct ksim_file *kf = NULL;

	pthread_mutex_lock(&g_fd_m);
	if (fd >= 0 && fd < MAX_FDS) {
		kf = g_fds[fd];
		g_fds[fd] = NULL;
	}
	pthread_mutex_unlock(&g_fd_m);
	if (!kf)
		return -EBADF;
	fput(&kf->f);
	return 0;
}

int anon_inode_getfd(const char *name, const struct file_operations *fops, void *priv, int flags)
{
	struct ksim_file *kf = kf_new(KF_PLAIN);
	int fd;

	(void)flags;
	kf->f.f_op = fops;
	kf->f.private_data = priv;
	kf->f.f_mode = FMODE_READ | 2;
	snprintf(kf->name, sizeof(kf->name), "anon_inode:%s", name);
	fd = fd_install(kf);
	if (fd < 0) {
		CNT_ADD(files_live, -1);
		free(kf);
		return -ENOMEM;
	}
	return fd;
}

const char *ksim_fd_name(int fd)
{
	const char *n = NULL;

	pthread_mutex_lock(&g_fd_m);
	if (fd >= 0 && fd < MAX_FDS && g_fds[fd])
		n = g_fds[fd]->name;
	pthread_mutex_unlock(&g_fd_m);
	return n;
}

/* ------------------------------------------------------------ block devices */
enum { DK_NS, DK_MD, DK_HEAD };

struct ksim_ctrl;
struct request_queue { bool mq; u32 lbs; u32 lbs_shift_sim; u32 max_hw_sectors; struct ksim_disk *disk; };

struct ksim_disk {
	struct gendisk disk;
	struct block_device part0;
	struct request_queue q;
	struct block_device_operations fops;
	int kind;
	bool live;
	sector_t capacity;                  /* 512-B sectors */
	/* namespace */
	struct ksim_ctrl *ctrl;
	u32 nsid;
	u8 *image;
	/* md raid0 (single zone) / multipath head */
	int nmembers;
	struct ksim_disk *members[KSIM_MD_MAX];
	u32 chunk_sects;
	u64 data_offset[KSIM_MD_MAX];
};

#define MAX_DISKS 64
static struct ksim_disk *g_disks[MAX_DISKS];
static int g_ndisks;
static int g_next_minor[16];
static u64 g_diskseq = 1;

bool queue_is_mq(struct request_queue *q) { return q->mq; }
unsigned int queue_logical_block_size(const struct request_queue *q) { return q->lbs; }
unsigned int queue_max_hw_sectors(const struct request_queue *q) { return q->max_hw_sectors; }
sector_t get_capacity(struct gendisk *disk) { return container_of(disk, struct ksim_disk, disk)->capacity; }
sector_t get_start_sect(struct block_device *bdev) { return bdev->bd_start_sect; }
dev_t disk_devt(struct gendisk *disk) { return MKDEV(disk->major, disk->first_minor); }
bool disk_live(struct gendisk *disk)
{
	return __atomic_load_n(&container_of(disk, struct ksim_disk, disk)->live, __ATOMIC_SEQ_CST);
}

static void bd_acct(struct block_device *b, long inflight, unsigned long ios, unsigned long sectors)
{
	__atomic_add_fetch(&b->kinflight, inflight, __ATOMIC_SEQ_CST);
	__atomic_add_fetch(&b->kios, ios, __ATOMIC_SEQ_CST);
	__atomic_add_fetch(&b->ksectors, sectors, __ATOMIC_SEQ_CST);
}

unsigned long bdev_start_io_acct(struct block_device *bdev, enum req_op op, unsigned long start)
{
	(void)op;
	bd_acct(bdev, 1, 0, 0);
	if (bdev != bdev->bd_disk->part0)            /* a partition counts on its disk too */
		bd_acct(bdev->bd_disk->part0, 1, 0, 0);
	return start;
}

void bdev_end_io_acct(struct block_device *bdev, enum req_op op, unsigned int sectors,
		      unsigned long start)
{
	(void)op;
	(void)start;
	bd_acct(bdev, -1, 1, sectors);
	if (bdev != bdev->bd_disk->part0)
		bd_acct(bdev->bd_disk->part0, -1, 1, sectors);
}

static struct ksim_disk *disk_by_devt(dev_t devt)
{
	int i;

	for (i = 0; i < g_ndisks; i++)
		if (g_disks[i] && g_disks[i]->live && g_disks[i]->disk.major &&
		    disk_devt(&g_disks[i]->disk) == devt)
			return g_disks[i];
	return NULL;
}

struct file *bdev_file_open_by_dev(dev_t dev, blk_mode_t mode, void *holder, const void *hops)
{
	struct ksim_disk *d;
	struct ksim_file *kf;

	(void)mode;
	(void)holder;
	(void)hops;
	check_sleepable("bdev_file_open_by_dev", NULL, 0);
	d = disk_by_devt(dev);
	if (!d)
		return ERR_PTR(-ENXIO);
	kf = kf_new(KF_BDEV);
	kf->bdev = &d->part0;
	get_device(&d->part0.bd_device);
	return &kf->f;
}

struct block_device *file_bdev(struct file *f)
{
	return kf_of(f)->bdev;
}

struct bdev_handle *bdev_open_by_dev(dev_t dev, blk_mode_t mode, void *holder, const void *hops)
{
	struct ksim_disk *d;
	struct bdev_handle *h;

	(void)mode;
	(void)holder;
	(void)hops;
	d = disk_by_devt(dev);
	if (!d)
		return ERR_PTR(-ENXIO);
	h = kzalloc(sizeof(*h), GFP_KERNEL);
	h->bdev = &d->part0;
	get_device(&d->part0.bd_device);
	return h;
}

void bdev_release(struct bdev_handle *h)
{
	put_device(&h->bdev->bd_device);
	kfree(h);
}

static int ns_ioctl(struct block_device *b, blk_mode_t mode, unsigned int cmd, unsigned long arg)
{
	struct ksim_disk *d = container_of(b->bd_disk, struct ksim_disk, disk);

	(void)mode;
	(void)arg;
	if (cmd != NVME_IOCTL_ID)
		return -ENOTTY_SIM;
	return d->kind == DK_HEAD ? (int)d->members[0]->nsid : (int)d->nsid;
}

static int md_ioctl(struct block_device *b, blk_mode_t mode, unsigned int cmd, unsigned long arg)
{
	(void)b;
	(void)mode;
	(void)cmd;
	(void)arg;
	return -ENOTTY_SIM;
}

/* ------------------------------------------------------------ NVMe controllers */
struct ksim_ctrl {
	struct device pci;
	struct device cdev;
	int idx;
	pthread_t th;
	pthread_mutex_t m;
	pthread_cond_t c;
	struct request *q[4096];
	int nq;
	bool stop, reorder, hold;
	int delay_us;
	unsigned int seed;
	u64 ncmds;
};

#define MAX_CTRLS 16
static struct ksim_ctrl *g_ctrls[MAX_CTRLS];
static int g_nctrls;
static int g_fail_cmd_at;                 /* fail the Nth command (1-based, all ctrls) */
static int g_fail_status;
static int g_cmd_seq;

void ksim_fail_cmd(int nth, int blk_status)
{
	__atomic_store_n(&g_fail_status, blk_status, __ATOMIC_SEQ_CST);
	__atomic_store_n(&g_fail_cmd_at, nth, __ATOMIC_SEQ_CST);
	__atomic_store_n(&g_cmd_seq, 0, __ATOMIC_SEQ_CST);
}

int blk_status_to_errno(blk_status_t s)
{
	switch (s) {
	case 0: return 0;
	case 1: return -EOPNOTSUPP;          /* BLK_STS_NOTSUPP */
	case 7: return -ENODATA;             /* BLK_STS_MEDIUM */
	case 9: return -ENOMEM;              /* BLK_STS_RESOURCE */
	default: return -EIO;                /* BLK_STS_IOERR (10) and the rest */
	}
}

struct request *blk_mq_alloc_request(struct request_queue *q, unsigned int opf, unsigned int flags)
{
	struct request *rq;

	if (!(flags & 1))                         /* BLK_MQ_REQ_NOWAIT not set: may sleep */
		check_sleepable("blk_mq_alloc_request", NULL, 0);
	if (!q->mq) {
		violation("blk_mq_alloc_request on a bio-based queue");
		return ERR_PTR(-EINVAL);
	}
	if (opf != REQ_OP_DRV_IN)
		violation("passthrough request with opf %u", opf);
	rq = calloc(1, sizeof(*rq));
	rq->q = q;
	rq->opf = opf;
	CNT_ADD(requests_live, 1);
	return rq;
}

void nvme_init_request(struct request *req, struct nvme_command *cmd)
{
	req->cmd = cmd;
}

void blk_execute_rq_nowait(struct request *rq, bool at_head)
{
	struct ksim_ctrl *c = rq->q->disk->ctrl;

	(void)at_head;

	if (!rq->end_io || !rq->cmd)
		violation("request submitted without end_io or command");
	pthread_mutex_lock(&c->m);
	while (c->nq == (int)ARRAY_SIZE(c->q)) {
		pthread_mutex_unlock(&c->m);
		usleep(50);
		pthread_mutex_lock(&c->m);
	}
	c->q[c->nq++] = rq;
	pthread_cond_broadcast(&c->c);
	pthread_mutex_unlock(&c->m);
	CNT_ADD(cmds_submitted, 1);
}

/* PRP walk of one READ: the spec's rules for PRP1 / PRP2 / the list page */
static int nvme_read(struct ksim_ctrl *c, struct ksim_disk *ns, const struct nvme_rw_command *rw,
		     char *why, size_t whylen)
{
	struct kshim_iommu *dom = c->pci.iommu;
	const u64 lbsz = 1ull << ns->q.lbs_shift_sim;
	const u64 nlb = (u64)rw->length + 1;
	const u64 total = nlb * lbsz;
	const u64 slba = rw->slba;
	u64 prp1 = rw->dptr.prp1, prp2 = rw->dptr.prp2, done = 0, first;
	u64 entries[STROM_SIM_MAX_PRPS];
	int nent = 0, i;
	const u64 *list = NULL;

#define BAD(...) do { snprintf(why, whylen, __VA_ARGS__); return -1; } while (0)
	if (rw->opcode != nvme_cmd_read)
		BAD("opcode %#x is not READ", rw->opcode);
	if (rw->nsid != ns->nsid)
		BAD("nsid %u sent to namespace %u", rw->nsid, ns->nsid);
	if (slba + nlb > (ns->capacity >> (ns->q.lbs_shift_sim - 9)))
		BAD("slba %llu + %llu blocks past capacity", (unsigned long long)slba,
		    (unsigned long long)nlb);
	if (prp1 & 3)
		BAD("PRP1 %#llx not dword aligned", (unsigned long long)prp1);
	first = PAGE_SIZE - (prp1 & (PAGE_SIZE - 1));
	entries[nent++] = prp1;
	if (total > first) {
		u64 rest = total - first, need = DIV_ROUND_UP(rest, PAGE_SIZE);

		if (need == 1) {
			if (prp2 & (PAGE_SIZE - 1))
				BAD("PRP2 %#llx (2nd page) not page aligned", (unsigned long long)prp2);
			entries[nent++] = prp2;
		} else {
			u64 in_page = (PAGE_SIZE - (prp2 & (PAGE_SIZE - 1))) / 8;

			if (prp2 & 7)
				BAD("PRP list pointer %#llx not qword aligned", (unsigned long long)prp2);
			if (need > in_page)
				BAD("PRP list of %llu entries crosses its page (chaining not used)",
				    (unsigned long long)need);
			if (need + 1 > STROM_SIM_MAX_PRPS)
				BAD("request too large for the model");
			list = (const u64 *)iommu_xlate(dom, prp2);
			if (!list)
				BAD("PRP list page %#llx not mapped for %s", (unsigned long long)prp2,
				    c->pci.kname);
			for (i = 0; i < (int)need; i++) {
				if (list[i] & (PAGE_SIZE - 1))
					BAD("PRP list entry %d (%#llx) not page aligned", i,
					    (unsigned long long)list[i]);
				entries[nent++] = list[i];
			}
		}
	} else if (prp2) {
		BAD("PRP2 %#llx set for a one-page transfer", (unsigned long long)prp2);
	}
	/* translate everything before moving a byte */
	for (i = 0; i < nent; i++) {
		u64 len = i == 0 ? min(first, total) : min((u64)PAGE_SIZE, total - done);

		if (!iommu_mapped(dom, entries[i], len))
			BAD("PRP entry %d %#llx (+%llu) not mapped for %s", i,
			    (unsigned long long)entries[i], (unsigned long long)len, c->pci.kname);
		done += len;
	}
	done = 0;
	for (i = 0; i < nent; i++) {
		u64 len = i == 0 ? min(first, total) : min((u64)PAGE_SIZE, total - done);

		memcpy(iommu_xlate(dom, entries[i]), ns->image + slba * lbsz + done, len);
		done += len;
	}
#undef BAD
	return 0;
}

static void *ctrl_thread(void *p)
{
	struct ksim_ctrl *c = p;

	pthread_mutex_lock(&c->m);
	for (;;) {
		struct request *rq;
		struct ksim_disk *ns;
		blk_status_t st = 0;
		char why[256] = "";
		int k, seq, f;

		while ((!c->nq || c->hold) && !c->stop)
			pthread_cond_wait(&c->c, &c->m);
		if (c->stop && (!c->nq || c->hold))
			break;
		k = c->reorder ? (int)(rand_r(&c->seed) % c->nq) : 0;
		rq = c->q[k];
		memmove(&c->q[k], &c->q[k + 1], (c->nq - k - 1) * sizeof(c->q[0]));
		c->nq--;
		pthread_mutex_unlock(&c->m);
		if (c->delay_us)
			usleep(c->delay_us);
		ns = rq->q->disk;
		seq = __atomic_add_fetch(&g_cmd_seq, 1, __ATOMIC_SEQ_CST);
		f = __atomic_load_n(&g_fail_cmd_at, __ATOMIC_SEQ_CST);
		if (f && seq == f) {
			st = (blk_status_t)__atomic_load_n(&g_fail_status, __ATOMIC_SEQ_CST);
			CNT_ADD(cmds_failed_injected, 1);
		} else if (!__atomic_load_n(&ns->live, __ATOMIC_SEQ_CST)) {
			st = 10;
		} else if (nvme_read(c, ns, &rq->cmd->rw, why, sizeof(why))) {
			violation("NVMe %s: %s", ns->disk.disk_name, why);
			CNT_ADD(cmds_bad, 1);
			st = 10;
		} else {
			CNT_ADD(cmds_ok, 1);
			CNT_ADD(bytes_moved, ((u64)rq->cmd->rw.length + 1) << ns->q.lbs_shift_sim);
		}
		c->ncmds++;
		/* completion: blk-mq calls end_io from the IRQ / softirq path */
		t_in_irq = 1;
		if (rq->end_io(rq, st) != RQ_END_IO_FREE)
			violation("end_io did not free the request");
		t_in_irq = 0;
		CNT_ADD(requests_live, -1);
		free(rq);
		pthread_mutex_lock(&c->m);
	}
	pthread_mutex_unlock(&c->m);
	return NULL;
}

int ksim_ctrl_new(const char *pci_name, int numa_node)
{
	struct ksim_ctrl *c = calloc(1, sizeof(*c));
	char name[16];

	c->idx = g_nctrls;
	c->seed = 1234 + c->idx;
	dev_register(&c->pci, NULL, &pci_bus_type, NULL, pci_name);
	c->pci.numa_node = numa_node;
	c->pci.iommu = iommu_new(c->idx);
	snprintf(name, sizeof(name), "nvme%d", c->idx);
	dev_register(&c->cdev, &c->pci, &nvme_bus, NULL, name);
	c->cdev.numa_node = numa_node;
	pthread_mutex_init(&c->m, NULL);
	pthread_cond_init(&c->c, NULL);
	pthread_create(&c->th, NULL, ctrl_thread, c);
	g_ctrls[g_nctrls] = c;
	return g_nctrls++;
}

void ksim_ctrl_config(int ci, int reorder, int delay_us, int hold)
{
	struct ksim_ctrl *c = g_ctrls[ci];

	pthread_mutex_lock(&c->m);
	c->reorder = reorder;
	c->delay_us = delay_us;
	c->hold = hold;
	pthread_cond_broadcast(&c->c);
	pthread_mutex_unlock(&c->m);
}

int ksim_ctrl_queued(int ci)
{
	struct ksim_ctrl *c = g_ctrls[ci];
	int n;

	pthread_mutex_lock(&c->m);
	n = c->nq;
	pthread_mutex_unlock(&c->m);
	return n;
}

void ksim_ctrl_set_dma_mask_bits(int ci, int bits)
{
	g_ctrls[ci]->pci.dma_mask = DMA_BIT_MASK(bits);
}

static struct ksim_disk *disk_new(int kind, const char *name, int major, bool visible)
{
	struct ksim_disk *d = calloc(1, sizeof(*d));

	d->kind = kind;
	d->live = true;
	snprintf(d->disk.disk_name, sizeof(d->disk.disk_name), "%s", name);
	d->disk.major = visible ? major : 0;
	d->disk.first_minor = visible ? g_next_minor[major & 15]++ : 0;
	d->disk.queue = &d->q;
	d->disk.part0 = &d->part0;
	d->disk.fops = &d->fops;
	d->disk.diskseq = g_diskseq++;
	d->part0.bd_disk = &d->disk;
	d->q.disk = d;
	d->q.lbs = 512;
	d->q.lbs_shift_sim = 9;
	g_disks[g_ndisks++] = d;
	return d;
}

int ksim_ns_new(int ci, u32 nsid, int lba_shift, u64 nsects, u32 max_hw_sectors, int hidden)
{
	struct ksim_ctrl *c = g_ctrls[ci];
	struct ksim_disk *d;
	char name[32];

	if (hidden)
		snprintf(name, sizeof(name), "nvme%dc%dn%u", c->idx, c->idx, nsid);
	else
		snprintf(name, sizeof(name), "nvme%dn%u", c->idx, nsid);
	d = disk_new(DK_NS, name, 259, !hidden);
	d->ctrl = c;
	d->nsid = nsid;
	d->capacity = nsects;
	d->image = calloc(1, nsects << 9);
	d->q.mq = true;
	d->q.lbs = 1u << lba_shift;
	d->q.lbs_shift_sim = lba_shift;
	d->q.max_hw_sectors = max_hw_sectors;
	d->fops.ioctl = ns_ioctl;
	dev_register(&d->part0.bd_device, &c->cdev, NULL, &block_class, name);
	d->part0.bd_device.numa_node = c->pci.numa_node;
	return g_ndisks - 1;
}

int ksim_md_new(const int *members, int n, u32 chunk_sects, const u64 *data_offset)
{
	char name[16];
	struct ksim_disk *d;
	u64 per = UINT64_MAX;
	int i;

	if (n < 1 || n > KSIM_MD_MAX)
		abort();
	snprintf(name, sizeof(name), "md%d", g_next_minor[9]);
	d = disk_new(DK_MD, name, 9, true);
	d->nmembers = n;
	d->chunk_sects = chunk_sects;
	d->fops.ioctl = md_ioctl;
	for (i = 0; i < n; i++) {
		d->members[i] = g_disks[members[i]];
		d->data_offset[i] = data_offset ? data_offset[i] : 0;
		per = min(per, d->members[i]->capacity - d->data_offset[i]);
	}
	per = per / chunk_sects * chunk_sects;
	d->capacity = per * n;
	d->q.mq = false;
	dev_register(&d->part0.bd_device, NULL, NULL, &block_class, name);
	return g_ndisks - 1;
}

int ksim_head_new(int path)
{
	struct ksim_disk *p = g_disks[path], *d;
	char name[32];

	snprintf(name, sizeof(name), "nvme%dn%u", p->ctrl->idx, p->nsid);
	d = disk_new(DK_HEAD, name, 259, true);
	d->nmembers = 1;
	d->members[0] = p;
	d->capacity = p->capacity;
	d->q.mq = false;
	d->fops.ioctl = ns_ioctl;
	dev_register(&d->part0.bd_device, NULL, NULL, &block_class, name);
	return g_ndisks - 1;
}

u32 ksim_disk_devt(int di)
{
	return disk_devt(&g_disks[di]->disk);
}

const char *ksim_disk_name(int di)
{
	return g_disks[di]->disk.disk_name;
}

/* a disk that went away (hot removal); with `replace`, a new disk instance
 * takes the same dev_t (diskseq changes) */
int ksim_disk_remove(int di, int replace)
{
	struct ksim_disk *o = g_disks[di], *d;

	__atomic_store_n(&o->live, false, __ATOMIC_SEQ_CST);
	if (!replace)
		return di;
	d = calloc(1, sizeof(*d));
	*d = *o;
	d->live = true;
	d->disk.queue = &d->q;
	d->disk.part0 = &d->part0;
	d->disk.fops = &d->fops;
	d->disk.diskseq = g_diskseq++;
	d->part0.bd_disk = &d->disk;
	d->part0.kios = d->part0.ksectors = 0;
	d->part0.kinflight = 0;
	d->part0.bd_device.krefs = 0;
	d->q.disk = d;
	d->image = malloc(o->capacity << 9);
	memcpy(d->image, o->image, o->capacity << 9);
	dev_unregister(&o->part0.bd_device);
	dev_register(&d->part0.bd_device, o->part0.bd_device.parent, NULL, &block_class,
		     o->disk.disk_name);
	d->part0.bd_device.numa_node = o->part0.bd_device.numa_node;
	g_disks[g_ndisks++] = d;
	return g_ndisks - 1;
}

void ksim_disk_stats(int di, u64 *ios, u64 *sectors, s64 *inflight)
{
	struct block_device *b = &g_disks[di]->part0;

	*ios = __atomic_load_n(&b->kios, __ATOMIC_SEQ_CST);
	*sectors = __atomic_load_n(&b->ksectors, __ATOMIC_SEQ_CST);
	*inflight = __atomic_load_n(&b->kinflight, __ATOMIC_SEQ_CST);
}

/* write 512-B sectors of a volume through its own layout (not strom_core's) */
static void vol_write(struct ksim_disk *d, u64 sect, const u8 *src, u64 nsect)
{
	u64 i;

	for (i = 0; i < nsect; i++, sect++, src += 512) {
		struct ksim_disk *t = d;
		u64 s = sect;

		while (t->kind != DK_NS) {
			if (t->kind == DK_HEAD) {
				t = t->members[0];
				continue;
			}
			{
				u64 chunk = s / t->chunk_sects, row = chunk / t->nmembers;
				int m = (int)(chunk % t->nmembers);

				s = row * t->chunk_sects + s % t->chunk_sects + t->data_offset[m];
				t = t->members[m];
			}
		}
		if (s >= t->capacity)
			abort();
		memcpy(t->image + (s << 9), src, 512);
	}
}

/* ------------------------------------------------------------ filesystem */
struct address_space { struct ksim_fsfile *ff; };

struct ksim_fs {
	struct super_block sb;
	struct file_system_type type;
	struct block_device part;            /* the partition (or the disk's part0 copy) */
	struct ksim_disk *disk;
	bool whole;
};

struct ksim_fsfile {
	struct inode inode;
	struct address_space mapping;
	struct ksim_fs *fs;
	pthread_mutex_t m;
	u8 *data;                            /* logical content (what the page cache shows) */
	u8 *pc;                              /* per page: 0 absent, 1 clean, 2 dirty */
	struct folio *folios;
	u64 *blkmap;                         /* fs block -> volume fs block (0 = hole) */
	u64 nblocks;
};

#define MAX_FS 16
#define MAX_FF 64
static struct ksim_fs *g_fs[MAX_FS];
static int g_nfs;
static struct ksim_fsfile *g_ff[MAX_FF];
static int g_nff;

int ksim_fs_new(int di, u64 part_start_sect, const char *fstype, int blkbits)
{
	struct ksim_fs *fs = calloc(1, sizeof(*fs));
	struct ksim_disk *d = g_disks[di];

	fs->disk = d;
	fs->type.name = strdup(fstype);
	fs->sb.s_type = &fs->type;
	fs->sb.s_blocksize = 1ul << blkbits;
	if (part_start_sect) {
		fs->part.bd_disk = &d->disk;
		fs->part.bd_start_sect = part_start_sect;
		fs->sb.s_bdev = &fs->part;
	} else {
		fs->whole = true;
		fs->sb.s_bdev = &d->part0;
	}
	g_fs[g_nfs] = fs;
	return g_nfs++;
}

int ksim_file_new(int fsi, u64 size, const u8 *content, const u64 *blkmap, u64 nblocks)
{
	struct ksim_fs *fs = g_fs[fsi];
	struct ksim_fsfile *ff = calloc(1, sizeof(*ff));
	const u64 bs = fs->sb.s_blocksize, npages = DIV_ROUND_UP(size, PAGE_SIZE);
	u8 *blk = calloc(1, bs);
	u64 b;

	ff->fs = fs;
	ff->inode.i_mode = 0100644;
	ff->inode.i_blkbits = (unsigned char)ilog2(bs);
	ff->inode.i_sb = &fs->sb;
	ff->inode.i_size = (loff_t)size;
	ff->inode.i_mapping = &ff->mapping;
	ff->mapping.ff = ff;
	pthread_mutex_init(&ff->m, NULL);
	ff->data = calloc(1, npages * PAGE_SIZE + bs);
	memcpy(ff->data, content, size);
	ff->pc = calloc(npages + 1, 1);
	ff->folios = calloc(npages + 1, sizeof(struct folio));
	ff->blkmap = calloc(nblocks + 1, sizeof(u64));
	memcpy(ff->blkmap, blkmap, nblocks * sizeof(u64));
	ff->nblocks = nblocks;
	for (b = 0; b < nblocks; b++) {
		if (!blkmap[b])
			continue;
		memset(blk, 0, bs);
		if (b * bs < size)
			memcpy(blk, content + b * bs, min(bs, size - b * bs));
		vol_write(fs->disk, fs->sb.s_bdev->bd_start_sect + blkmap[b] * (bs >> 9), blk, bs >> 9);
	}
	free(blk);
	g_ff[g_nff] = ff;
	return g_nff++;
}

/* open the file as a process would: an fd whose struct file points at it */
int ksim_file_open(int fi, int readable)
{
	struct ksim_fsfile *ff = g_ff[fi];
	struct ksim_file *kf = kf_new(KF_FS);

	kf->inode = &ff->inode;
	kf->obj = ff;
	kf->f.f_mode = readable ? FMODE_READ : 0;
	kf->f.f_mapping = &ff->mapping;
	return fd_install(kf);
}

/* page cache control: 0 evict, 1 clean, 2 dirty (leaves the content) */
void ksim_pc_set(int fi, u64 page, int state)
{
	struct ksim_fsfile *ff = g_ff[fi];

	pthread_mutex_lock(&ff->m);
	ff->pc[page] = (u8)state;
	pthread_mutex_unlock(&ff->m);
}

int ksim_pc_get(int fi, u64 page)
{
	struct ksim_fsfile *ff = g_ff[fi];
	int s;

	pthread_mutex_lock(&ff->m);
	s = ff->pc[page];
	pthread_mutex_unlock(&ff->m);
	return s;
}

/* a buffered write: new bytes in the page cache, dirty, not on the device */
void ksim_file_write(int fi, u64 off, const u8 *src, u64 len)
{
	struct ksim_fsfile *ff = g_ff[fi];
	u64 p;

	pthread_mutex_lock(&ff->m);
	memcpy(ff->data + off, src, len);
	for (p = off / PAGE_SIZE; p <= (off + len - 1) / PAGE_SIZE; p++)
		ff->pc[p] = 2;
	pthread_mutex_unlock(&ff->m);
}

const u8 *ksim_file_data(int fi)
{
	return g_ff[fi]->data;
}

struct folio *filemap_get_folio(struct address_space *mapping, pgoff_t index)
{
	struct ksim_fsfile *ff = mapping->ff;
	struct folio *f = ERR_PTR(-ENOENT);

	pthread_mutex_lock(&ff->m);
	if (index * PAGE_SIZE < (u64)ff->inode.i_size && ff->pc[index]) {
		f = &ff->folios[index];
		f->flags = ff->pc[index];
	}
	pthread_mutex_unlock(&ff->m);
	if (!IS_ERR(f))
		CNT_ADD(folio_refs, 1);
	return f;
}

bool folio_test_dirty(struct folio *f)
{
	return f->flags == 2;
}

void folio_put(struct folio *f)
{
	(void)f;
	CNT_ADD(folio_refs, -1);
}

int filemap_write_and_wait_range(struct address_space *mapping, loff_t lstart, loff_t lend)
{
	struct ksim_fsfile *ff = mapping->ff;
	const u64 bs = ff->fs->sb.s_blocksize;
	u64 p;

	check_sleepable("filemap_write_and_wait_range", NULL, 0);
	pthread_mutex_lock(&ff->m);
	for (p = (u64)lstart / PAGE_SIZE; p * PAGE_SIZE <= (u64)lend; p++) {
		u64 b;

		if (p * PAGE_SIZE >= (u64)ff->inode.i_size || ff->pc[p] != 2)
			continue;
		for (b = p * PAGE_SIZE / bs; b < (p + 1) * PAGE_SIZE / bs; b++)
			if (b < ff->nblocks && ff->blkmap[b])
				vol_write(ff->fs->disk,
					  ff->fs->sb.s_bdev->bd_start_sect + ff->blkmap[b] * (bs >> 9),
					  ff->data + b * bs, bs >> 9);
		ff->pc[p] = 1;
		CNT_ADD(writebacks, 1);
	}
	pthread_mutex_unlock(&ff->m);
	return 0;
}

ssize_t kernel_read(struct file *f, void *buf, size_t n, loff_t *pos)
{
	struct ksim_file *kf = kf_of(f);
	struct ksim_fsfile *ff;
	u64 end, p;

	check_sleepable("kernel_read", NULL, 0);
	if (kf->kind != KF_FS)
		return -EINVAL;
	ff = kf->obj;
	pthread_mutex_lock(&ff->m);
	if (*pos >= ff->inode.i_size) {
		pthread_mutex_unlock(&ff->m);
		return 0;
	}
	end = min((u64)*pos + n, (u64)ff->inode.i_size);
	memcpy(buf, ff->data + *pos, end - *pos);
	for (p = *pos / PAGE_SIZE; p * PAGE_SIZE < end; p++)
		if (!ff->pc[p])
			ff->pc[p] = 1;               /* a buffered read populates the cache */
	n = end - *pos;
	*pos = end;
	pthread_mutex_unlock(&ff->m);
	return (ssize_t)n;
}

int bmap(struct inode *inode, sector_t *block)
{
	struct ksim_fsfile *ff = container_of(inode, struct ksim_fsfile, inode);

	*block = *block < ff->nblocks ? ff->blkmap[*block] : 0;
	return 0;
}

/* ------------------------------------------------------------ mm / VMAs */
struct mm_struct { pthread_rwlock_t lock; };
static struct mm_struct g_mm = { PTHREAD_RWLOCK_INITIALIZER };
static struct task_struct g_task = { &g_mm };
struct task_struct *current = &g_task;

struct ksim_vma { struct vm_area_struct vma; struct page **pages; size_t npages; };
#define MAX_VMAS 64
static struct ksim_vma *g_vmas[MAX_VMAS];
static unsigned long g_next_va = 0x7f0000000000ul;
static __thread int t_mmap_locked;

void mmap_read_lock(struct mm_struct *mm)
{
	check_sleepable("mmap_read_lock", NULL, 0);
	pthread_rwlock_rdlock(&mm->lock);
	t_mmap_locked++;
}

void mmap_read_unlock(struct mm_struct *mm)
{
	t_mmap_locked--;
	pthread_rwlock_unlock(&mm->lock);
}

struct vm_area_struct *find_vma(struct mm_struct *mm, unsigned long addr)
{
	struct vm_area_struct *best = NULL;
	int i;

	(void)mm;
	if (!t_mmap_locked)
		violation("find_vma without mmap_lock");
	for (i = 0; i < MAX_VMAS; i++)
		if (g_vmas[i] && g_vmas[i]->vma.vm_end > addr &&
		    (!best || g_vmas[i]->vma.vm_start < best->vm_start))
			best = &g_vmas[i]->vma;
	return best;
}

void vm_flags_set(struct vm_area_struct *vma, unsigned long flags)
{
	vma->vm_flags |= flags;
}

static int g_last_mmap_rc;

int ksim_last_mmap_rc(void)
{
	return __atomic_load_n(&g_last_mmap_rc, __ATOMIC_SEQ_CST);
}

unsigned long ksim_mmap(int fd, u64 len, u64 off, int shared)
{
	struct file *f = fget(fd);
	struct ksim_vma *v;
	int i, rc;

	__atomic_store_n(&g_last_mmap_rc, 0, __ATOMIC_SEQ_CST);
	if (!f)
		return 0;
	v = calloc(1, sizeof(*v));
	len = (len + PAGE_SIZE - 1) & ~(PAGE_SIZE - 1);
	v->vma.vm_start = __atomic_fetch_add(&g_next_va, len + (1ul << 24), __ATOMIC_SEQ_CST);
	v->vma.vm_end = v->vma.vm_start + len;
	v->vma.vm_pgoff = off >> PAGE_SHIFT;
	v->vma.vm_flags = shared ? VM_SHARED : 0;
	v->vma.vm_file = f;                        /* the fget reference */
	v->npages = len >> PAGE_SHIFT;
	v->pages = calloc(v->npages, sizeof(*v->pages));
	rc = f->f_op && f->f_op->mmap ? f->f_op->mmap(f, &v->vma) : -ENODEV_SIM;
	if (rc) {
		__atomic_store_n(&g_last_mmap_rc, rc, __ATOMIC_SEQ_CST);
		fput(f);
		free(v->pages);
		free(v);
		return 0;
	}
	pthread_rwlock_wrlock(&g_mm.lock);
	for (i = 0; i < MAX_VMAS && g_vmas[i]; i++)
		;
	g_vmas[i] = v;
	pthread_rwlock_unlock(&g_mm.lock);
	return v->vma.vm_start;
}

int ksim_munmap(unsigned long addr)
{
	struct ksim_vma *v = NULL;
	size_t k;
	int i;

	pthread_rwlock_wrlock(&g_mm.lock);
	for (i = 0; i < MAX_VMAS; i++)
		if (g_vmas[i] && g_vmas[i]->vma.vm_start == addr) {
			v = g_vmas[i];
			g_vmas[i] = NULL;
			break;
		}
	pthread_rwlock_unlock(&g_mm.lock);
	if (!v)
		return -EINVAL;
	for (k = 0; k < v->npages; k++)
		if (v->pages[k])
			__free_page(v->pages[k]);          /* the fault's reference */
	fput(v->vma.vm_file);
	free(v->pages);
	free(v);
	return 0;
}

/* read user memory of a VMA through its fault handler (as a CPU access would) */
int ksim_user_read(unsigned long addr, void *dst, u64 len)
{
	char *out = dst;

	while (len) {
		struct ksim_vma *v = NULL;
		size_t idx, n, off;
		int i;

		pthread_rwlock_rdlock(&g_mm.lock);
		for (i = 0; i < MAX_VMAS; i++)
			if (g_vmas[i] && g_vmas[i]->vma.vm_start <= addr && addr < g_vmas[i]->vma.vm_end)
				v = g_vmas[i];
		if (!v) {
			pthread_rwlock_unlock(&g_mm.lock);
			return -EFAULT;
		}
		idx = (addr - v->vma.vm_start) >> PAGE_SHIFT;
		if (!v->pages[idx]) {
			struct vm_fault vmf = { &v->vma, v->vma.vm_pgoff + idx, NULL };

			if (v->vma.vm_ops->fault(&vmf) || !vmf.page) {
				pthread_rwlock_unlock(&g_mm.lock);
				return -EFAULT;
			}
			v->pages[idx] = vmf.page;
		}
		off = addr & (PAGE_SIZE - 1);
		n = min((u64)(PAGE_SIZE - off), len);
		memcpy(out, (char *)v->pages[idx]->kaddr + off, n);
		pthread_rwlock_unlock(&g_mm.lock);
		out += n;
		addr += n;
		len -= n;
	}
	return 0;
}

/* ------------------------------------------------------------ dma-buf exporter */
struct dma_resv { int locked; };

struct ksim_dmabuf {
	struct dma_buf db;
	struct dma_resv resv;
	int refs;
	u8 *mem;
	size_t size;
	int nsegs;
	u64 seg_off[64], seg_len[64];
	int order[64];                       /* sg order (shuffled) is still offset order */
	int npinned, nattach, nmapped;
	bool deny_p2p;
};

struct ksim_att {
	struct dma_buf_attachment a;
	struct ksim_dmabuf *b;
	struct device *dev;
	bool pinned;
};

int dma_resv_lock(struct dma_resv *obj, void *ctx)
{
	(void)ctx;
	check_sleepable("dma_resv_lock", NULL, 0);
	while (__atomic_exchange_n(&obj->locked, 1, __ATOMIC_ACQUIRE))
		usleep(10);
	t_resv_held++;
	return 0;
}

void dma_resv_unlock(struct dma_resv *obj)
{
	t_resv_held--;
	__atomic_store_n(&obj->locked, 0, __ATOMIC_RELEASE);
}

static void resv_assert_held(struct ksim_dmabuf *b, const char *what)
{
	if (!t_resv_held || !__atomic_load_n(&b->resv.locked, __ATOMIC_SEQ_CST))
		violation("%s without the reservation lock", what);
}

static void dmabuf_get(struct ksim_dmabuf *b)
{
	__atomic_add_fetch(&b->refs, 1, __ATOMIC_SEQ_CST);
}

static void dmabuf_putref(struct ksim_dmabuf *b)
{
	if (__atomic_sub_fetch(&b->refs, 1, __ATOMIC_SEQ_CST) == 0) {
		if (b->npinned || b->nattach || b->nmapped)
			violation("dma-buf freed with %d pins, %d attachments, %d maps", b->npinned,
				  b->nattach, b->nmapped);
		free(b->mem);
		free(b);
		CNT_ADD(dmabufs_live, -1);
	}
}

static void dmabuf_file_release(struct ksim_file *kf)
{
	dmabuf_putref(kf->obj);
}

/* an exporter-side buffer of `size` bytes in `nsegs` pieces (VRAM blocks) */
int ksim_dmabuf_new(u64 size, int nsegs, unsigned int seed)
{
	struct ksim_dmabuf *b = calloc(1, sizeof(*b));
	struct ksim_file *kf;
	u64 pages = size / PAGE_SIZE, left = pages, off = 0;
	int i, fd;

	if (nsegs < 1)
		nsegs = 1;
	if (nsegs > 64)
		nsegs = 64;
	b->size = size;
	b->mem = aligned_alloc(PAGE_SIZE, size);
	memset(b->mem, 0x41, size);
	b->db.size = size;
	b->db.resv = &b->resv;
	b->refs = 1;
	b->nsegs = nsegs;
	for (i = 0; i < nsegs; i++) {
		u64 n = i == nsegs - 1 ? left : max((u64)1, (left / (nsegs - i)) + (rand_r(&seed) % 3) - 1);

		if (n > left - (nsegs - i - 1))
			n = left - (nsegs - i - 1);
		b->seg_off[i] = off * PAGE_SIZE;
		b->seg_len[i] = n * PAGE_SIZE;
		off += n;
		left -= n;
	}
	CNT_ADD(dmabufs_live, 1);
	kf = kf_new(KF_DMABUF);
	kf->obj = b;
	snprintf(kf->name, sizeof(kf->name), "dmabuf:vram%llu", (unsigned long long)size);
	fd = fd_install(kf);
	return fd;
}

static struct ksim_dmabuf *dmabuf_of_fd(int fd)
{
	struct ksim_dmabuf *b = NULL;

	pthread_mutex_lock(&g_fd_m);
	if (fd >= 0 && fd < MAX_FDS && g_fds[fd] && g_fds[fd]->kind == KF_DMABUF)
		b = g_fds[fd]->obj;
	pthread_mutex_unlock(&g_fd_m);
	return b;
}

u8 *ksim_dmabuf_mem(int fd)
{
	struct ksim_dmabuf *b = dmabuf_of_fd(fd);

	return b ? b->mem : NULL;
}

void ksim_dmabuf_state(int fd, int *pinned, int *attached, int *mapped, int *refs)
{
	struct ksim_dmabuf *b = dmabuf_of_fd(fd);

	*pinned = __atomic_load_n(&b->npinned, __ATOMIC_SEQ_CST);
	*attached = __atomic_load_n(&b->nattach, __ATOMIC_SEQ_CST);
	*mapped = __atomic_load_n(&b->nmapped, __ATOMIC_SEQ_CST);
	*refs = __atomic_load_n(&b->refs, __ATOMIC_SEQ_CST);
}

void ksim_dmabuf_deny_p2p(int fd, int deny)
{
	dmabuf_of_fd(fd)->deny_p2p = deny;
}

struct dma_buf *dma_buf_get(int fd)
{
	struct ksim_dmabuf *b;

	pthread_mutex_lock(&g_fd_m);
	b = (fd >= 0 && fd < MAX_FDS && g_fds[fd] && g_fds[fd]->kind == KF_DMABUF) ?
		    g_fds[fd]->obj : NULL;
	if (b)
		dmabuf_get(b);
	pthread_mutex_unlock(&g_fd_m);
	return b ? &b->db : ERR_PTR(-EINVAL);
}

void dma_buf_put(struct dma_buf *db)
{
	dmabuf_putref(container_of(db, struct ksim_dmabuf, db));
}

struct dma_buf_attachment *dma_buf_dynamic_attach(struct dma_buf *db, struct device *dev,
						  const struct dma_buf_attach_ops *ops, void *priv)
{
	struct ksim_dmabuf *b = container_of(db, struct ksim_dmabuf, db);
	struct ksim_att *a;

	(void)priv;
	check_sleepable("dma_buf_dynamic_attach", NULL, 0);
	if (!ops || !ops->move_notify)
		violation("dynamic importer without move_notify");
	a = calloc(1, sizeof(*a));
	a->b = b;
	a->dev = dev;
	a->a.peer2peer = ops && ops->allow_peer2peer && !b->deny_p2p;
	__atomic_add_fetch(&b->nattach, 1, __ATOMIC_SEQ_CST);
	return &a->a;
}

void dma_buf_detach(struct dma_buf *db, struct dma_buf_attachment *att)
{
	struct ksim_att *a = container_of(att, struct ksim_att, a);

	(void)db;
	if (a->pinned)
		violation("detach of a pinned attachment");
	__atomic_sub_fetch(&a->b->nattach, 1, __ATOMIC_SEQ_CST);
	free(a);
}

int dma_buf_pin(struct dma_buf_attachment *att)
{
	struct ksim_att *a = container_of(att, struct ksim_att, a);

	resv_assert_held(a->b, "dma_buf_pin");
	a->pinned = true;
	__atomic_add_fetch(&a->b->npinned, 1, __ATOMIC_SEQ_CST);
	return 0;
}

void dma_buf_unpin(struct dma_buf_attachment *att)
{
	struct ksim_att *a = container_of(att, struct ksim_att, a);

	resv_assert_held(a->b, "dma_buf_unpin");
	a->pinned = false;
	__atomic_sub_fetch(&a->b->npinned, 1, __ATOMIC_SEQ_CST);
}

struct sg_table *dma_buf_map_attachment(struct dma_buf_attachment *att, enum dma_data_direction dir)
{
	struct ksim_att *a = container_of(att, struct ksim_att, a);
	struct ksim_dmabuf *b = a->b;
	struct sg_table *t;
	int i;

	(void)dir;
	resv_assert_held(b, "dma_buf_map_attachment");
	if (!a->pinned)
		violation("map of an unpinned dynamic attachment");
	if (!a->dev->iommu)
		return ERR_PTR(-EINVAL);
	t = calloc(1, sizeof(*t));
	t->sgl = calloc(b->nsegs, sizeof(*t->sgl));
	t->nents = t->orig_nents = b->nsegs;
	/* each VRAM block gets its own bus range in the importer's domain: the
	 * table is discontiguous on the bus even where VRAM is contiguous */
	for (i = 0; i < b->nsegs; i++) {
		t->sgl[i].dma_address = iommu_map(a->dev->iommu, (char *)b->mem + b->seg_off[i],
						  b->seg_len[i]);
		t->sgl[i].dma_length = (unsigned int)b->seg_len[i];
		t->sgl[i].length = (unsigned int)b->seg_len[i];
	}
	__atomic_add_fetch(&b->nmapped, 1, __ATOMIC_SEQ_CST);
	return t;
}

void dma_buf_unmap_attachment(struct dma_buf_attachment *att, struct sg_table *t,
			      enum dma_data_direction dir)
{
	struct ksim_att *a = container_of(att, struct ksim_att, a);
	unsigned int i;

	(void)dir;
	resv_assert_held(a->b, "dma_buf_unmap_attachment");
	for (i = 0; i < t->nents; i++)
		iommu_unmap(a->dev->iommu, t->sgl[i].dma_address, t->sgl[i].dma_length);
	free(t->sgl);
	free(t);
	__atomic_sub_fetch(&a->b->nmapped, 1, __ATOMIC_SEQ_CST);
}

/* ------------------------------------------------------------ misc + proc */
static struct miscdevice *g_misc;
static const struct proc_ops *g_proc_ops;
static int g_proc_token;

int misc_register(struct miscdevice *m)
{
	g_misc = m;
	return 0;
}

void misc_deregister(struct miscdevice *m)
{
	if (g_misc == m)
		g_misc = NULL;
}

struct proc_dir_entry *proc_create(const char *name, unsigned short mode,
				   struct proc_dir_entry *parent, const struct proc_ops *ops)
{
	(void)name;
	(void)mode;
	(void)parent;
	g_proc_ops = ops;
	return (struct proc_dir_entry *)&g_proc_token;
}

void proc_remove(struct proc_dir_entry *e)
{
	(void)e;
	g_proc_ops = NULL;
}

/* /proc/nvme-strom opened through proc_ops: a file_operations adapter */
static int proc_release_adapter(struct inode *i, struct file *f)
{
	return g_proc_ops->proc_release(i, f);
}

static long proc_ioctl_adapter(struct file *f, unsigned int cmd, unsigned long arg)
{
	return g_proc_ops->proc_ioctl(f, cmd, arg);
}

static ssize_t proc_read_adapter(struct file *f, char __user *b, size_t n, loff_t *pos)
{
	return g_proc_ops->proc_read(f, b, n, pos);
}

static const struct file_operations proc_fops_adapter = {
	.release = proc_release_adapter,
	.read = proc_read_adapter,
	.unlocked_ioctl = proc_ioctl_adapter,
};

int ksim_dev_open(int via_proc)
{
	struct ksim_file *kf = kf_new(KF_DEV);
	int rc;

	if (via_proc) {
		if (!g_proc_ops)
			return -ENOENT;
		kf->f.f_op = &proc_fops_adapter;
		rc = g_proc_ops->proc_open(kf->inode, &kf->f);
	} else {
		if (!g_misc)
			return -ENOENT;
		if (!(g_misc->mode & 0004))
			return -EACCES;
		kf->f.f_op = g_misc->fops;
		rc = kf->f.f_op->open(kf->inode, &kf->f);
	}
	if (rc) {
		CNT_ADD(files_live, -1);
		free(kf);
		return rc;
	}
	return fd_install(kf);
}

long ksim_ioctl(int fd, unsigned int cmd, void *arg)
{
	struct file *f = fget(fd);
	long rc;

	if (!f)
		return -EBADF;
	rc = f->f_op->unlocked_ioctl(f, cmd, (unsigned long)arg);
	fput(f);
	return rc;
}

long ksim_read(int fd, void *buf, u64 n)
{
	struct file *f = fget(fd);
	loff_t pos = 0;
	long rc;

	if (!f)
		return -EBADF;
	rc = f->f_op->read(f, buf, n, &pos);
	fput(f);
	return rc;
}

/* ------------------------------------------------------------ world */
int kshim_module_init(void);
void kshim_module_exit(void);

int ksim_init(void)
{
	memset(&g_cnt, 0, sizeof(g_cnt));
	g_viol_msg[0] = 0;
	g_fput_wq = alloc_workqueue("delayed_fput", 0, 0);
	g_admin = 0;
	g_signal = 0;
	t_euid = 1000;
	ksim_fail_cmd(0, 0);
	ksim_fail_map(0);
	return 0;
}

int ksim_module_load(void)
{
	return kshim_module_init();
}

void ksim_module_unload(void)
{
	kshim_module_exit();
}

/* let in-flight requests complete (unless their controller is held) and
 * deferred work (delayed fputs) run out */
void ksim_quiesce(void)
{
	for (;;) {
		s64 held = 0;
		int i;

		for (i = 0; i < g_nctrls; i++) {
			pthread_mutex_lock(&g_ctrls[i]->m);
			if (g_ctrls[i]->hold)
				held += g_ctrls[i]->nq;
			pthread_mutex_unlock(&g_ctrls[i]->m);
		}
		wq_drain(g_fput_wq);
		if (__atomic_load_n(&g_cnt.requests_live, __ATOMIC_SEQ_CST) <= held)
			break;
		usleep(100);
	}
	wq_drain(g_fput_wq);
}

/* tear the world down; leaks and violations stay readable in the counters */
void ksim_fini(void)
{
	int i;

	ksim_quiesce();
	for (i = 0; i < g_nctrls; i++) {
		struct ksim_ctrl *c = g_ctrls[i];

		pthread_mutex_lock(&c->m);
		c->stop = true;
		c->hold = false;
		pthread_cond_broadcast(&c->c);
		pthread_mutex_unlock(&c->m);
		pthread_join(c->th, NULL);
	}
	destroy_workqueue(g_fput_wq);
	for (i = 0; i < MAX_FDS; i++)
		if (g_fds[i]) {
			CNT_ADD(fds_leaked, 1);
			ksim_close(i);
		}
	for (i = 0; i < g_ndisks; i++) {
		struct ksim_disk *d = g_disks[i];

		if (d->part0.bd_device.krefs)
			CNT_ADD(dev_refs_leaked, d->part0.bd_device.krefs);
		free(d->image);
		free(d);
		g_disks[i] = NULL;
	}
	for (i = 0; i < g_nctrls; i++) {
		struct ksim_ctrl *c = g_ctrls[i];

		if (c->pci.krefs)
			CNT_ADD(dev_refs_leaked, c->pci.krefs);
		if (c->pci.iommu->used)
			CNT_ADD(iommu_pages_leaked, c->pci.iommu->used);
		iommu_free(c->pci.iommu);
		pthread_mutex_destroy(&c->m);
		pthread_cond_destroy(&c->c);
		free(c);
		g_ctrls[i] = NULL;
	}
	for (i = 0; i < g_nff; i++) {
		struct ksim_fsfile *ff = g_ff[i];

		free(ff->data);
		free(ff->pc);
		free(ff->folios);
		free(ff->blkmap);
		pthread_mutex_destroy(&ff->m);
		free(ff);
	}
	for (i = 0; i < g_nfs; i++) {
		free((char *)g_fs[i]->type.name);
		free(g_fs[i]);
	}
	g_ndisks = g_nctrls = g_nff = g_nfs = g_ndevs = 0;
	memset(g_next_minor, 0, sizeof(g_next_minor));
	ksim_poison_user(NULL, 0);
}

void ksim_counters(struct ksim_counters *out)
{
	const int64_t *src = (const int64_t *)&g_cnt;
	int64_t *dst = (int64_t *)out;
	size_t i;

	for (i = 0; i < sizeof(g_cnt) / sizeof(int64_t); i++)
		dst[i] = __atomic_load_n(&src[i], __ATOMIC_SEQ_CST);
}

const char *ksim_last_violation(void)
{
	return g_viol_msg;
}
