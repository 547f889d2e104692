/* kshim.h — a behavioural MODEL of the Linux (6.8 .. 6.18) kernel API surface
 * the nvme-strom module uses.
 *
 * Two uses:
 *  1. `gcc -fsyntax-only` type-checks the module sources against it on a
 *     machine without kernel headers, on each side of the version gates
 *     (tests/test_kmod_core_cpu.py::test_kmod_sources_typecheck_against_api_model);
 *  2. kshim_rt.c IMPLEMENTS it in userspace — blk-mq queues completing on
 *     other threads ("IRQ context"), a fake NVMe controller that validates
 *     every READ against the spec, per-device IOMMU domains, a dma-buf
 *     exporter with reservation-lock rules, a page cache with clean and dirty
 *     pages, ext4-like block maps, md raid0 volumes, workqueues, file
 *     refcounts with deferred release — so the REAL kmod/strom_*.c files are
 *     linked and executed through their ioctl entry points
 *     (kmod/testshim/kmod_exec.c, tests/test_kmod_exec_cpu.py), plain and
 *     under ASAN+UBSAN and TSAN.
 *
 * Every declaration follows the kernel's public headers in that range
 * (include/linux/{blkdev,blk-mq,dma-buf,fs,device,...}.h).  Struct members
 * marked "model" do not exist in the kernel: the runtime's bookkeeping.  It
 * is not a kernel and proves nothing about ABI; kmod/kernel-check.sh checks
 * the real tree.  What it does check at run time: the module's use of the
 * API contracts it models (sleeping in IRQ context or under a spinlock,
 * dma-buf pin/map without the reservation lock, DMA to addresses not mapped
 * for the issuing device, PRP rules, leaked mappings/pages/references).
 */
#ifndef KSHIM_H
#define KSHIM_H
#include <stddef.h>
#include <stdbool.h>
#include <stdint.h>
#include <limits.h>

#define KERNEL_VERSION(a, b, c) (((a) << 16) + ((b) << 8) + (c))
#ifndef KSHIM_VERSION                 /* -DKSHIM_VERSION=... checks the other gates */
#define KSHIM_VERSION KERNEL_VERSION(6, 18, 0)
#endif
#define LINUX_VERSION_CODE KSHIM_VERSION
#define UTS_RELEASE "6.18.0-shim"
#define __LITTLE_ENDIAN 1234
#define __user
#define __init
#define __exit
#define __always_unused
#define likely(x) (x)
#define unlikely(x) (x)

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t s64;
typedef u16 __le16;
typedef u32 __le32;
typedef u64 __le64;
typedef u32 __u32;
typedef u64 __u64;
typedef long loff_t;                 /* glibc's width: the runtime includes both */
typedef long ssize_t;
typedef u64 sector_t;
typedef unsigned long dev_t;
typedef u64 dma_addr_t;
typedef unsigned int gfp_t;
typedef unsigned int blk_mode_t;
typedef u8 blk_status_t;
typedef unsigned int vm_fault_t;
typedef unsigned long pgoff_t;
typedef struct { int counter; } atomic_t;
typedef struct { s64 counter; } atomic64_t;
typedef struct { unsigned int val; } kuid_t;
typedef struct { int locked; } spinlock_t;           /* model: test-and-set word */
typedef struct { int x; } wait_queue_head_t;
typedef unsigned int fmode_t;

#define EPERM 1
#define ENOENT 2
#define EINTR 4
#define EIO 5
#define ENXIO 6
#define E2BIG 7
#define EBADF 9
#define ENOMEM 12
#define EACCES 13
#define EFAULT 14
#define ENODEV 19
#define EINVAL 22
#define ERANGE 34
#define ESPIPE 29
#define ENODATA 61
#define ETIME 62
#define EOPNOTSUPP 95
#define ERESTARTSYS 512
#define ENOIOCTLCMD 515

#define GFP_KERNEL 0u
#define GFP_ATOMIC 2u
#define __GFP_ZERO 1u
#define PAGE_SHIFT 12
#define PAGE_SIZE (1UL << PAGE_SHIFT)
#define SECTOR_SHIFT 9
#define HZ 250
#define MAX_SCHEDULE_TIMEOUT LONG_MAX
#define NUMA_NO_NODE (-1)
#define DMA_BIT_MASK(n) (((n) == 64) ? ~0ULL : ((1ULL << (n)) - 1))
#define DMA_MAPPING_ERROR (~(dma_addr_t)0)
#define FMODE_READ 1u
#define BLK_OPEN_READ 1u
#define S_ISREG(m) (((m) & 0170000) == 0100000)
#define S_ISDIR(m) (((m) & 0170000) == 0040000)
#define O_RDWR 2
#define O_CLOEXEC 02000000
#define VM_SHARED 0x8ul
#define VM_DONTEXPAND 0x40000ul
#define VM_DONTDUMP 0x4000000ul
#define VM_FAULT_SIGBUS 0x2u
#define CAP_SYS_ADMIN 21
#define MISC_DYNAMIC_MINOR 255
#define WQ_UNBOUND 2
#define TASK_UNINTERRUPTIBLE 2

#define ARRAY_SIZE(a) (sizeof(a) / sizeof((a)[0]))
#define DIV_ROUND_UP(n, d) (((n) + (d) - 1) / (d))
#define round_up(x, y) ((((x) - 1) | ((__typeof__(x))((y) - 1))) + 1)
#define min(a, b) ((a) < (b) ? (a) : (b))
#define max(a, b) ((a) > (b) ? (a) : (b))
#define min_t(t, a, b) ((t)(a) < (t)(b) ? (t)(a) : (t)(b))
#define container_of(p, t, m) ((t *)((char *)(p) - offsetof(t, m)))
#define struct_size(p, m, n) (sizeof(*(p)) + sizeof((p)->m[0]) * (n))
#define IS_ERR(p) ((unsigned long)(p) > (unsigned long)-4096)
#define IS_ERR_OR_NULL(p) (!(p) || IS_ERR(p))
#define PTR_ERR(p) ((long)(p))
#define ERR_PTR(e) ((void *)(long)(e))
void kshim_bug(const char *what, const char *file, int line);
#define BUG_ON(c) do { if (c) kshim_bug(#c, __FILE__, __LINE__); } while (0)
void kshim_warn(const char *what, const char *file, int line);
#define WARN_ON_ONCE(c) ({ int __w = !!(c); if (__w) kshim_warn(#c, __FILE__, __LINE__); __w; })
void kshim_might_sleep(const char *file, int line);
#define might_sleep() kshim_might_sleep(__FILE__, __LINE__)
void kshim_printk(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
#define pr_info(...) kshim_printk(__VA_ARGS__)
#define pr_notice(...) kshim_printk(__VA_ARGS__)
#define pr_warn(...) kshim_printk(__VA_ARGS__)
#define cmpxchg(p, o, n) __sync_val_compare_and_swap(p, o, n)
#define uid_eq(a, b) ((a).val == (b).val)
#define MKDEV(ma, mi) (((ma) << 20) | (mi))
#define cpu_to_le16(x) ((__le16)(x))
#define cpu_to_le32(x) ((__le32)(x))
#define cpu_to_le64(x) ((__le64)(x))
#define ilog2(n) (63 - __builtin_clzll(n))
/* user pointers are host pointers in the model; kshim_uaccess_ok() knows
 * the "unmapped" ones (NULL page, harness-poisoned ranges) */
bool kshim_uaccess_ok(const void *p, size_t n);
#define put_user(x, p) (kshim_uaccess_ok((p), sizeof(*(p))) ? (*(p) = (x), 0) : -EFAULT)
#define get_user(x, p) (kshim_uaccess_ok((p), sizeof(*(p))) ? ((x) = *(p), 0) : -EFAULT)
#define dev_is_pci(d) ((d)->bus == &pci_bus_type)
#define DEFINE_SPINLOCK(x) spinlock_t x = { 0 }
#define DEFINE_MUTEX(x) struct mutex x = { 0 }
#define LIST_HEAD(x) struct list_head x = { &(x), &(x) }
#define DEFINE_HASHTABLE(n, bits) struct hlist_head n[1 << (bits)]
#define ATOMIC64_INIT(i) { (i) }
#define EXPORT_SYMBOL(x)
#define MODULE_AUTHOR(x)
#define MODULE_DESCRIPTION(x)
#define MODULE_VERSION(x)
#define MODULE_LICENSE(x)
#define MODULE_IMPORT_NS(x)
#define MODULE_PARM_DESC(a, b)
#define module_param_named(a, b, t, p)
#define module_init(f) int kshim_module_init(void) { return f(); }  /* not init_module: libc has one */
#define module_exit(f) void kshim_module_exit(void) { f(); }
#define THIS_MODULE ((struct module *)0)
#define __stringify(x) #x

struct module;
struct list_head { struct list_head *next, *prev; };
struct hlist_node { struct hlist_node *next, **pprev; };
struct hlist_head { struct hlist_node *first; };
struct mutex { int locked; };                        /* model: sleeping lock word */
struct kref { atomic_t refcount; };
struct work_struct {
	void (*func)(struct work_struct *);
	struct work_struct *next;                     /* model: queue link */
	int pending;                                  /* model */
};
struct workqueue_struct;
struct srcu_struct;
struct rcu_head { void *p; };
struct bus_type { const char *name; };
struct class { const char *name; };
struct kshim_iommu;
struct device {
	struct device *parent;
	const struct bus_type *bus;
	const struct class *class;
	/* model */
	char kname[40];
	int krefs;
	int numa_node;
	u64 dma_mask;
	struct kshim_iommu *iommu;
};
struct page {
	unsigned long flags;
	/* model */
	void *kaddr;
	int refcount;
	struct kshim_pblock *blk;
};
struct folio { unsigned long flags; };
struct address_space;
struct super_block;
struct file_system_type { const char *name; };
struct block_device;
struct inode {
	unsigned int i_mode;
	unsigned char i_blkbits;
	struct super_block *i_sb;
	loff_t i_size;                                /* model: i_size_read() */
	struct address_space *i_mapping;
};
struct super_block { unsigned long s_blocksize; struct file_system_type *s_type; struct block_device *s_bdev; };
struct file { fmode_t f_mode; struct address_space *f_mapping; void *private_data; const struct file_operations *f_op; };
struct fd { struct file *file; };
#if KSHIM_VERSION >= KERNEL_VERSION(6, 12, 0)
#define fd_file(f) ((f).file)
#endif
struct vm_area_struct { unsigned long vm_start, vm_end, vm_pgoff, vm_flags; struct file *vm_file;
	const struct vm_operations_struct *vm_ops; };
static inline unsigned long vma_pages(const struct vm_area_struct *v)
{
	return (v->vm_end - v->vm_start) >> PAGE_SHIFT;
}
struct vm_fault { struct vm_area_struct *vma; pgoff_t pgoff; struct page *page; };
struct vm_operations_struct { vm_fault_t (*fault)(struct vm_fault *); };
struct mm_struct;
struct task_struct { struct mm_struct *mm; };
extern struct task_struct *current;
struct file_operations {
	struct module *owner;
	int (*open)(struct inode *, struct file *);
	int (*release)(struct inode *, struct file *);
	ssize_t (*read)(struct file *, char __user *, size_t, loff_t *);
	long (*unlocked_ioctl)(struct file *, unsigned int, unsigned long);
	long (*compat_ioctl)(struct file *, unsigned int, unsigned long);
	int (*mmap)(struct file *, struct vm_area_struct *);
};
struct proc_ops {
	int (*proc_open)(struct inode *, struct file *);
	int (*proc_release)(struct inode *, struct file *);
	ssize_t (*proc_read)(struct file *, char __user *, size_t, loff_t *);
	long (*proc_ioctl)(struct file *, unsigned int, unsigned long);
};
struct proc_dir_entry;
struct miscdevice { int minor; const char *name; const struct file_operations *fops; unsigned short mode; };

/* block layer */
struct request_queue;
struct block_device_operations {
	int (*ioctl)(struct block_device *, blk_mode_t, unsigned int, unsigned long);
};
struct gendisk {
	int major, first_minor;
	char disk_name[32];
	const struct block_device_operations *fops;
	struct request_queue *queue;
	struct block_device *part0;
	u64 diskseq;
};
struct block_device {
	struct gendisk *bd_disk;
	sector_t bd_start_sect;
	struct device bd_device;
	/* model: /proc/diskstats of this block device */
	unsigned long kios, ksectors;
	long kinflight;
};
struct bdev_handle { struct block_device *bdev; };
enum req_op { REQ_OP_READ = 0, REQ_OP_DRV_IN = 34 };
enum rq_end_io_ret { RQ_END_IO_NONE, RQ_END_IO_FREE };
struct request;
typedef enum rq_end_io_ret (rq_end_io_fn)(struct request *, blk_status_t);
struct nvme_command;
struct request {
	unsigned int timeout;
	rq_end_io_fn *end_io;
	void *end_io_data;
	/* model */
	struct request_queue *q;
	struct nvme_command *cmd;                     /* nvme_init_request() */
	unsigned int opf;
	struct request *knext;
};
struct request *blk_mq_alloc_request(struct request_queue *q, unsigned int opf, unsigned int flags);
void blk_execute_rq_nowait(struct request *rq, bool at_head);
int blk_status_to_errno(blk_status_t status);
bool queue_is_mq(struct request_queue *q);
unsigned int queue_logical_block_size(const struct request_queue *q);
unsigned int queue_max_hw_sectors(const struct request_queue *q);
sector_t get_capacity(struct gendisk *disk);
sector_t get_start_sect(struct block_device *bdev);
dev_t disk_devt(struct gendisk *disk);
bool disk_live(struct gendisk *disk);
#define disk_to_dev(disk) (&((disk)->part0->bd_device))
#define dev_to_bdev(d) container_of(d, struct block_device, bd_device)
#define dev_to_disk(d) (dev_to_bdev(d)->bd_disk)
unsigned long bdev_start_io_acct(struct block_device *bdev, enum req_op op, unsigned long start_time);
void bdev_end_io_acct(struct block_device *bdev, enum req_op op, unsigned int sectors,
		      unsigned long start_time);
struct file *bdev_file_open_by_dev(dev_t dev, blk_mode_t mode, void *holder, const void *hops);
struct block_device *file_bdev(struct file *bdev_file);
struct bdev_handle *bdev_open_by_dev(dev_t dev, blk_mode_t mode, void *holder, const void *hops);
void bdev_release(struct bdev_handle *handle);
extern unsigned long jiffies;
unsigned long nsecs_to_jiffies(u64 n);
int bmap(struct inode *inode, sector_t *block);

/* nvme (include/linux/nvme.h) */
#define NVME_IOCTL_ID 0x4e40
enum nvme_opcode { nvme_cmd_read = 0x02 };
union nvme_data_ptr { struct { __le64 prp1; __le64 prp2; }; };
struct nvme_rw_command {
	u8 opcode, flags; u16 command_id; __le32 nsid; __le32 cdw2, cdw3; __le64 metadata;
	union nvme_data_ptr dptr; __le64 slba; __le16 length, control; __le32 dsmgmt, reftag;
	__le16 lbat, lbatm;
};
struct nvme_command { union { struct nvme_rw_command rw; }; };

/* dma / dma-buf */
enum dma_data_direction { DMA_BIDIRECTIONAL = 0, DMA_FROM_DEVICE = 2 };
struct scatterlist { unsigned long page_link; unsigned int offset, length; dma_addr_t dma_address; unsigned int dma_length; };
struct sg_table { struct scatterlist *sgl; unsigned int nents, orig_nents; };
#define sg_dma_address(sg) ((sg)->dma_address)
#define sg_dma_len(sg) ((sg)->dma_length)
#define for_each_sgtable_dma_sg(sgt, sg, i) for ((i) = 0, (sg) = (sgt)->sgl; (i) < (int)(sgt)->nents; (i)++, (sg)++)
struct dma_resv;
struct dma_buf { size_t size; struct dma_resv *resv; };
struct dma_buf_attachment { bool peer2peer; };
struct dma_buf_attach_ops { bool allow_peer2peer; void (*move_notify)(struct dma_buf_attachment *); };
struct dma_buf *dma_buf_get(int fd);
void dma_buf_put(struct dma_buf *);
struct dma_buf_attachment *dma_buf_dynamic_attach(struct dma_buf *, struct device *,
		const struct dma_buf_attach_ops *, void *importer_priv);
void dma_buf_detach(struct dma_buf *, struct dma_buf_attachment *);
int dma_buf_pin(struct dma_buf_attachment *);
void dma_buf_unpin(struct dma_buf_attachment *);
struct sg_table *dma_buf_map_attachment(struct dma_buf_attachment *, enum dma_data_direction);
void dma_buf_unmap_attachment(struct dma_buf_attachment *, struct sg_table *, enum dma_data_direction);
int dma_resv_lock(struct dma_resv *obj, void *ctx);
void dma_resv_unlock(struct dma_resv *obj);
struct dma_pool;
struct dma_pool *dma_pool_create(const char *, struct device *, size_t size, size_t align, size_t boundary);
void dma_pool_destroy(struct dma_pool *);
void *dma_pool_alloc(struct dma_pool *, gfp_t, dma_addr_t *);
void dma_pool_free(struct dma_pool *, void *, dma_addr_t);
dma_addr_t dma_map_page(struct device *, struct page *, size_t off, size_t sz, enum dma_data_direction);
void dma_unmap_page(struct device *, dma_addr_t, size_t, enum dma_data_direction);
void dma_sync_single_for_cpu(struct device *, dma_addr_t, size_t, enum dma_data_direction);
int dma_mapping_error(struct device *, dma_addr_t);
u64 dma_get_mask(struct device *);
int dev_to_node(struct device *);

/* devices */
extern const struct bus_type pci_bus_type;
struct device *get_device(struct device *);
void put_device(struct device *);
struct device *bus_find_device_by_name(const struct bus_type *, struct device *start, const char *name);
struct device *device_find_child_by_name(struct device *parent, const char *name);
int misc_register(struct miscdevice *);
void misc_deregister(struct miscdevice *);
struct proc_dir_entry *proc_create(const char *, unsigned short, struct proc_dir_entry *, const struct proc_ops *);
void proc_remove(struct proc_dir_entry *);
bool capable(int cap);

/* files, mm */
struct file *fget(unsigned int fd);
void fput(struct file *);
struct file *get_file(struct file *f);
struct fd fdget(unsigned int fd);
void fdput(struct fd fd);
struct inode *file_inode(const struct file *f);
loff_t i_size_read(const struct inode *inode);
ssize_t kernel_read(struct file *, void *, size_t, loff_t *);
ssize_t simple_read_from_buffer(void __user *to, size_t count, loff_t *ppos, const void *from, size_t available);
long compat_ptr_ioctl(struct file *file, unsigned int cmd, unsigned long arg);
int anon_inode_getfd(const char *name, const struct file_operations *fops, void *priv, int flags);
struct folio *filemap_get_folio(struct address_space *mapping, pgoff_t index);
bool folio_test_dirty(struct folio *);
void folio_put(struct folio *);
int filemap_write_and_wait_range(struct address_space *mapping, loff_t lstart, loff_t lend);
void mmap_read_lock(struct mm_struct *);
void mmap_read_unlock(struct mm_struct *);
struct vm_area_struct *find_vma(struct mm_struct *, unsigned long addr);
void vm_flags_set(struct vm_area_struct *, unsigned long);
struct page *alloc_pages_node(int nid, gfp_t gfp, unsigned int order);
void split_page(struct page *, unsigned int order);
void __free_page(struct page *);
void get_page(struct page *);
unsigned long __get_free_page(gfp_t);
void free_page(unsigned long);
void *kmap_local_page(struct page *);
void kunmap_local(const void *);
int numa_node_id(void);
extern unsigned int nr_node_ids;
bool node_online(int nid);

/* memory + strings */
void *kzalloc(size_t, gfp_t);
void *kmalloc_array(size_t n, size_t size, gfp_t);
void *krealloc_array(void *p, size_t n, size_t size, gfp_t);
void *kvmalloc_array(size_t n, size_t size, gfp_t);
void kfree(const void *);
void kvfree(const void *);
void *memdup_user(const void __user *, size_t);
void *memset(void *, int, size_t);
void *memcpy(void *, const void *, size_t);
int strcmp(const char *, const char *);
int sscanf(const char *, const char *, ...);
int strncmp(const char *, const char *, size_t);
char *strchr(const char *, int);
long strscpy(char *dst, const char *src, size_t count);
int snprintf(char *buf, size_t size, const char *fmt, ...);
unsigned long copy_from_user(void *to, const void __user *from, unsigned long n);
unsigned long copy_to_user(void __user *to, const void *from, unsigned long n);
unsigned long clear_user(void __user *to, unsigned long n);

/* sync: spinlocks spin (and mark the thread atomic), mutexes and waits
 * sleep — the runtime checks that nothing sleeps in IRQ context or under a
 * spinlock */
void spin_lock_init(spinlock_t *);
void spin_lock(spinlock_t *);
void spin_unlock(spinlock_t *);
void spin_lock_irq(spinlock_t *);
void spin_unlock_irq(spinlock_t *);
#define spin_lock_irqsave(l, f) ((f) = 0, spin_lock(l))
#define spin_unlock_irqrestore(l, f) ((void)(f), spin_unlock(l))
void mutex_init(struct mutex *);
void mutex_lock(struct mutex *);
void mutex_unlock(struct mutex *);
void init_waitqueue_head(wait_queue_head_t *);
void wake_up_all(wait_queue_head_t *);
/* one sleep slice on a wait queue (bounded, so a wakeup racing the
 * condition check costs at most a slice); asserts a sleepable context */
void kshim_wait_slice(wait_queue_head_t *wq, const char *file, int line);
u64 kshim_now_ns(void);
bool kshim_signal_pending(void);
#define wait_event(wq, cond)                                                   \
	do {                                                                   \
		while (!(cond))                                                \
			kshim_wait_slice(&(wq), __FILE__, __LINE__);            \
	} while (0)
#define wait_event_interruptible_timeout(wq, cond, timeout)                    \
	({                                                                     \
		long __to = (timeout), __ret;                                  \
		u64 __dl = __to == MAX_SCHEDULE_TIMEOUT ? UINT64_MAX :         \
			   kshim_now_ns() + (u64)__to * (1000000000ull / HZ);  \
		for (;;) {                                                     \
			u64 __now;                                             \
			if (cond) {                                            \
				__now = kshim_now_ns();                        \
				__ret = __dl == UINT64_MAX ? __to :            \
					max(1L, (long)((__dl > __now ? __dl - __now : 0) / (1000000000ull / HZ))); \
				break;                                         \
			}                                                      \
			if (kshim_signal_pending()) {                          \
				__ret = -ERESTARTSYS;                          \
				break;                                         \
			}                                                      \
			if (kshim_now_ns() >= __dl) {                          \
				__ret = (cond) ? 1 : 0;                        \
				break;                                         \
			}                                                      \
			kshim_wait_slice(&(wq), __FILE__, __LINE__);            \
		}                                                              \
		__ret;                                                         \
	})
void kref_init(struct kref *);
void kref_get(struct kref *);
int kref_put(struct kref *, void (*release)(struct kref *));
void atomic_set(atomic_t *, int);
int atomic_read(const atomic_t *);
void atomic_inc(atomic_t *);
bool atomic_dec_and_test(atomic_t *);
s64 atomic64_read(const atomic64_t *);
void atomic64_inc(atomic64_t *);
void atomic64_dec(atomic64_t *);
void atomic64_add(s64, atomic64_t *);
s64 atomic64_inc_return(atomic64_t *);
s64 atomic64_cmpxchg(atomic64_t *, s64, s64);
s64 atomic64_xchg(atomic64_t *, s64);
#define INIT_WORK(w, f) ((w)->func = (f), (w)->next = NULL, (w)->pending = 0)
struct workqueue_struct *alloc_workqueue(const char *fmt, unsigned int flags, int max_active, ...);
bool queue_work(struct workqueue_struct *, struct work_struct *);
void destroy_workqueue(struct workqueue_struct *);
void __module_get(struct module *);
void module_put(struct module *);
u64 rdtsc_ordered(void);
kuid_t current_euid(void);
unsigned int from_kuid(void *ns, kuid_t uid);
void *current_user_ns(void);
unsigned int hash_long(unsigned long v, unsigned int bits);

/* lists + hashtables */
#define INIT_LIST_HEAD(l) ((l)->next = (l)->prev = (l))
void list_add(struct list_head *n, struct list_head *h);
void list_add_tail(struct list_head *n, struct list_head *h);
void list_del(struct list_head *e);
#define list_entry(p, t, m) container_of(p, t, m)
#define list_for_each_entry(pos, head, member) \
	for (pos = list_entry((head)->next, __typeof__(*pos), member); &pos->member != (head); \
	     pos = list_entry(pos->member.next, __typeof__(*pos), member))
#define list_for_each_entry_safe(pos, n, head, member) \
	for (pos = list_entry((head)->next, __typeof__(*pos), member), \
	     n = list_entry(pos->member.next, __typeof__(*pos), member); &pos->member != (head); \
	     pos = n, n = list_entry(n->member.next, __typeof__(*n), member))
#define INIT_HLIST_HEAD(h) ((h)->first = NULL)
void hlist_add_head(struct hlist_node *n, struct hlist_head *h);
void hlist_del(struct hlist_node *n);
#define hlist_entry_safe(p, t, m) ((p) ? container_of(p, t, m) : NULL)
#define hlist_for_each_entry(pos, head, member) \
	for (pos = hlist_entry_safe((head)->first, __typeof__(*(pos)), member); pos; \
	     pos = hlist_entry_safe((pos)->member.next, __typeof__(*(pos)), member))
#define hash_init(t) do { for (size_t __i = 0; __i < ARRAY_SIZE(t); __i++) INIT_HLIST_HEAD(&(t)[__i]); } while (0)
#define hash_add(t, n, key) hlist_add_head(n, &(t)[hash_long((unsigned long)(key), ilog2(ARRAY_SIZE(t)))])
#define hash_del(n) hlist_del(n)
#define hash_for_each_possible(t, obj, member, key) \
	hlist_for_each_entry(obj, &(t)[hash_long((unsigned long)(key), ilog2(ARRAY_SIZE(t)))], member)
#define hash_for_each(t, bkt, obj, member) \
	for ((bkt) = 0; (bkt) < (int)ARRAY_SIZE(t); (bkt)++) hlist_for_each_entry(obj, &(t)[bkt], member)
#endif
