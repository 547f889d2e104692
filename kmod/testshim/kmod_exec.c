/* kmod_exec.c — executes the kernel provider (kmod/strom_*.c, unmodified)
 * on the CPU, through its misc-device fops, against the behavioural kernel
 * model (kshim_rt.c).  VERDICT r2 #2: the submission path, completions in
 * IRQ context, task lifetime, dma-buf import, page-cache copies and the
 * error drain had only been type-checked.
 *
 *   build/kmod_exec [scenario...]          (plain, -asan, -tsan builds)
 *
 * Every scenario builds a fresh machine, loads the module, runs ioctls,
 * checks bytes and counters against an independent model of the expected
 * result, closes everything, unloads, and then requires the model's
 * contract counters to be clean: no violation (sleep in IRQ context or
 * under a spinlock, resv-lock rules, DMA to addresses the controller has no
 * mapping for, PRP rule breaks, ...) and nothing leaked (allocations, pages,
 * IOMMU mappings, requests, files, device/module references, dma-bufs).
 *
 * Reference behaviour exercised (kmod/nvme_strom.c): SSD2GPU landing and
 * chunk_ids rewrite :1546-1571, page-cache hybrid :1532-1557, relseg :1524,
 * SSD2RAM identity landing :1767-1884, async READ + completion :994-1120,
 * failed-task list / WAIT -EIO+status :680-715 :1150-1170, release reclaim
 * :2064-2091, raid0 remap :755-820, diskstats on member and md :1012-1034,
 * STAT_INFO :1986-2028, GPU map registry :216-495 (as dma-buf import).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "strom/uapi.h"
#include "kshim_sim.h"

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

static int g_failures;
static const char *g_scn;

#define CHECK(c)                                                                     \
	do {                                                                         \
		if (!(c)) {                                                          \
			fprintf(stderr, "[%s] %s:%d: CHECK(%s) failed\n", g_scn, __FILE__, \
				__LINE__, #c);                                       \
			g_failures++;                                                \
			return 1;                                                    \
		}                                                                    \
	} while (0)
#define CHECK_EQ(a, b)                                                                   \
	do {                                                                             \
		long long __a = (long long)(a), __b = (long long)(b);                    \
		if (__a != __b) {                                                        \
			fprintf(stderr, "[%s] %s:%d: %s == %lld, expected %s == %lld\n", g_scn, \
				__FILE__, __LINE__, #a, __a, #b, __b);                   \
			g_failures++;                                                    \
			return 1;                                                        \
		}                                                                        \
	} while (0)

/* ------------------------------------------------------------ helpers */
static u32 rnd(u32 *s)
{
	*s ^= *s << 13;
	*s ^= *s >> 17;
	*s ^= *s << 5;
	return *s;
}

static u8 *rand_bytes(u64 n, u32 seed)
{
	u8 *p = malloc(n);
	u64 i;

	for (i = 0; i < n; i++)
		p[i] = (u8)(rnd(&seed) >> 7);
	return p;
}

struct fmodel {                          /* what a file is, for the expectations */
	int fi;                          /* sim file index */
	u64 size;
	u8 *data;                        /* logical content (kept in sync with writes) */
};

/* A fragmented block map: extents of 1..max_ext blocks placed at scattered,
 * non-overlapping device blocks from `base`, some in reverse device order,
 * with optional holes (blkmap 0) */
static u64 *frag_map(u64 nblocks, u64 base, u32 seed, int max_ext)
{
	u64 *m = calloc(nblocks, sizeof(u64));
	u64 b = 0, dev = base;

	while (b < nblocks) {
		u64 n = 1 + rnd(&seed) % (u32)max_ext, k;

		if (n > nblocks - b)
			n = nblocks - b;
		dev += rnd(&seed) % 7;                  /* gap */
		for (k = 0; k < n; k++)
			m[b + k] = dev + k;
		dev += n;
		b += n;
	}
	return m;
}

static u64 *linear_map(u64 nblocks, u64 base)
{
	u64 *m = calloc(nblocks, sizeof(u64)), i;

	for (i = 0; i < nblocks; i++)
		m[i] = base + i;
	return m;
}

static struct fmodel new_file(int fs, u64 size, u32 seed, u64 *blkmap)
{
	struct fmodel f;
	u64 nb = (size + 4095) / 4096;

	f.size = size;
	f.data = rand_bytes(size, seed);
	f.fi = ksim_file_new(fs, size, f.data, blkmap, nb);
	free(blkmap);
	return f;
}

/* chunk content as the page cache shows it, zero padded past EOF */
static void chunk_bytes(const struct fmodel *f, u64 fpos, u32 cs, u8 *out)
{
	u64 n = fpos < f->size ? (f->size - fpos < cs ? f->size - fpos : cs) : 0;

	memset(out, 0, cs);
	memcpy(out, f->data + fpos, n);
}

static u64 fpos_of(u32 id, u32 cs, u32 relseg)
{
	return (u64)(relseg ? id % relseg : id) * cs;
}

/* the majority rule, independently: clean page 1, dirty page threshold+1 */
static int chunk_cached(const struct fmodel *f, u64 fpos, u32 cs)
{
	u32 np = cs / 4096, thr = np / 2, score = 0, i;

	for (i = 0; i < np; i++) {
		u64 pg = fpos / 4096 + i;
		int st;

		if (pg * 4096 >= f->size)
			continue;
		st = ksim_pc_get(f->fi, pg);
		score += st == 2 ? thr + 1 : st == 1 ? 1 : 0;
	}
	return score > thr;
}

static int counters_clean(const char *when)
{
	struct ksim_counters c;

	ksim_counters(&c);
#define Z(f)                                                                            \
	if (c.f) {                                                                      \
		fprintf(stderr, "[%s] %s: counter %s = %lld\n", g_scn, when, #f, (long long)c.f); \
		g_failures++;                                                           \
		return 1;                                                               \
	}
	Z(violations) Z(kmallocs_live) Z(pages_live) Z(iommu_pages_live) Z(requests_live)
	Z(files_live) Z(module_refs) Z(dmabufs_live) Z(folio_refs) Z(fds_leaked)
	Z(dev_refs_leaked) Z(iommu_pages_leaked)
#undef Z
	return 0;
}

/* ------------------------------------------------------------ the machine */
struct world {
	int ctrl, ns, fs, dev;
};

static void up(struct world *w, int lba_shift, u32 max_hw_sectors)
{
	ksim_init();
	w->ctrl = ksim_ctrl_new("0000:41:00.0", 0);
	w->ns = ksim_ns_new(w->ctrl, 1, lba_shift, 64ull << 11, max_hw_sectors, 0);
	w->fs = ksim_fs_new(w->ns, 2048, "ext4", 12);
	if (ksim_module_load())
		abort();
	w->dev = ksim_dev_open(0);
}

static int down(struct world *w)
{
	if (w->dev >= 0)
		ksim_close(w->dev);
	ksim_quiesce();
	ksim_module_unload();
	ksim_fini();
	return counters_clean("after teardown");
}

static unsigned long map_dmabuf(int dev, int dbfd, u64 off, u64 len)
{
	struct strom_map_gpu_dmabuf m = { 0 };

	m.dmabuf_fd = dbfd;
	m.vaddress = 0x7e0000000000ull + off;
	m.length = len;
	m.dmabuf_offset = off;
	if (ksim_ioctl(dev, STROM_IOCTL__MAP_GPU_DMABUF, &m))
		return 0;
	return m.handle;
}

static long unmap(int dev, unsigned long h)
{
	struct strom_unmap_gpu_memory u = { h };

	return ksim_ioctl(dev, STROM_IOCTL__UNMAP_GPU_MEMORY, &u);
}

static long wait_task(int dev, unsigned long id, long *status)
{
	struct strom_memcpy_wait w = { id, 0 };
	long rc = ksim_ioctl(dev, STROM_IOCTL__MEMCPY_WAIT, &w);

	*status = w.status;
	return rc;
}

/* SSD2GPU + WAIT, then every slot checked against the model (`hbm` is the
 * host view of the mapping's byte 0, `off` the destination inside it):
 * storage chunks packed at the head in request order, page-cache chunks
 * from the tail (wb_buffer, or HBM when wb == NULL) */
static int ssd2gpu_check(int dev, unsigned long h, u8 *hbm, u64 off, int fd,
			 const struct fmodel *f, const u32 *ids, u32 n, u32 cs, u32 relseg, u8 *wb)
{
	struct strom_memcpy_ssd2gpu a = { 0 };
	u32 *io = malloc(n * sizeof(u32)), *want = malloc(n * sizeof(u32));
	u8 *exp = malloc(cs);
	u32 i, nram = 0, nssd = 0;
	long st;

	for (i = 0; i < n; i++) {
		io[i] = ids[i];
		if (chunk_cached(f, fpos_of(ids[i], cs, relseg), cs))
			want[n - 1 - nram++] = ids[i];
		else
			want[nssd++] = ids[i];
	}
	a.handle = h;
	a.offset = off;
	a.file_desc = fd;
	a.nr_chunks = n;
	a.chunk_sz = cs;
	a.relseg_sz = relseg;
	a.chunk_ids = io;
	a.wb_buffer = (char *)wb;
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), 0);
	CHECK(a.dma_task_id != 0);
	CHECK_EQ(wait_task(dev, a.dma_task_id, &st), 0);
	CHECK_EQ(st, 0);
	CHECK_EQ(a.nr_ram2gpu, nram);
	CHECK_EQ(a.nr_ssd2gpu, nssd);
	CHECK(a.nr_dma_submit >= 1 || nssd == 0);
	for (i = 0; i < n; i++) {
		u64 fpos = fpos_of(io[i], cs, relseg);
		u64 valid = f->size - fpos < cs ? ((f->size - fpos + 4095) & ~4095ull) : cs;
		const u8 *got;

		CHECK_EQ(io[i], want[i]);
		chunk_bytes(f, fpos, cs, exp);
		if (i < nssd || !wb)
			got = hbm + off + (u64)i * cs;
		else
			got = wb + (u64)i * cs, valid = cs;
		if (memcmp(got, exp, valid)) {
			fprintf(stderr, "[%s] slot %u (chunk %u, %s) differs\n", g_scn, i, io[i],
				i < nssd ? "ssd" : "ram");
			g_failures++;
			return 1;
		}
	}
	free(io);
	free(want);
	free(exp);
	return 0;
}

/* ------------------------------------------------------------ scenarios */
static int scn_ssd2gpu_landing(void)
{
	struct world w;
	const u32 cs = 64 << 10, nch = 48;
	u8 *wb = malloc((u64)nch * cs);
	u32 ids[48], i, s = 7;
	unsigned long h;
	struct fmodel f;
	int fd, db;
	u8 *hbm;

	up(&w, 9, 256);
	f = new_file(w.fs, 8ull << 20, 11, frag_map(2048, 100, 5, 40));
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(16ull << 20, 7, 3);
	hbm = ksim_dmabuf_mem(db);
	h = map_dmabuf(w.dev, db, 1ull << 20, 8ull << 20);
	CHECK(h);
	/* page cache: chunk 3 fully clean, chunk 5 one clean page of 16 (loses),
	 * chunk 9 one dirty page (wins), chunk 20 half + 1 clean (wins) */
	for (i = 0; i < 16; i++)
		ksim_pc_set(f.fi, 3 * 16 + i, 1);
	ksim_pc_set(f.fi, 5 * 16 + 4, 1);
	{
		u8 nb[100];

		memset(nb, 0x5a, sizeof(nb));
		ksim_file_write(f.fi, 9 * (u64)cs + 4096 * 3 + 17, nb, sizeof(nb));
		memcpy(f.data + 9 * (u64)cs + 4096 * 3 + 17, nb, sizeof(nb));
	}
	for (i = 0; i < 9; i++)
		ksim_pc_set(f.fi, 20 * 16 + i, 1);
	for (i = 0; i < nch; i++)
		ids[i] = (i * 37 + 5) % 128;              /* a permutation slice */
	ids[0] = 3, ids[1] = 9, ids[2] = 5, ids[3] = 20;
	/* with a wb_buffer (the reference's mode) */
	/* the mapping starts 1 MiB into the dma-buf; the copy 1 MiB into it */
	if (ssd2gpu_check(w.dev, h, hbm + (1 << 20), 1ull << 20, fd, &f, ids, nch, cs, 0, wb))
		return 1;
	/* dirty data stayed dirty: it went through the page cache */
	CHECK_EQ(ksim_pc_get(f.fi, 9 * 16 + 3), 2);
	/* wb_buffer == NULL: cached chunks DMA'd to the tail after write-back */
	for (i = 0; i < nch; i++)
		ids[i] = (rnd(&s) % 128);
	ids[0] = 3, ids[1] = 9;
	if (ssd2gpu_check(w.dev, h, hbm + (1 << 20), 1ull << 20, fd, &f, ids, nch, cs, 0, NULL))
		return 1;
	CHECK_EQ(ksim_pc_get(f.fi, 9 * 16 + 3), 1);   /* written back */
	/* HBM outside the mapped range untouched */
	for (i = 0; i < (1u << 20); i += 4096)
		CHECK_EQ(hbm[i], 0x41);
	CHECK_EQ(unmap(w.dev, h), 0);
	ksim_close(fd);
	ksim_close(db);
	free(wb);
	free(f.data);
	return down(&w);
}

static int scn_relseg_eof(void)
{
	struct world w;
	const u32 cs = 16 << 10;
	u32 ids[3] = { 17, 33, 2 };
	struct strom_memcpy_ssd2gpu a = { 0 };
	unsigned long h;
	struct fmodel f;
	int fd, db;
	u8 *hbm;

	up(&w, 12, 512);
	/* 16 chunks + a 5000-byte tail: chunk 16 straddles EOF */
	f = new_file(w.fs, 16 * cs + 5000, 21, linear_map((16 * cs + 5000 + 4095) / 4096, 64));
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(4ull << 20, 3, 9);
	hbm = ksim_dmabuf_mem(db);
	h = map_dmabuf(w.dev, db, 0, 4ull << 20);
	/* relseg: chunk ids wrap every 16 chunks (PG segment files) */
	if (ssd2gpu_check(w.dev, h, hbm, 0, fd, &f, ids, 3, cs, 16, NULL))
		return 1;
	/* straddling chunk: pages up to EOF transferred, the rest untouched */
	ids[0] = 16;
	if (ssd2gpu_check(w.dev, h, hbm, 1 << 20, fd, &f, ids, 1, cs, 0, NULL))
		return 1;
	CHECK_EQ(hbm[(1 << 20) + 8192 + 1], 0x41);
	/* a chunk starting at EOF: -ERANGE, nothing in flight afterwards */
	ids[0] = 17;
	a.handle = h;
	a.file_desc = fd;
	a.nr_chunks = 1;
	a.chunk_sz = cs;
	a.chunk_ids = ids;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), -ERANGE);
	/* bad chunk sizes, an unaligned destination, a range past the mapping */
	a.chunk_sz = 6000;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), -EINVAL);
	a.chunk_sz = cs;
	a.offset = 512;
	ids[0] = 1;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), -EINVAL);
	a.offset = (4ull << 20) - 4096;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), -ERANGE);
	a.offset = UINT64_MAX - 4095;                  /* wraps: overflow-safe check */
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), -ERANGE);
	/* not readable / unknown fd */
	a.offset = 0;
	{
		int wfd = ksim_file_open(f.fi, 0);

		a.file_desc = wfd;
		CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), -EBADF);
		ksim_close(wfd);
		a.file_desc = 999;
		CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), -EBADF);
	}
	CHECK_EQ(unmap(w.dev, h), 0);
	CHECK_EQ(unmap(w.dev, h), -ENOENT);
	ksim_close(fd);
	ksim_close(db);
	free(f.data);
	return down(&w);
}

static int scn_ssd2ram(void)
{
	struct world w;
	const u32 cs = 64 << 10, n = 100;
	struct strom_alloc_dma_buffer ab = { 12ull << 20, -1, -1 };
	struct strom_memcpy_ssd2ram r = { 0 };
	struct ksim_counters c0, c1;
	u32 ids[100], i;
	unsigned long ua;
	struct fmodel f;
	u8 *got, *exp;
	const char *nm;
	long st;
	int fd;

	up(&w, 9, 256);
	f = new_file(w.fs, 8ull << 20, 31, frag_map(2048, 4000, 9, 64));
	fd = ksim_file_open(f.fi, 1);
	/* the node is validated before anything is allocated */
	ab.node_id = 7;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__ALLOC_DMA_BUFFER, &ab), -EINVAL);
	ab.node_id = -1;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__ALLOC_DMA_BUFFER, &ab), 0);
	nm = ksim_fd_name(ab.dmabuf_fdesc);
	CHECK(nm && !strcmp(nm, "anon_inode:dmabuf0:12582912"));
	CHECK(ksim_mmap(ab.dmabuf_fdesc, 12ull << 20, 0, 0) == 0);   /* private: refused */
	ua = ksim_mmap(ab.dmabuf_fdesc, 12ull << 20, 0, 1);
	CHECK(ua);
	ksim_close(ab.dmabuf_fdesc);            /* the mapping keeps the buffer */
	for (i = 0; i < 8; i++)
		ksim_pc_set(f.fi, 40 * 16 + i * 2, 1);     /* chunk 40: 8 of 16 (loses) */
	for (i = 0; i < 16; i++)
		ksim_pc_set(f.fi, 60 * 16 + i, 1);         /* chunk 60 cached */
	for (i = 0; i < n; i++)
		ids[i] = (i * 7 + 40) % 128;
	ksim_counters(&c0);
	for (int rep = 0; rep < 2; rep++) {
		r.dest_uaddr = (void *)(ua + (u64)rep * 4096 * 3);
		r.file_desc = fd;
		r.nr_chunks = n;
		r.chunk_sz = cs;
		r.chunk_ids = ids;
		CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2RAM, &r), 0);
		CHECK_EQ(wait_task(w.dev, r.dma_task_id, &st), 0);
		CHECK_EQ(st, 0);
		CHECK_EQ(r.nr_ram2ram + r.nr_ssd2ram, n);
		got = malloc((u64)n * cs);
		exp = malloc(cs);
		CHECK_EQ(ksim_user_read((unsigned long)r.dest_uaddr, got, (u64)n * cs), 0);
		for (i = 0; i < n; i++) {               /* identity landing */
			chunk_bytes(&f, (u64)ids[i] * cs, cs, exp);
			CHECK(!memcmp(got + (u64)i * cs, exp, cs));
		}
		free(got);
		free(exp);
	}
	/* the 3 segments were mapped once for the controller, not per page */
	ksim_counters(&c1);
	CHECK(c1.dma_map_calls - c0.dma_map_calls <= 3);
	/* a destination not inside a DMA buffer */
	r.dest_uaddr = (void *)(ua - (1ul << 20));
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2RAM, &r), -EINVAL);
	/* a range running past the buffer */
	r.dest_uaddr = (void *)(ua + (12ull << 20) - (u64)cs * 10);
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2RAM, &r), -EINVAL);
	/* node 1 exists */
	ab.node_id = 1;
	ab.length = 1;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__ALLOC_DMA_BUFFER, &ab), 0);
	ksim_close(ab.dmabuf_fdesc);
	CHECK_EQ(ksim_munmap(ua), 0);
	ksim_close(fd);
	free(f.data);
	return down(&w);
}

static int scn_errors_and_reclaim(void)
{
	struct world w;
	const u32 cs = 32 << 10;
	struct strom_memcpy_ssd2gpu a = { 0 };
	struct strom_memcpy_wait_timed wt = { 0 };
	struct ksim_counters c0, c1;
	u32 ids[64], i;
	unsigned long h;
	struct fmodel f;
	int fd, db, dev2;
	long st;

	up(&w, 9, 64);                        /* 32 KiB max transfer: many commands */
	f = new_file(w.fs, 4ull << 20, 41, linear_map(1024, 9000));
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(4ull << 20, 2, 1);
	h = map_dmabuf(w.dev, db, 0, 4ull << 20);
	for (i = 0; i < 64; i++)
		ids[i] = i;
	/* the 5th command fails with an I/O error: WAIT says -EIO + status */
	ksim_fail_cmd(5, 10);
	a.handle = h;
	a.file_desc = fd;
	a.nr_chunks = 64;
	a.chunk_sz = cs;
	a.chunk_ids = ids;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), 0);
	CHECK_EQ(wait_task(w.dev, a.dma_task_id, &st), -EIO);
	CHECK_EQ(st, -EIO);
	/* consumed: a second WAIT finds a finished task */
	CHECK_EQ(wait_task(w.dev, a.dma_task_id, &st), 0);
	/* medium error -> -ENODATA status */
	ksim_fail_cmd(2, 7);
	for (i = 0; i < 64; i++)
		ids[i] = i;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), 0);
	CHECK_EQ(wait_task(w.dev, a.dma_task_id, &st), -EIO);
	CHECK_EQ(st, -ENODATA);
	ksim_fail_cmd(0, 0);
	/* never issued -> -ENOENT (the reference returned success, defect #9) */
	CHECK_EQ(wait_task(w.dev, 1ul << 40, &st), -ENOENT);
	/* timed WAIT on a held controller -> -ETIME, then completes */
	ksim_ctrl_config(w.ctrl, 0, 0, 1);
	for (i = 0; i < 64; i++)
		ids[i] = i;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), 0);
	wt.dma_task_id = a.dma_task_id;
	wt.timeout_ns = 2000000;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_WAIT_TIMED, &wt), -ETIME);
	/* a signal interrupts a waiter */
	ksim_set_signal(1);
	CHECK_EQ(wait_task(w.dev, a.dma_task_id, &st), -EINTR);
	ksim_set_signal(0);
	ksim_ctrl_config(w.ctrl, 0, 0, 0);
	CHECK_EQ(wait_task(w.dev, a.dma_task_id, &st), 0);
	/* release reclaim: a second session's failed task nobody waits for */
	dev2 = ksim_dev_open(0);
	ksim_fail_cmd(1, 10);
	for (i = 0; i < 64; i++)
		ids[i] = i;
	CHECK_EQ(ksim_ioctl(dev2, STROM_IOCTL__MEMCPY_SSD2GPU, &a), 0);
	ksim_quiesce();
	ksim_counters(&c0);
	ksim_close(dev2);
	ksim_quiesce();
	ksim_counters(&c1);
	CHECK(c1.printk > c0.printk);            /* "failed task(s) reclaimed on close" */
	/* close with requests still in flight: release waits for the last one */
	ksim_fail_cmd(0, 0);
	dev2 = ksim_dev_open(0);
	ksim_ctrl_config(w.ctrl, 1, 0, 1);
	for (i = 0; i < 64; i++)
		ids[i] = i;
	CHECK_EQ(ksim_ioctl(dev2, STROM_IOCTL__MEMCPY_SSD2GPU, &a), 0);
	ksim_close(dev2);
	usleep(2000);
	ksim_ctrl_config(w.ctrl, 1, 0, 0);
	ksim_quiesce();
	/* EFAULT on an unreadable chunk_ids array and on the argument itself */
	ksim_poison_user(ids, sizeof(ids));
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), -EFAULT);
	ksim_poison_user(NULL, 0);
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, (void *)16), -EFAULT);
	CHECK_EQ(unmap(w.dev, h), 0);
	ksim_close(fd);
	ksim_close(db);
	free(f.data);
	return down(&w);
}

struct unmap_arg { int dev; unsigned long h; volatile int done; long rc; };

static void *unmap_thread(void *p)
{
	struct unmap_arg *u = p;

	u->rc = unmap(u->dev, u->h);
	__atomic_store_n(&u->done, 1, __ATOMIC_SEQ_CST);
	return NULL;
}

static int scn_unmap_inflight(void)
{
	struct world w;
	const u32 cs = 128 << 10;
	struct strom_memcpy_ssd2gpu a = { 0 };
	struct unmap_arg u = { 0 };
	int pinned, attached, mapped, refs;
	u32 ids[16], i;
	pthread_t th;
	struct fmodel f;
	int fd, db;
	long st;

	up(&w, 9, 256);
	f = new_file(w.fs, 2ull << 20, 51, frag_map(512, 300, 3, 16));
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(2ull << 20, 4, 5);
	u.dev = w.dev;
	u.h = map_dmabuf(w.dev, db, 0, 2ull << 20);
	for (i = 0; i < 16; i++)
		ids[i] = i;
	ksim_ctrl_config(w.ctrl, 1, 0, 1);        /* hold every completion */
	a.handle = u.h;
	a.file_desc = fd;
	a.nr_chunks = 16;
	a.chunk_sz = cs;
	a.chunk_ids = ids;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), 0);
	CHECK(ksim_ctrl_queued(w.ctrl) > 0);
	pthread_create(&th, NULL, unmap_thread, &u);
	usleep(20000);
	CHECK_EQ(__atomic_load_n(&u.done, __ATOMIC_SEQ_CST), 0);   /* drains first */
	ksim_dmabuf_state(db, &pinned, &attached, &mapped, &refs);
	CHECK_EQ(pinned, 1);
	ksim_ctrl_config(w.ctrl, 1, 100, 0);
	pthread_join(th, NULL);
	CHECK_EQ(u.rc, 0);
	CHECK_EQ(wait_task(w.dev, a.dma_task_id, &st), 0);
	CHECK_EQ(st, 0);
	ksim_quiesce();
	usleep(5000);
	ksim_quiesce();
	/* the teardown work unpinned, unmapped, detached, dropped the dma-buf */
	for (i = 0; i < 200; i++) {
		ksim_dmabuf_state(db, &pinned, &attached, &mapped, &refs);
		if (refs == 1)
			break;
		usleep(1000);
	}
	CHECK_EQ(pinned, 0);
	CHECK_EQ(attached, 0);
	CHECK_EQ(mapped, 0);
	CHECK_EQ(refs, 1);
	/* the data landed before the unmap completed */
	{
		u8 *exp = malloc(cs), *hbm = ksim_dmabuf_mem(db);

		for (i = 0; i < 16; i++) {
			chunk_bytes(&f, (u64)ids[i] * cs, cs, exp);
			CHECK(!memcmp(hbm + (u64)i * cs, exp, cs));
		}
		free(exp);
	}
	/* P2P refused by the exporter: SSD2GPU fails cleanly */
	ksim_dmabuf_deny_p2p(db, 1);
	u.h = map_dmabuf(w.dev, db, 0, 1ull << 20);
	a.handle = u.h;
	a.nr_chunks = 4;
	for (i = 0; i < 4; i++)
		ids[i] = i;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a), -EOPNOTSUPP);
	CHECK_EQ(unmap(w.dev, u.h), 0);
	ksim_close(fd);
	ksim_close(db);
	free(f.data);
	return down(&w);
}

/* raid0 over three namespaces on three controllers, via SET_ROUTE */
static int scn_raid0_route(void)
{
	const u32 chunk_sects = 128;            /* 64 KiB stripe chunk */
	struct strom_set_route *r = calloc(1, sizeof(*r));
	int ctrl[3], ns[3], md, fs, dev, fd, db, i;
	u64 ios[4], sect[4], tot_ios = 0, tot_sect = 0;
	int64_t infl;
	unsigned long h;
	struct fmodel f;
	u32 ids[96];
	u8 *hbm;

	ksim_init();
	for (i = 0; i < 3; i++) {
		char pci[16];

		snprintf(pci, sizeof(pci), "0000:%02x:00.0", 0x41 + i);
		ctrl[i] = ksim_ctrl_new(pci, 0);
		ns[i] = ksim_ns_new(ctrl[i], 1, 9, 32ull << 11, 256, 0);
		ksim_ctrl_config(ctrl[i], 1, 0, 0);
	}
	md = ksim_md_new(ns, 3, chunk_sects, NULL);
	fs = ksim_fs_new(md, 0, "xfs", 12);
	f = new_file(fs, 12ull << 20, 61, linear_map(3072, 256));
	CHECK_EQ(ksim_module_load(), 0);
	dev = ksim_dev_open(0);
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(16ull << 20, 5, 2);
	hbm = ksim_dmabuf_mem(db);
	h = map_dmabuf(dev, db, 0, 16ull << 20);
	/* bio-based md without a route: not served */
	{
		struct strom_check_file cf = { fd, 0, 0 };

		CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__CHECK_FILE, &cf), -EOPNOTSUPP);
	}
	r->volume_major = ksim_disk_devt(md) >> 20;
	r->volume_minor = ksim_disk_devt(md) & 0xfffff;
	r->nmembers = 3;
	r->chunk_sects = chunk_sects;
	r->nzones = 1;
	r->zone_end[0] = (32ull << 11) / chunk_sects * chunk_sects * 3;
	r->zone_nb_dev[0] = 3;
	for (i = 0; i < 3; i++) {
		r->zone_devs[0][i] = (unsigned char)i;
		r->member_major[i] = ksim_disk_devt(ns[i]) >> 20;
		r->member_minor[i] = ksim_disk_devt(ns[i]) & 0xfffff;
	}
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__SET_ROUTE, r), -EPERM);
	ksim_set_admin(1);
	r->zone_end[0] += chunk_sects * 3;       /* larger than the members: refused */
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__SET_ROUTE, r), -EINVAL);
	r->zone_end[0] -= chunk_sects * 3;
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__SET_ROUTE, r), 0);
	ksim_set_admin(0);
	{
		struct strom_check_file cf = { fd, 0, 0 };

		CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__CHECK_FILE, &cf), 0);
		CHECK_EQ(cf.numa_node_id, 0);
		CHECK_EQ(cf.support_dma64, 1);
	}
	/* 128 KiB chunks over 64 KiB stripes: every chunk spans two members */
	for (i = 0; i < 96; i++)
		ids[i] = (u32)((i * 13) % 96);
	if (ssd2gpu_check(dev, h, hbm, 0, fd, &f, ids, 96, 128 << 10, 0, NULL))
		return 1;
	ksim_quiesce();
	/* every member did I/O; the md volume accounts all of it (iostat md0) */
	for (i = 0; i < 3; i++) {
		ksim_disk_stats(ns[i], &ios[i], &sect[i], &infl);
		CHECK(ios[i] > 0);
		CHECK_EQ(infl, 0);
		tot_ios += ios[i];
		tot_sect += sect[i];
	}
	ksim_disk_stats(md, &ios[3], &sect[3], &infl);
	CHECK_EQ(ios[3], tot_ios);
	CHECK_EQ(sect[3], tot_sect);
	CHECK_EQ(tot_sect, 96 * 256);
	CHECK_EQ(infl, 0);
	/* drop the route: no longer served */
	ksim_set_admin(1);
	r->nmembers = 0;
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__SET_ROUTE, r), 0);
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__SET_ROUTE, r), -ENOENT);
	ksim_set_admin(0);
	CHECK_EQ(unmap(dev, h), 0);
	ksim_close(fd);
	ksim_close(db);
	ksim_close(dev);
	ksim_quiesce();
	ksim_module_unload();
	ksim_fini();
	free(r);
	free(f.data);
	return counters_clean("after teardown");
}

/* SSD2RAM from a 12-controller raid0 route into one DMA buffer whose DMA
 * layer cannot map a 4 MiB segment at once (swiotlb-like 256 KiB cap): the
 * buffer keeps a map per controller (more than STROM_MAX_ATTACH), each page
 * by page, and every chunk lands intact.  Also: mmap of the buffer must lie
 * inside it (reference pmemmap.c:593). */
static int scn_ssd2ram_wide_route(void)
{
	enum { NM = 12 };
	const u32 chunk_sects = 128, cs = 128 << 10, n = 96;
	struct strom_set_route *r = calloc(1, sizeof(*r));
	struct strom_alloc_dma_buffer ab = { 12ull << 20, -1, -1 };
	struct strom_memcpy_ssd2ram q = { 0 };
	struct ksim_counters c0, c1;
	int ctrl[NM], ns[NM], md, fs, dev, fd, i;
	unsigned long ua;
	struct fmodel f;
	u32 ids[96];
	u8 *got, *exp;
	long st;

	ksim_init();
	for (i = 0; i < NM; i++) {
		char pci[16];

		snprintf(pci, sizeof(pci), "0000:%02x:00.0", 0x41 + i);
		ctrl[i] = ksim_ctrl_new(pci, 0);
		ns[i] = ksim_ns_new(ctrl[i], 1, 9, 32ull << 11, 256, 0);
		ksim_ctrl_config(ctrl[i], 1, 0, 0);
	}
	md = ksim_md_new(ns, NM, chunk_sects, NULL);
	fs = ksim_fs_new(md, 0, "xfs", 12);
	f = new_file(fs, 12ull << 20, 67, linear_map(3072, 256));
	CHECK_EQ(ksim_module_load(), 0);
	dev = ksim_dev_open(0);
	fd = ksim_file_open(f.fi, 1);
	r->volume_major = ksim_disk_devt(md) >> 20;
	r->volume_minor = ksim_disk_devt(md) & 0xfffff;
	r->nmembers = NM;
	r->chunk_sects = chunk_sects;
	r->nzones = 1;
	r->zone_end[0] = (32ull << 11) / chunk_sects * chunk_sects * NM;
	r->zone_nb_dev[0] = NM;
	for (i = 0; i < NM; i++) {
		r->zone_devs[0][i] = (unsigned char)i;
		r->member_major[i] = ksim_disk_devt(ns[i]) >> 20;
		r->member_minor[i] = ksim_disk_devt(ns[i]) & 0xfffff;
	}
	ksim_set_admin(1);
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__SET_ROUTE, r), 0);
	ksim_set_admin(0);
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__ALLOC_DMA_BUFFER, &ab), 0);
	/* mappings must lie inside the 12 MiB buffer */
	CHECK(ksim_mmap(ab.dmabuf_fdesc, 13ull << 20, 0, 1) == 0);
	CHECK_EQ(ksim_last_mmap_rc(), -EINVAL);
	CHECK(ksim_mmap(ab.dmabuf_fdesc, 2ull << 20, 11ull << 20, 1) == 0);
	CHECK_EQ(ksim_last_mmap_rc(), -EINVAL);
	CHECK(ksim_mmap(ab.dmabuf_fdesc, 4096, 12ull << 20, 1) == 0);
	CHECK_EQ(ksim_last_mmap_rc(), -EINVAL);
	ua = ksim_mmap(ab.dmabuf_fdesc, 12ull << 20, 0, 1);
	CHECK(ua);
	ksim_close(ab.dmabuf_fdesc);
	ksim_dma_max_mapping(256 << 10);
	for (i = 0; i < (int)n; i++)
		ids[i] = (u32)((i * 37 + 5) % 96);
	ksim_counters(&c0);
	q.dest_uaddr = (void *)ua;
	q.file_desc = fd;
	q.nr_chunks = n;
	q.chunk_sz = cs;
	q.chunk_ids = ids;
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__MEMCPY_SSD2RAM, &q), 0);
	CHECK_EQ(wait_task(dev, q.dma_task_id, &st), 0);
	CHECK_EQ(st, 0);
	CHECK_EQ(q.nr_ssd2ram, n);
	got = malloc((u64)n * cs);
	exp = malloc(cs);
	CHECK_EQ(ksim_user_read(ua, got, (u64)n * cs), 0);
	for (i = 0; i < (int)n; i++) {
		chunk_bytes(&f, (u64)ids[i] * cs, cs, exp);
		CHECK(!memcmp(got + (u64)i * cs, exp, cs));
	}
	/* one refused segment map, then page by page, once per controller */
	ksim_counters(&c1);
	CHECK(c1.dma_map_calls - c0.dma_map_calls <= NM * (1 + 3 * 1024));
	CHECK(c1.dma_map_calls - c0.dma_map_calls >= NM * 3 * 1024);
	/* a second copy reuses the maps */
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__MEMCPY_SSD2RAM, &q), 0);
	CHECK_EQ(wait_task(dev, q.dma_task_id, &st), 0);
	CHECK_EQ(st, 0);
	ksim_counters(&c0);
	CHECK_EQ(c0.dma_map_calls - c1.dma_map_calls, 0);
	ksim_dma_max_mapping(0);
	free(got);
	free(exp);
	CHECK_EQ(ksim_munmap(ua), 0);
	ksim_close(fd);
	ksim_close(dev);
	ksim_quiesce();
	ksim_module_unload();
	ksim_fini();
	free(r);
	free(f.data);
	return counters_clean("after teardown");
}

/* NVMe multipath: the head is bio-based; its hidden path disk is named */
static int scn_multipath_alias(void)
{
	struct strom_set_route *r = calloc(1, sizeof(*r));
	int ctrl, path, head, fs, dev, fd, db, other, octrl;
	unsigned long h;
	struct fmodel f;
	u32 ids[32], i;

	ksim_init();
	ctrl = ksim_ctrl_new("0000:81:00.0", 1);
	path = ksim_ns_new(ctrl, 3, 12, 16ull << 11, 256, 1);
	head = ksim_head_new(path);
	octrl = ksim_ctrl_new("0000:82:00.0", 1);
	other = ksim_ns_new(octrl, 4, 12, 16ull << 11, 256, 1);
	fs = ksim_fs_new(head, 0, "ext4", 12);
	f = new_file(fs, 4ull << 20, 71, frag_map(1024, 32, 11, 30));
	CHECK_EQ(ksim_module_load(), 0);
	dev = ksim_dev_open(1);                   /* through /proc/nvme-strom */
	{
		char sig[256] = { 0 };

		CHECK(ksim_read(dev, sig, sizeof(sig) - 1) > 0);
		CHECK(!strncmp(sig, "version: ", 9));
	}
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(4ull << 20, 3, 8);
	h = map_dmabuf(dev, db, 0, 4ull << 20);
	r->volume_major = ksim_disk_devt(head) >> 20;
	r->volume_minor = ksim_disk_devt(head) & 0xfffff;
	r->nmembers = 1;
	ksim_set_admin(1);
	/* a path of another namespace (nsid 4 != 3): refused */
	snprintf(r->member_name[0], sizeof(r->member_name[0]), "0000:82:00.0/nvme1/%s",
		 ksim_disk_name(other));
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__SET_ROUTE, r), -EINVAL);
	snprintf(r->member_name[0], sizeof(r->member_name[0]), "0000:81:00.0/nvme0/%s",
		 ksim_disk_name(path));
	CHECK_EQ(ksim_ioctl(dev, STROM_IOCTL__SET_ROUTE, r), 0);
	ksim_set_admin(0);
	for (i = 0; i < 32; i++)
		ids[i] = 31 - i;
	if (ssd2gpu_check(dev, h, ksim_dmabuf_mem(db), 0, fd, &f, ids, 32, 128 << 10, 0, NULL))
		return 1;
	CHECK_EQ(unmap(dev, h), 0);
	ksim_close(fd);
	ksim_close(db);
	ksim_close(dev);
	ksim_quiesce();
	ksim_module_unload();
	ksim_fini();
	free(r);
	free(f.data);
	return counters_clean("after teardown");
}

/* an unregistered (plain namespace) volume is a cache: a disk replaced
 * under the same dev_t must not be served through the stale entry */
static int scn_stale_volume_cache(void)
{
	struct world w;
	struct fmodel f, g;
	unsigned long h;
	int fd, db, ns2, fs2, fd2;
	u32 ids[8], i;

	up(&w, 9, 256);
	f = new_file(w.fs, 1ull << 20, 81, linear_map(256, 10));
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(1ull << 20, 2, 4);
	h = map_dmabuf(w.dev, db, 0, 1ull << 20);
	for (i = 0; i < 8; i++)
		ids[i] = i;
	if (ssd2gpu_check(w.dev, h, ksim_dmabuf_mem(db), 0, fd, &f, ids, 8, 128 << 10, 0, NULL))
		return 1;
	/* hot removal + a new namespace instance on the same dev_t */
	ns2 = ksim_disk_remove(w.ns, 1);
	fs2 = ksim_fs_new(ns2, 2048, "ext4", 12);
	g = new_file(fs2, 1ull << 20, 82, linear_map(256, 5000));
	fd2 = ksim_file_open(g.fi, 1);
	if (ssd2gpu_check(w.dev, h, ksim_dmabuf_mem(db), 0, fd2, &g, ids, 8, 128 << 10, 0, NULL))
		return 1;
	CHECK_EQ(unmap(w.dev, h), 0);
	ksim_close(fd);
	ksim_close(fd2);
	ksim_close(db);
	free(f.data);
	free(g.data);
	return down(&w);
}

static int scn_registry_and_stats(void)
{
	struct world w;
	struct strom_stat_info si = { 0 };
	struct strom_list_gpu_memory *l = calloc(1, sizeof(*l) + 8 * sizeof(unsigned long));
	struct strom_info_gpu_memory *in = calloc(1, sizeof(*in) + 64 * sizeof(u64));
	unsigned long h1, h2;
	struct fmodel f;
	u32 ids[4] = { 0, 1, 2, 3 };
	int fd, db;

	up(&w, 9, 256);
	f = new_file(w.fs, 1ull << 20, 91, linear_map(256, 700));
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(4ull << 20, 4, 6);
	h1 = map_dmabuf(w.dev, db, 0, 2ull << 20);
	h2 = map_dmabuf(w.dev, db, 2ull << 20, 2ull << 20);
	CHECK(h1 && h2 && h1 != h2);
	l->nrooms = 8;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__LIST_GPU_MEMORY, l), 0);
	CHECK_EQ(l->nitems, 2);
	/* another user sees none of them and cannot unmap them */
	ksim_set_euid(1001);
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__LIST_GPU_MEMORY, l), 0);
	CHECK_EQ(l->nitems, 0);
	in->handle = h1;
	in->nrooms = 64;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__INFO_GPU_MEMORY, in), -ENOENT);
	CHECK_EQ(unmap(w.dev, h1), -ENOENT);
	ksim_set_euid(1000);
	if (ssd2gpu_check(w.dev, h2, ksim_dmabuf_mem(db) + (2 << 20), 0, fd, &f, ids, 4, 64 << 10, 0,
			  NULL))
		return 1;
	/* INFO: one entry per 64 KiB, bus addresses once attached */
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__INFO_GPU_MEMORY, in), 0);
	CHECK_EQ(in->map_length, 2ull << 20);
	CHECK_EQ(in->owner, 1000);
	CHECK_EQ(in->nitems, 32);
	CHECK(in->paddrs[0] == 0);                 /* h1 never attached */
	in->handle = h2;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__INFO_GPU_MEMORY, in), 0);
	CHECK(in->paddrs[0] != 0 && in->paddrs[31] != 0);
	/* STAT_INFO v1 */
	si.version = 2;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__STAT_INFO, &si), -EINVAL);
	si.version = 1;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__STAT_INFO, &si), 0);
	CHECK(si.nr_ssd2gpu >= 1 && si.nr_setup_prps >= si.nr_submit_dma && si.nr_wait_dtask >= 1);
	CHECK_EQ(si.cur_dma_count, 0);
	CHECK(si.max_dma_count >= 1);
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__STAT_INFO, &si), 0);
	CHECK_EQ(si.max_dma_count, 0);             /* read-and-reset */
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MAP_GPU_MEMORY, &si), -EOPNOTSUPP);
	CHECK_EQ(ksim_ioctl(w.dev, 0x1234, &si), -EINVAL);
	CHECK_EQ(unmap(w.dev, h1), 0);
	CHECK_EQ(unmap(w.dev, h2), 0);
	ksim_close(fd);
	ksim_close(db);
	free(l);
	free(in);
	free(f.data);
	return down(&w);
}

/* several sessions hammering one mapping, completions reordered, errors
 * injected, a lister running alongside (the TSAN build's main course) */
struct stress_arg {
	int dev, fd, tid;
	unsigned long h;
	const struct fmodel *f;
	u8 *hbm;
	int errors, ok, bad;
};

static void *stress_thread(void *p)
{
	struct stress_arg *s = p;
	u32 seed = 1000 + s->tid, ids[16], i, it;
	const u32 cs = 32 << 10;
	u8 *exp = malloc(cs);

	for (it = 0; it < 60; it++) {
		struct strom_memcpy_ssd2gpu a = { 0 };
		long st, rc;

		for (i = 0; i < 16; i++)
			ids[i] = rnd(&seed) % 128;
		a.handle = s->h;
		a.offset = (u64)s->tid * 16 * cs;
		a.file_desc = s->fd;
		a.nr_chunks = 16;
		a.chunk_sz = cs;
		a.chunk_ids = ids;
		rc = ksim_ioctl(s->dev, STROM_IOCTL__MEMCPY_SSD2GPU, &a);
		if (rc) {
			s->bad++;
			continue;
		}
		rc = wait_task(s->dev, a.dma_task_id, &st);
		if (rc == -EIO) {
			s->errors++;
			continue;
		}
		if (rc || st) {
			s->bad++;
			continue;
		}
		for (i = 0; i < 16; i++) {
			chunk_bytes(s->f, (u64)ids[i] * cs, cs, exp);
			if (memcmp(s->hbm + a.offset + (u64)i * cs, exp, cs))
				s->bad++;
		}
		s->ok++;
	}
	free(exp);
	return NULL;
}

static int scn_concurrent_sessions(void)
{
	struct world w;
	struct stress_arg sa[4];
	pthread_t th[4];
	struct fmodel f;
	unsigned long h;
	int fd, db, i, ok = 0, errors = 0;

	up(&w, 9, 128);
	ksim_ctrl_config(w.ctrl, 1, 0, 0);
	f = new_file(w.fs, 4ull << 20, 101, frag_map(1024, 64, 13, 20));
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(2ull << 20, 3, 7);
	h = map_dmabuf(w.dev, db, 0, 2ull << 20);
	ksim_fail_cmd(37, 10);
	for (i = 0; i < 4; i++) {
		sa[i] = (struct stress_arg){ ksim_dev_open(i & 1), fd, i, h, &f, ksim_dmabuf_mem(db) };
		pthread_create(&th[i], NULL, stress_thread, &sa[i]);
	}
	for (i = 0; i < 4; i++) {
		pthread_join(th[i], NULL);
		CHECK_EQ(sa[i].bad, 0);
		ok += sa[i].ok;
		errors += sa[i].errors;
		ksim_close(sa[i].dev);
	}
	CHECK_EQ(errors, 1);
	CHECK_EQ(ok + errors, 240);
	CHECK_EQ(unmap(w.dev, h), 0);
	ksim_close(fd);
	ksim_close(db);
	free(f.data);
	return down(&w);
}

/* ------------------------------------------------------------ driver */
/* MEMCPY_SSD2GPU_EXTENTS on a fragmented file: every extent's bytes at its
 * dst_off (a dirty page inside one written back first and read by DMA),
 * bytes_read = extents + gap bytes = the sectors requested, errors for
 * unsorted and past-EOF extents, a plan-only call reading nothing */
static int scn_extents(void)
{
	struct world w;
	struct strom_memcpy_ssd2gpu_extents a = { 0 };
	struct strom_file_extent x[64], y[2];
	u64 pos = 777, want = 0;
	u32 i, n = 0, s = 99;
	unsigned long h;
	struct fmodel f;
	int fd, db;
	long st;
	u8 *hbm;

	up(&w, 9, 256);
	f = new_file(w.fs, 8ull << 20, 17, frag_map(2048, 100, 5, 40));
	fd = ksim_file_open(f.fi, 1);
	db = ksim_dmabuf_new(16ull << 20, 7, 3);
	hbm = ksim_dmabuf_mem(db);
	h = map_dmabuf(w.dev, db, 0, 16ull << 20);
	CHECK(h);
	while (n < 64 && pos < (8ull << 20) - 200000) {
		x[n].file_off = pos;
		x[n].len = 1 + rnd(&s) % 150000;
		x[n].dst_off = 0;
		x[n].reserved = 0;
		pos += x[n].len + (rnd(&s) % 3 ? rnd(&s) % 20000 : 200000 + rnd(&s) % 100000);
		pos = (pos + 7) & ~7ull;
		want += x[n].len;
		n++;
	}
	{   /* a dirty page inside extent 3 */
		u8 nb[64];
		const u64 at = x[3].file_off + 10;

		memset(nb, 0x3c, sizeof(nb));
		ksim_file_write(f.fi, at, nb, sizeof(nb));
		memcpy(f.data + at, nb, sizeof(nb));
	}
	a.file_desc = fd;
	a.nr_extents = n;
	a.gap_max = 16384;
	a.extents = x;
	a.flags = STROM_EXTENTS_PLAN_ONLY;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU_EXTENTS, &a), 0);
	CHECK_EQ(a.dma_task_id, 0);
	CHECK_EQ(a.bytes_read, want + a.gap_bytes);
	CHECK(a.dst_bytes <= (16ull << 20) - 65536);
	a.flags = 0;
	a.handle = h;
	a.offset = 65536;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU_EXTENTS, &a), 0);
	CHECK(a.dma_task_id != 0);
	CHECK_EQ(wait_task(w.dev, a.dma_task_id, &st), 0);
	CHECK_EQ(st, 0);
	CHECK_EQ((u64)a.nr_dma_blocks * 512, a.bytes_read);
	CHECK(a.nr_dma_submit >= 1);
	for (i = 0; i < n; i++) {
		if (memcmp(hbm + 65536 + x[i].dst_off, f.data + x[i].file_off, x[i].len)) {
			fprintf(stderr, "[%s] extent %u differs\n", g_scn, i);
			g_failures++;
			return 1;
		}
	}
	CHECK_EQ(ksim_pc_get(f.fi, (x[3].file_off + 10) >> 12), 1);   /* written back */
	/* unsorted, then past EOF */
	y[0] = x[5];
	y[1] = x[2];
	a.extents = y;
	a.nr_extents = 2;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU_EXTENTS, &a), -EINVAL);
	y[0].file_off = (8ull << 20) - 100;
	y[0].len = 200;
	a.nr_extents = 1;
	CHECK_EQ(ksim_ioctl(w.dev, STROM_IOCTL__MEMCPY_SSD2GPU_EXTENTS, &a), -ERANGE);
	CHECK_EQ(unmap(w.dev, h), 0);
	ksim_close(fd);
	ksim_close(db);
	free(f.data);
	return down(&w);
}

static const struct { const char *name; int (*fn)(void); } scenarios[] = {
	{ "extents", scn_extents },
	{ "ssd2gpu_landing", scn_ssd2gpu_landing },
	{ "relseg_eof", scn_relseg_eof },
	{ "ssd2ram", scn_ssd2ram },
	{ "errors_and_reclaim", scn_errors_and_reclaim },
	{ "unmap_inflight", scn_unmap_inflight },
	{ "raid0_route", scn_raid0_route },
	{ "ssd2ram_wide_route", scn_ssd2ram_wide_route },
	{ "multipath_alias", scn_multipath_alias },
	{ "stale_volume_cache", scn_stale_volume_cache },
	{ "registry_and_stats", scn_registry_and_stats },
	{ "concurrent_sessions", scn_concurrent_sessions },
};

int main(int argc, char **argv)
{
	size_t i;
	int ran = 0, j;

	if (getenv("KSIM_VERBOSE"))
		ksim_set_verbose(1);
	for (i = 0; i < sizeof(scenarios) / sizeof(scenarios[0]); i++) {
		int want = argc < 2;

		for (j = 1; j < argc; j++)
			want |= !strcmp(argv[j], scenarios[i].name);
		if (!want)
			continue;
		g_scn = scenarios[i].name;
		ran++;
		if (scenarios[i].fn())
			printf("FAIL %s (%s)\n", g_scn, ksim_last_violation());
		else
			printf("ok   %s\n", g_scn);
		fflush(stdout);
	}
	printf("%d scenario(s), %d failure(s)\n", ran, g_failures);
	return g_failures ? 1 : 0;
}
