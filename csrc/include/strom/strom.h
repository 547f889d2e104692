/*
 * strom/strom.h — C ABI of libstrom, the MI355X-native direct-storage
 * engine.  Everything a client needs: the ioctl-compatible entry points
 * (sessions stand in for open file descriptors on /proc/nvme-strom), engine
 * configuration, and the CDNA4 post-read kernels (verify, reorder, scan,
 * decompress, filter) that run on HBM-resident data.
 *
 * Return convention: 0 or a non-negative count on success, -errno on error
 * (never sets errno) — except nvme_strom_ioctl(), which mimics ioctl(2).
 */
#ifndef STROM_STROM_H
#define STROM_STROM_H

#include <stddef.h>
#include <stdint.h>

#include "strom/uapi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- sessions + dispatch ---------------------------------------------- */
const char *strom_version(void);
/* 0 = userspace engine, 1 = kernel module (/proc or /dev node present). */
int strom_provider(void);
int strom_open(void);                    /* new session id (> 0) */
int strom_close(int session);            /* reclaims failed tasks: count */
int strom_ioctl(int session, unsigned long cmd, void *arg);
/* v0.6-style wrapper (utils_common.h): lazily opened per-thread session,
 * returns 0 / -1 with errno set. */
int nvme_strom_ioctl(unsigned long cmd, const void *arg);

/* Synchronous "pread into HBM": [file_off, file_off+len) of fd lands at
 * offset of a mapped GPU range, through the same engine path as
 * MEMCPY_SSD2GPU + WAIT (page-cache pages included, in file order).
 * file_off and len must be 4 KiB multiples.  Returns len or -errno. */
long strom_pread_gpu(int session, unsigned long handle, size_t offset, int fd,
                     uint64_t file_off, uint64_t len);
/* QD1 latency probe: n strom_pread_gpu calls of len bytes at file_offs[i],
 * wall time of each in ns_out[i] (native loop, no caller overhead).
 * Returns 0 or the first failure's -errno. */
int strom_pread_gpu_lat(int session, unsigned long handle, size_t offset, int fd,
                        const uint64_t *file_offs, uint32_t n, uint64_t len, uint64_t *ns_out);
/* The same QD1 probe through the ioctl pair a v0.6 client issues
 * (MEMCPY_SSD2GPU of len/4096 chunks + MEMCPY_WAIT per read): task table,
 * residency probe and planner included.  len <= 1 MiB. */
int strom_ioctl_lat(int session, unsigned long handle, size_t offset, int fd,
                    const uint64_t *file_offs, uint32_t n, uint64_t len, uint64_t *ns_out);
/* The same probe split into phases: phase_ns[i*STROM_NPHASE + k] is the time
 * from the start of read i to the end of phase k, 0 when k was not reached:
 *   0 file lookup   1 chunk plan (residency probe + merge)   2 task + requests
 *   3 storage read   4 stores into HBM (BAR) or the SDMA copy   5 HDP flush
 *   6 request completion   7 WAIT returned (the total). */
#define STROM_NPHASE 8
int strom_pread_gpu_phases(int session, unsigned long handle, size_t offset, int fd,
                           const uint64_t *file_offs, uint32_t n, uint64_t len,
                           uint64_t *phase_ns);
/* The floor under those reads: O_DIRECT pread of len bytes at each offset
 * into aligned host memory (no engine, no HBM), ns per read. */
int strom_pread_raw_lat(int fd, const uint64_t *file_offs, uint32_t n, uint64_t len,
                        uint64_t *ns_out);
/* QD1 pairs, interleaved: a raw O_DIRECT pread (offs[2i]) and a
 * strom_pread_gpu (offs[2i+1]) per pair, order flipped every pair; ns each. */
int strom_pread_pair_lat(int session, unsigned long handle, size_t offset, int fd,
			 const uint64_t *file_offs, uint32_t npairs, uint64_t len,
			 uint64_t *ns_engine, uint64_t *ns_raw);

/* Host primitive costs (ns per call, mean of n) on this machine, for the
 * latency breakdown: {clock_gettime, rdtsc, fstat(fd), mincore 1 page of fd,
 * bare syscall, mutex lock+unlock, condvar notify} -> out[7]. */
int strom_host_costs(int fd, uint64_t *out, int n);
/* the engine's own steps of a synchronous read (registry lookup, freed-range
 * check, file cache, completion bookkeeping), ns per call; out[6..13] are a
 * 4 KiB BAR store and the first locked instruction after it,
 * for memcpy / whole-line non-temporal / the same last line first / rep movsb,
 * then the 4 KiB split over two cores (start to both halves drained) and
 * that split's hand-off alone -> out[16] */
int strom_engine_costs(unsigned long handle, int fd, uint64_t *out, int n);

/* Storage ceiling for a block size, no engine: `threads` io_uring rings,
 * each `qd` deep, O_DIRECT reads of `block` bytes at random aligned
 * offsets (or, `sequential`, each ring its own run in file order) into
 * host memory until `nreq` reads are done. */
int strom_raw_read_rate(int fd, uint64_t block, uint32_t nreq, uint32_t threads, uint32_t qd,
                        int sequential, double *iops, double *gibps);
/* The same rings reading exactly the requests (off[i], len[i]), 4 KiB
 * aligned, thread t taking the t-th contiguous share of the list: the
 * storage's rate for the access pattern an engine call produced. */
int strom_raw_read_list(int fd, const uint64_t *off, const uint32_t *len, uint32_t n,
                        uint32_t threads, uint32_t qd, int mode, double *iops, double *gibps);

/* dma-buf fd of the HIP allocation holding [va, va+len) and va's byte
 * offset inside it: what MAP_GPU_MEMORY registers with the kernel provider
 * (MAP_GPU_DMABUF).  The caller closes the fd. */
int strom_export_dmabuf(uint64_t va, uint64_t len, int *fd, uint64_t *offset);

/* Stripe set: a logical file of `size` bytes striped in `unit`-byte
 * stripes (multiple of 4 KiB) over n member files (stripe s in member
 * s % n at offset (s / n) * unit) — one member per SSD aggregates them
 * without md.  Returns a pseudo descriptor usable as file_desc for
 * CHECK_FILE / SSD2GPU / SSD2RAM / strom_pread_gpu until closed; -ERANGE
 * when a member is too short.  Userspace provider only. */
int strom_stripe_open(const int *fds, uint32_t n, uint32_t unit, uint64_t size);
int strom_stripe_close(int sfd);
/* Registered file (as io_uring's registered files): the descriptor is
 * resolved once; the returned id is accepted wherever a file descriptor is
 * and skips the per-read identity check (fstat / kcmp).  The engine reads
 * through descriptors of its own: the caller may close fd.  An id lives
 * until strom_unregister_file() or an engine reset (-EBADF after). */
int strom_register_file(int fd);
int strom_unregister_file(int rfd);

/* SSD2RAM destinations: mmap (MAP_SHARED, read/write) `length` bytes of an
 * ALLOC_DMA_BUFFER fd through the engine, so the range is found in the
 * registry's address index; NULL + errno on failure.  Unmap with
 * strom_dmabuf_munmap.  A caller's own mmap of the fd works too (looked up
 * by one PROCMAP_QUERY per request). */
void *strom_dmabuf_mmap(int fd, size_t length);
int strom_dmabuf_munmap(void *addr, size_t length);
/* Drop DMA buffers no fd and no mapping of the process refers to any more;
 * returns how many stay registered. */
int strom_dmabuf_gc(void);
/* Mappings detached because their allocation was freed or replaced. */
long strom_gpu_detached(void);
/* Bytes of a mapping the CPU can store into through the large BAR (0: none;
 * small reads then go staging -> SDMA / ingest grid instead). */
long strom_gpu_bar_bytes(unsigned long handle);

/* Placement facts of a file for GPU<->SSD affinity (CHECK_FILE tells
 * only the NUMA node): the backing disk, its members (md raid0) and the
 * PCI function of each member's controller (NVMe, or whatever PCI device
 * the disk hangs off; "" when unknown).  nmembers = 0 for a virtual filesystem (overlay, tmpfs). */
#define STROM_TOPO_MAX_MEMBERS 16
typedef struct strom_file_topo {
  uint32_t dev_major, dev_minor; /* st_dev of the file */
  int32_t numa_node;
  uint32_t nmembers;
  char fs_name[16];
  char disk[32];
  char member_disk[STROM_TOPO_MAX_MEMBERS][32];
  char member_pci[STROM_TOPO_MAX_MEMBERS][16];
} strom_file_topo;
int strom_file_topology(int fd, strom_file_topo *out);
/* PCI function "dddd:bb:dd.f" of a HIP device (no GPU init past the
 * runtime's own); -ENODEV without one. */
int strom_gpu_pci_bdf(int device, char *buf, size_t len);

/* HBM ingest grid of a device (the persistent GPU pull kernel that moves
 * staged reads into HBM): out[4] = {available, grid launches, descriptors
 * posted, descriptors outstanding}.  -ENODEV when it cannot run there. */
int strom_ingest_info(int device, uint64_t *out);

/* Worker phase attribution (config io_prof=1): out[0] workers, out[1] TSC
 * kHz, out[2..12] TSC cycles summed over the workers per phase (idle, take,
 * start, submit, reap, bar, post, hdp, finish, retire, wait), out[13..17]
 * counts (requests, batches, io_uring_enter calls, sleeps, HBM
 * descriptors), out[18..21] the submitting side (SSD2GPU/SSD2RAM calls and
 * TSC cycles planning, building requests, handing them over).  reset != 0
 * zeroes them.  Returns the number of u64 written (22) or -errno. */
int strom_io_prof(uint64_t *out, int nout, int reset);

/* ---- configuration (env STROM_<KEY> is read at first use) ------------- */
int strom_config_set(const char *key, const char *value);
int strom_config_get(const char *key, char *buf, size_t buflen);
/* Tear the engine down (waits for in-flight I/O); next call re-creates it
 * with the current configuration. */
int strom_engine_reset(void);

/* ---- fault injection (fake + real backends; CPU tests) ---------------- */
/* Fail the n-th storage request after this call (1-based) with -err; 0
 * disables.  short_at makes the n-th request read `short_bytes` less. */
int strom_fault_inject(long fail_at, int err, long short_at, int short_bytes,
                       int delay_us);

/* Fake namespace backend (backend=fake): completions come back in a seeded
 * random order.  Sets the seed (0 keeps it; takes effect at the next
 * engine reset) and reads the completion / out-of-order counters. */
int strom_fake_backend(uint64_t seed, uint64_t *completions, uint64_t *reordered);

/* ---- host helpers ------------------------------------------------------ */
/* Bytes of a file range resident in the page cache (mincore). */
long strom_resident_bytes(int fd, uint64_t offset, uint64_t length);
/* Drop clean page-cache pages of a file (posix_fadvise DONTNEED). */
int strom_evict_file(int fd);
/* CRC32C (Castagnoli) on the host, same convention as the GPU kernels. */
uint32_t strom_crc32c_host(uint32_t crc, const void *buf, size_t len);
/* md raid0 remap for a described geometry (tests + kmod parity). */
int strom_raid0_map(const uint64_t *zone_end, const uint64_t *zone_dev_start,
                    const int *zone_nb_dev, int nzones,
                    uint32_t chunk_sects, const uint64_t *data_offset,
                    int raid_disks, uint64_t sector, uint32_t nr_sects,
                    int *member, uint64_t *member_sector);
/* Host LZ4 / snappy block codecs (test-data generation + CPU reference). */
long strom_lz4_compress_host(const void *src, size_t n, void *dst, size_t cap);
long strom_lz4_decompress_host(const void *src, size_t n, void *dst, size_t cap);
long strom_snappy_compress_host(const void *src, size_t n, void *dst, size_t cap);
long strom_snappy_decompress_host(const void *src, size_t n, void *dst, size_t cap);

/* ---- CDNA4 kernels (device pointers, hipStream_t passed as void*) ----- */
int strom_gpu_count(void);
/* Per-chunk CRC32C: out[i] = crc32c(in + i*chunk, min(chunk, n - i*chunk)). */
int strom_crc32c_chunks(const void *d_in, uint64_t nbytes, uint32_t chunk,
                        uint32_t *d_out, void *stream);
/* Fold per-chunk CRCs (equal chunk sizes, last may be short) into the CRC
 * of the whole buffer; d_out is one u32. */
int strom_crc32c_combine(const uint32_t *d_crcs, uint32_t nchunks,
                         uint32_t chunk, uint64_t nbytes, uint32_t *d_out,
                         void *stream);
/* Chunk scatter: dst + pos[i]*chunk <- src + i*chunk, i < n. */
int strom_chunk_scatter(const void *d_src, void *d_dst, const uint32_t *d_pos,
                        uint32_t n, uint32_t chunk, void *stream);
/* Chunk gather: dst + i*chunk <- src + idx[i]*chunk. */
int strom_chunk_gather(const void *d_src, void *d_dst, const uint32_t *d_idx,
                       uint32_t n, uint32_t chunk, void *stream);
/* Compare against a 32-bit pattern / a reference buffer: out[0] = mismatching
 * 4-byte words, out[1] = first mismatching byte offset (or ~0). */
int strom_verify_pattern(const void *d_buf, uint64_t nbytes, uint32_t pattern,
                         uint64_t *d_out, void *stream);
int strom_verify_equal(const void *d_a, const void *d_b, uint64_t nbytes,
                       uint64_t *d_out, void *stream);
int strom_fill_pattern(void *d_buf, uint64_t nbytes, uint32_t pattern,
                       void *stream);

/* The full HeapTupleSatisfiesMVCC inputs (heapam_visibility.c): snapshot
 * (xmin, xmax, xip, subxip / suboverflowed), the scanning transaction's own
 * xids and command id, and windows of the SLRU logs — pg_xact (2 bits per
 * xid from clog_base), pg_subtrans (parent xid per xid from subtrans_base),
 * pg_multixact offsets (member offset per multixact from mx_base, n + 1
 * entries: the last is the next offset) and members (PostgreSQL's page
 * layout: 409 groups of 4 flag bytes + 4 xids per 8 KiB page, from member
 * offset mxm_base).  Transaction ids compare modulo 2^32. */
struct strom_pg_mvcc {
	uint32_t xmin, xmax;
	const uint32_t *xip;
	uint32_t nxip;
	uint32_t suboverflowed;
	const uint32_t *subxip;
	uint32_t nsubxip;
	uint32_t curcid;
	const uint32_t *curxids;  /* the scanning transaction: top xid + its subxacts */
	uint32_t ncurxids;
	uint32_t clog_base;
	const uint8_t *clog;
	uint64_t clog_n;
	const uint32_t *subtrans;
	uint32_t subtrans_base, subtrans_n;
	const uint32_t *mx_offsets;
	uint32_t mx_base, mx_n;
	const uint8_t *mx_members;
	uint64_t mxm_n;
	uint32_t mxm_base, pad;
};

/* PostgreSQL heap pages (8 KiB by default). */
struct strom_heap_scan_args {
	const void *pages;       /* device: npages * page_sz bytes */
	uint32_t npages;
	uint32_t page_sz;
	uint32_t flags;          /* STROM_HEAP_* */
	int32_t  attr_off;       /* byte offset of the filtered int column in
	                            tuple data (after t_hoff), -1 = no filter */
	int32_t  attr_width;     /* 4 or 8 */
	int64_t  lo, hi;         /* keep rows with lo <= v <= hi */
	uint32_t *out_items;     /* device: (page << 16) | lineno, capacity below */
	uint32_t out_cap;
	uint32_t *out_count;     /* device: u32[1], total qualifying */
	uint32_t *page_status;   /* device: per page bitfield (STROM_PAGE_*) */
	uint32_t blkno_base;     /* block number of page 0 (checksum input) */
	const uint32_t *blknos;  /* device, optional: block number per page
	                            (pages landed out of order); overrides
	                            blkno_base + page */
};
#define STROM_HEAP_VERIFY_CHECKSUM 1u
#define STROM_HEAP_SKIP_INVISIBLE  2u   /* honour xmin/xmax hint bits */
#define STROM_PAGE_BAD_HEADER  1u
#define STROM_PAGE_BAD_CHECKSUM 2u
#define STROM_PAGE_EMPTY       4u
int strom_heap_scan(const struct strom_heap_scan_args *a, void *stream);

/* General tuple deforming + qualifier lists (the reference hands every tuple
 * to ExecScan, which deforms it and evaluates any qual list:
 * pgsql/nvme_strom.c:1137-1143, :1054-1092).  A tuple descriptor in
 * PostgreSQL's pg_attribute terms locates every attribute: the null bitmap
 * (HEAP_HASNULL, t_bits), attalign padding, fixed lengths, and varlena
 * headers (1-byte short, 4-byte, 1-byte-external TOAST pointers).  Tuples
 * with fewer stored attributes than the descriptor (ALTER TABLE ADD COLUMN)
 * read the missing ones as NULL. */
#define STROM_HEAP_MAX_ATTS  64
#define STROM_HEAP_MAX_QUALS 8
struct strom_heap_tupdesc {
	int32_t natts;
	int16_t attlen[STROM_HEAP_MAX_ATTS];    /* > 0 fixed, -1 varlena, -2 cstring */
	uint8_t attalign[STROM_HEAP_MAX_ATTS];  /* 1, 2, 4 or 8 ('c' 's' 'i' 'd') */
	int16_t cacheoff[STROM_HEAP_MAX_ATTS];  /* offset after t_hoff when every earlier
	                                           attribute is fixed-length (tuples without
	                                           nulls), else -1 (attcacheoff) */
};
#define STROM_QUAL_INT_RANGE    1  /* lo <= v <= hi, v an int of attlen 1/2/4/8 */
#define STROM_QUAL_FLOAT_RANGE  2  /* lo <= v <= hi as doubles (bit patterns in lo/hi),
                                      v a float4 / float8 */
#define STROM_QUAL_IS_NULL      3
#define STROM_QUAL_NOT_NULL     4
#define STROM_QUAL_TEXT_EQ      5  /* varlena bytes == cbytes[0..nconst) */
#define STROM_QUAL_TEXT_PREFIX  6  /* varlena bytes start with cbytes[0..nconst) */
#define STROM_QUAL_INT_IN       7  /* v in { ((int64_t *)cbytes)[0..nconst) } (<= 4) */
struct strom_heap_qual {
	int16_t attno;       /* 0-based column */
	uint8_t kind;        /* STROM_QUAL_* */
	uint8_t nconst;      /* TEXT_*: constant length (<= 32); INT_IN: values (<= 4) */
	uint32_t pad;
	int64_t lo, hi;
	uint8_t cbytes[32];
};
/* A text qualifier meets a compressed or out-of-line (TOAST) value: the GPU
 * cannot decide it, the tuple is not emitted and its page is flagged
 * STROM_PAGE_RECHECK for the host to re-evaluate. */
#define STROM_PAGE_RECHECK     8u
#define STROM_QUAL_TEXT_IN      8  /* varlena bytes == one of nconst constants */
#define STROM_QUAL_NUMERIC_RANGE 9 /* lo <= v <= hi, v a PostgreSQL numeric */
#define STROM_QUAL2_FALSE 0x80   /* strom_heap_qual2.flags: the qual is constant false */
/* A qualifier of a program (strom_heap_scan2_args.prog): quals with the
 * same clause id are ORed and contiguous, clauses are ANDed (CNF); any
 * number of either.  Constants live in a device pool:
 *   TEXT_EQ / TEXT_PREFIX  nconst bytes at coff (any length)
 *   INT_IN                 nconst int64 at coff (any count)
 *   TEXT_IN                nconst (uint32 offset, uint32 length) at coff
 *   NUMERIC_RANGE          constants at pool offsets lo and hi: uint16 kind
 *                          (0 finite, 1 NaN, 2 +inf, 3 -inf), uint16 sign
 *                          (0 / 1 negative), int16 weight, uint16 ndigits,
 *                          int16 base-10000 digits (no leading / trailing 0s)
 * flags (NUMERIC_RANGE): 1 no lower bound, 2 no upper bound, 4 lower
 * strict, 8 upper strict. */
struct strom_heap_qual2 {
	int16_t attno;
	uint8_t kind;
	uint8_t flags;
	uint32_t clause;
	uint32_t nconst;
	uint32_t coff;
	int64_t lo, hi;
};
struct strom_heap_scan2_args {
	struct strom_heap_scan_args base;     /* base.attr_off must be -1 */
	struct strom_heap_tupdesc desc;
	int32_t nquals;                       /* ANDed; NULL never qualifies
	                                         except for IS_NULL */
	struct strom_heap_qual quals[STROM_HEAP_MAX_QUALS];
	uint32_t *recheck_count;              /* device, optional: undecidable tuples */
	/* program mode (prog != NULL; quals / nquals unused): nprog quals in
	 * device memory, their constants in cpool (cpool_len bytes) */
	const struct strom_heap_qual2 *prog;
	const uint8_t *cpool;                 /* 8-aligned constants, cpool_len % 8 == 0 */
	uint32_t nprog, cpool_len;
	/* Snapshot visibility on the device (mvcc_on != 0): every LP_NORMAL
	 * tuple of a page that is not PD_ALL_VISIBLE — and, with mvcc_pages,
	 * whose byte is nonzero (the visibility map said "not all-visible") — is
	 * checked with HeapTupleSatisfiesMVCC's rules (strom_pg_tuple_visible's,
	 * pgsql/nvme_strom.c:907-936 runs them per buffer-manager tuple).  An
	 * invisible tuple is dropped and counted in mvcc_removed[0]; one the
	 * inputs cannot decide (combo cid, an xid / multixact outside the
	 * windows) is kept, as the host check keeps it, and its page flagged
	 * STROM_PAGE_RECHECK.  mvcc's pointers are DEVICE memory, and xip /
	 * subxip / curxids must be sorted ascending (binary-searched). */
	struct strom_pg_mvcc mvcc;
	const uint8_t *mvcc_pages;            /* device, optional: per page */
	uint32_t *mvcc_removed;               /* device, optional: u32[1] */
	uint32_t mvcc_on;
	/* optional: bit k set when xid mvcc.xmin + k is running for the
	 * snapshot (in xip, or in subxip unless suboverflowed), k < running_bits
	 * = xmax - xmin: XidInMVCCSnapshot's list searches become one load */
	uint32_t mvcc_running_bits;
	const uint32_t *mvcc_running;
};
int strom_heap_scan2(const struct strom_heap_scan2_args *a, void *stream);
/* strom_heap_scan (the fixed-offset int predicate) with the device snapshot
 * check above; m holds device pointers (NULL m: hint bits only). */
int strom_heap_scan_mvcc(const struct strom_heap_scan_args *a, const struct strom_pg_mvcc *m,
                         const uint8_t *mvcc_pages, uint32_t *mvcc_removed,
                         uint32_t *recheck_count, const uint32_t *running,
                         uint32_t running_bits, void *stream);
/* The host ("buffer manager") path for blocks checked on the CPU: each
 * block blocks[i] is read (pread of page_sz bytes at (block % relseg_blocks)
 * * page_sz; relseg_blocks 0: no modulo) into stage + i * page_sz, a short
 * read zero-filled; with verify_checksum its checksum is tested first and,
 * when valid, re-stamped after the edit (as ReadBuffer + a hint-bit write);
 * then the tuples m hides are marked LP_UNUSED.  recheck_flags[i] (optional)
 * = 1 when the block holds tuples the inputs cannot decide.  Returns the
 * tuples removed, or -errno of a failed read. */
long strom_pg_read_check_pages(int fd, const uint32_t *blocks, uint32_t n, uint32_t relseg_blocks,
                               uint32_t page_sz, void *stage, const struct strom_pg_mvcc *m,
                               int verify_checksum, uint8_t *recheck_flags);
/* Checks a program and its pool (host copies of what prog / cpool hold)
 * before a launch: kinds against the attributes, contiguous clauses, every
 * constant (IN tables and the text entries they name, numeric digits)
 * inside the pool.  0 or -EINVAL. */
int strom_heap_prog_check(const struct strom_heap_tupdesc *d, const struct strom_heap_qual2 *prog,
			  uint32_t n, const uint8_t *pool, uint32_t pool_len);
/* Projection of one attribute of the tuples `items` (page << 16 | lineno,
 * as strom_heap_scan writes them) names: values[i] (8 bytes: the int
 * sign-extended, float4 widened to double, varlena: (offset in pages <<
 * 32 | data length) of the uncompressed inline bytes) and valid[i] (0 NULL,
 * 1 value, 2 compressed / out-of-line varlena).  *d_count (device) is the
 * number of items; at most cap are read. */
int strom_heap_project(const void *pages, uint32_t page_sz, const uint32_t *items,
                       const uint32_t *d_count, uint32_t cap,
                       const struct strom_heap_tupdesc *desc, int attno, int as_float,
                       uint64_t *values, uint8_t *valid, void *stream);
/* several attributes in one deform walk per tuple: values / valid are
 * [ncol][cap], column j as float64 when bit j of float_mask is set */
int strom_heap_project_n(const void *pages, uint32_t page_sz, const uint32_t *items,
                         const uint32_t *d_count, uint32_t cap,
                         const struct strom_heap_tupdesc *desc, const int32_t *attnos,
                         uint32_t ncol, uint64_t float_mask, uint64_t *values, uint8_t *valid,
                         void *stream);
uint16_t strom_pg_checksum_host(const void *page, uint32_t blkno,
                                uint32_t page_sz);
/* Per-tuple MVCC check of a heap page against a snapshot (xmin, xmax,
 * in-progress xids) and a commit log (pg_xact layout, 2 bits per xid):
 * invisible LP_NORMAL tuples are marked LP_UNUSED in place, as the
 * reference does before copying buffer-manager blocks into its chunk
 * (pgsql/nvme_strom.c:896-940).  PD_ALL_VISIBLE pages are left alone.
 * Returns the tuples removed. */
long strom_pg_apply_snapshot(void *page, uint32_t page_sz, uint32_t snap_xmin, uint32_t snap_xmax,
                             const uint32_t *xip, uint32_t nxip, const uint8_t *clog,
                             uint64_t clog_xids);
/* The same in-place marking with the full rules; tuples the inputs cannot
 * decide (a combo command id of the scanning transaction, an xid / multixact
 * outside the log windows) are kept and their line numbers (1-based)
 * written to recheck[] (up to cap), *nrecheck = their count.  Returns the
 * tuples removed, or -22 for a page that is not a heap page. */
long strom_pg_apply_mvcc(void *page, uint32_t page_sz, const struct strom_pg_mvcc *m,
                         uint16_t *recheck, uint32_t cap, uint32_t *nrecheck);
/* one tuple header: 1 visible, 0 not, -1 undecided */
int strom_pg_tuple_visible(const void *tuple_header, const struct strom_pg_mvcc *m);
/* fetch-and-add on shared memory (cross-process scan cursors) */
uint64_t strom_atomic_fetch_add_u64(uint64_t *addr, uint64_t v);
int strom_atomic_cas_u64(uint64_t *addr, uint64_t expect, uint64_t desired);
uint64_t strom_atomic_load_u64(const uint64_t *addr);

/* LZ4 / snappy raw-block batch decode: one block per wavefront. */
struct strom_decomp_desc {
	uint64_t src_off;      /* into d_src */
	uint64_t dst_off;      /* into d_dst */
	uint32_t src_len;
	uint32_t dst_len;      /* exact decoded size (or capacity) */
};
#define STROM_CODEC_LZ4    1
#define STROM_CODEC_SNAPPY 2
#define STROM_CODEC_COPY   3   /* stored block */
#define STROM_CODEC_LZ4_FRAME     4  /* LZ4 frame data blocks (after header) */
#define STROM_CODEC_LZ4_FRAME_BCS 5  /*   ... with 4-byte block checksums */
#define STROM_CODEC_ARROW_LZ4     6  /* Arrow IPC buffer: i64 length (-1 = raw) + LZ4 frame */
#define STROM_CODEC_ZSTD          7  /* Zstandard frame(s) (RFC 8878) */
#define STROM_CODEC_ARROW_ZSTD    8  /* Arrow IPC buffer: i64 length (-1 = raw) + zstd frame */
/* status[i] = decoded bytes, or -1 malformed / -2 overflow / -3 distance */
int strom_decompress(int codec, const void *d_src, void *d_dst,
                     const struct strom_decomp_desc *d_desc, uint32_t nblocks,
                     int32_t *d_status, void *stream);

/* Zstandard streams, one wavefront each (csrc/kernels/zstd.hip).  scratch:
 * 128 KiB of decoded literals per resident workgroup (NULL: a per-stream
 * buffer kept by the library).  strom_decompress() routes codecs 7/8 here. */
int strom_decompress_zstd(int codec, const void *d_src, void *d_dst,
                          const struct strom_decomp_desc *d_desc, uint32_t nstreams,
                          int32_t *d_status, void *scratch, uint64_t scratch_bytes,
                          void *stream);
/* the same with the decoder chosen by the caller: mode -1 the library's
 * choice, 0 one wave per stream, 1 frame-parallel (a frame's blocks on the
 * waves of a workgroup) */
int strom_decompress_zstd_mode(int codec, const void *d_src, void *d_dst,
                               const struct strom_decomp_desc *d_desc, uint32_t nstreams,
                               int32_t *d_status, void *scratch, uint64_t scratch_bytes,
                               void *stream, int mode);
/* decoder choice for strom_decompress_zstd: -1 by stream count (default),
 * 0 / 1 forced; returns the previous setting */
int strom_zstd_fp_mode(int mode);
/* buffers kept per (device, stream) by the zstd decoders (literal slots,
 * lane-parallel entry pools) */
uint32_t strom_zstd_scratch_keep(void);
/* free the library-kept zstd scratch (after the streams' last decodes) */
int strom_zstd_release(void);
/* the same decode on the CPU (the kernel's phases lane by lane) */
int strom_zstd_host(int codec, const uint8_t *src, uint32_t src_len, uint8_t *dst, uint32_t cap);

/* Columnar filter: bitmap[i/64] bit i%64 = valid(i) && lo <= v[i] <= hi. */
#define STROM_COL_I32 1
#define STROM_COL_I64 2
#define STROM_COL_F32 3
#define STROM_COL_F64 4
int strom_column_filter(int type, const void *d_values, const uint8_t *d_valid,
                        uint64_t n, double lo, double hi, uint64_t *d_bitmap,
                        uint64_t *d_count, void *stream);
/* Compact selected row indices from a bitmap (stable order). */
int strom_bitmap_to_indices(const uint64_t *d_bitmap, uint64_t n,
                            uint32_t *d_out, uint64_t *d_count, void *stream);

/* Batched scan over many record batches in ONE launch each, counts kept on
 * the device (no host sync per batch).  Batch b's rows occupy bitmap words
 * [word_base, word_base + ceil(nrows/64)) (every batch starts on a fresh
 * word); values / valid are device addresses (valid = 0: no nulls; Arrow
 * LSB-first bits, readable as whole 64-bit words). */
struct strom_filter_batch {
	uint64_t values;
	uint64_t valid;
	uint64_t nrows;
	uint64_t word_base;
	uint64_t row_base;     /* global row id of the batch's first row */
};
/* *d_count += selected rows (the caller zeroes it once per scan). */
int strom_column_filter_batched(int type, const struct strom_filter_batch *d_batches,
                                uint32_t nbatches, uint64_t nwords, double lo, double hi,
                                uint64_t *d_bitmap, uint64_t *d_count, void *stream);
/* Append the global row ids (int64, batch row_base + local row) of the set
 * bits to d_out at the device-side cursor *d_total, which advances by the
 * number appended: scans of successive groups fill one output in order. */
int strom_bitmap_to_rows(const uint64_t *d_bitmap, uint64_t nwords,
                         const struct strom_filter_batch *d_batches, uint32_t nbatches,
                         int64_t *d_out, uint64_t *d_total, void *stream);
/* Qualifier lists: combine != 0 ANDs the predicate into the existing
 * bitmap words (count = rows left selected). */
int strom_column_filter_batched2(int type, const struct strom_filter_batch *d_batches,
                                 uint32_t nbatches, uint64_t nwords, double lo, double hi,
                                 uint64_t *d_bitmap, uint64_t *d_count, int combine, void *stream);
/* bitmap_to_rows + projection: d_proj (same batches, another column's
 * values/valid pointers) non-NULL gathers each selected row's value (width 4
 * or 8 bytes) into d_pout[pos] and, when d_pvalid, its validity (0/1). */
int strom_bitmap_to_rows_proj(const uint64_t *d_bitmap, uint64_t nwords,
                              const struct strom_filter_batch *d_batches, uint32_t nbatches,
                              int64_t *d_out, uint64_t *d_total,
                              const struct strom_filter_batch *d_proj, uint32_t width,
                              void *d_pout, uint8_t *d_pvalid, void *stream);

/* General column qualifiers (Arrow scans; nvme_strom_amd/ops/colpred.py
 * compiles the predicates).  Storage types beyond STROM_COL_I32..F64: */
#define STROM_COL_I8 5
#define STROM_COL_I16 6
#define STROM_COL_U8 7
#define STROM_COL_U16 8
#define STROM_COL_U32 9
#define STROM_COL_U64 10
#define STROM_COL_BOOL 11   /* bit-packed values */
#define STROM_COL_STR32 12  /* utf8/binary: int32 offsets in values, bytes in aux */
#define STROM_COL_STR64 13  /* large utf8/binary: int64 offsets */
#define STROM_COL_DEC128 14 /* decimal128: 16-byte two's complement (value x 10^scale);
                               RANGES bounds are 16-byte pairs */
/* operators */
#define STROM_QOP_RANGES 1     /* v in one of nconst inclusive ranges: sorted, disjoint
                                  (lo, hi) pairs of int64 (U64: uint64; floats: double) */
#define STROM_QOP_STR_IN 2     /* the string equals one of nconst constants */
#define STROM_QOP_STR_PREFIX 3 /* starts with one of nconst constants */
#define STROM_QOP_LUT 4        /* index v < nconst with bit v of the uint32 LUT words set
                                  (dictionary-encoded columns) */
#define STROM_QOP_VALID 5      /* the row is not null (NEGATE: is null) */
#define STROM_QOP_STR_RANGES 6 /* bytewise-lexicographic ranges: per range two bounds of
                                  (start, len, mode) in offs, mode 0 unbounded,
                                  1 inclusive, 2 exclusive */
#define STROM_QUAL_NEGATE 1    /* NOT of the comparison (still false for nulls) */
#define STROM_QUAL_NAN 2       /* floats: NaN also matches (IN-lists holding NaN) */
struct strom_col_qual {
	int32_t type;
	int32_t op;
	uint32_t flags;
	uint32_t nconst;
	uint64_t consts;       /* device: ranges / string blob / LUT words */
	uint64_t offs;         /* device: strings, (start, len) uint32 pairs; starts 4-aligned */
	uint64_t const_bytes;  /* bytes at consts (staged in LDS, <= 64 KiB) */
	uint64_t offs_bytes;
};
/* strom_filter_batch + aux (the character data of a string column, aux_len
 * bytes: offsets outside it never match and are never followed) */
struct strom_qual_batch {
	uint64_t values;
	uint64_t valid;
	uint64_t nrows;
	uint64_t word_base;
	uint64_t row_base;
	uint64_t aux;
	uint64_t aux_len;
};
/* bitmap[w] = (pred_bits | (d_or ? d_or[w] : 0)) & (and_dst ? bitmap[w] : ~0);
 * *d_count += popcount of the words written.  A CNF qualifier list is a
 * sequence of these launches (OR within a clause, AND across clauses). */
int strom_column_qual(const struct strom_col_qual *q, const struct strom_qual_batch *d_batches,
                      uint32_t nbatches, uint64_t nwords, uint64_t *d_bitmap,
                      const uint64_t *d_or, int and_dst, uint64_t *d_count, void *stream);
/* bitmap_to_rows with a utf8/binary column projected (d_strtab: its
 * strom_qual_batch rows, offsets of owidth 4 or 8 bytes): each selected row's
 * characters are appended at the device cursor *d_char_cursor in d_pchars,
 * its start written to d_poff[pos] (and its validity to d_pvalid when given). */
int strom_bitmap_to_rows_str(const uint64_t *d_bitmap, uint64_t nwords,
                             const struct strom_filter_batch *d_batches, uint32_t nbatches,
                             int64_t *d_out, uint64_t *d_total,
                             const struct strom_qual_batch *d_strtab, uint32_t owidth,
                             int64_t *d_poff, uint8_t *d_pchars, uint8_t *d_pvalid,
                             uint64_t *d_char_cursor, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* STROM_STROM_H */
