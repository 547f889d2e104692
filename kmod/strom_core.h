/* SPDX-License-Identifier: GPL-2.0 */
/*
 * strom_core.h — the kernel-free logic of the nvme-strom providers.
 *
 * One C unit (strom_core.c) compiled three ways: into the kernel module
 * (kmod/Makefile), into libstrom.so (the userspace engine's planner uses the
 * same merge rules), and into the CPU test-suite through libstrom
 * (tests/test_kmod_core_cpu.py).  Nothing here touches kernel or libc state:
 * callers pass callbacks for block mapping, submission and bus addresses.
 *
 * Reference semantics re-derived (not copied) from kmod/nvme_strom.c:
 *   chunk position + EOF rule   do_memcpy_ssd2gpu/ssd2ram   :1524-1529, :1810-1814
 *   page-cache majority score   :1532-1540, :1820-1836 (dirty page = threshold+1)
 *   landing order               SSD chunks packed at the head, RAM chunks from
 *                               the tail (SSD2GPU); identity (SSD2RAM) :1546-1571
 *   request merge               memcpy_from_nvme_ssd :1303-1405 (same member,
 *                               contiguous sectors, contiguous destination,
 *                               <= max request, no destination-segment crossing)
 *   md raid0 remap              strom_raid0_map_sector :755-820 (-ESPIPE across
 *                               a stripe chunk)
 *   PRP1/PRP2/PRP list          submit_ssd2gpu_memcpy :1415-1482, with bus
 *                               addresses from a flattened dma-buf sg table
 *                               (never raw physical addresses: defect #8)
 */
#ifndef STROM_CORE_H
#define STROM_CORE_H

#ifdef __KERNEL__
#include <linux/errno.h>
#include <linux/types.h>
typedef u8 sc_u8;
typedef u32 sc_u32;
typedef u64 sc_u64;
typedef s64 sc_s64;
#else
#include <errno.h>
#include <stdbool.h>
#include <stdint.h>
typedef uint8_t sc_u8;
typedef uint32_t sc_u32;
typedef uint64_t sc_u64;
typedef int64_t sc_s64;
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define STROM_CORE_PAGE        4096u      /* NVMe controller page (CC.MPS = 0) */
#define STROM_CORE_PAGE_SHIFT  12
#define STROM_CORE_PRP_LIST_MAX 512u      /* entries of one 4 KiB PRP list page */
/* largest request whose PRPs fit PRP1 + one list page */
#define STROM_CORE_MAX_REQ     ((STROM_CORE_PRP_LIST_MAX + 1u) * STROM_CORE_PAGE)
#define STROM_RAID0_MAX_ZONES  16
#define STROM_RAID0_MAX_DISKS  32

/* ---- chunk position, page-cache score, landing order ------------------- */

/* File position of chunk `cid` (relseg_sz != 0: position inside its segment
 * file).  -ERANGE when the chunk starts at or past EOF (defect #10: the
 * reference accepted a chunk starting exactly at EOF). */
int strom_core_chunk_fpos(sc_u32 cid, sc_u32 chunk_sz, sc_u32 relseg_sz, sc_u64 isize,
			  sc_u64 *fpos);

/* Majority rule: a chunk of npages is served from the page cache when the
 * score of its resident pages exceeds npages/2; a dirty page scores
 * threshold + 1, so one dirty page always wins (dirty data is never bypassed). */
static inline sc_u32 strom_core_cache_threshold(sc_u32 npages) { return npages / 2; }
static inline sc_u32 strom_core_cache_add(sc_u32 score, sc_u32 threshold, bool dirty)
{
	return score + (dirty ? threshold + 1 : 1);
}
static inline bool strom_core_cache_wins(sc_u32 score, sc_u32 threshold)
{
	return score > threshold;
}

struct strom_landing {
	sc_u32 nr_chunks;
	sc_u32 nr_ram;           /* out: chunks served from RAM */
	sc_u32 nr_ssd;           /* out: chunks read from storage */
	bool reorder;            /* SSD2GPU: storage head / RAM tail; SSD2RAM: identity */
};

/* Destination slot of the i-th requested chunk. */
sc_u32 strom_core_land(struct strom_landing *l, sc_u32 i, bool cached);

/* ---- md raid0 ------------------------------------------------------------ */
struct strom_raid0 {
	sc_u32 chunk_sects;                  /* 512-B sectors per stripe chunk */
	sc_u32 nzones;
	sc_u32 ndisks;
	sc_u64 zone_end[STROM_RAID0_MAX_ZONES];        /* md sector, exclusive */
	sc_u64 zone_dev_start[STROM_RAID0_MAX_ZONES];  /* member sector of the zone start */
	sc_u32 zone_nb_dev[STROM_RAID0_MAX_ZONES];
	sc_u8 zone_devs[STROM_RAID0_MAX_ZONES][STROM_RAID0_MAX_DISKS]; /* member per slot */
	sc_u64 data_offset[STROM_RAID0_MAX_DISKS];     /* per member, sectors */
};

/* -EINVAL on an inconsistent geometry (zones not increasing, a zone wider
 * than the member count, a member index out of range, chunk not a multiple
 * of 8 sectors). */
int strom_core_raid0_check(const struct strom_raid0 *g);
/* Member + member sector of [sector, sector + nr): -ESPIPE when the range
 * crosses a stripe chunk, -ERANGE past the array. */
int strom_core_raid0_map(const struct strom_raid0 *g, sc_u64 sector, sc_u32 nr, int *member,
			 sc_u64 *msector);

/* ---- extent planner -------------------------------------------------------- */
struct strom_extent {
	sc_u64 file_off;         /* byte offset in the file */
	sc_u64 sect;             /* 512-B sector on the volume (member sector under raid0) */
	sc_u64 dest;             /* byte offset in the destination */
	sc_u32 len;              /* bytes, multiple of 4 KiB */
	int member;              /* raid0 member, -1 = the volume itself */
};

struct strom_planner {
	/* configuration */
	sc_u32 max_req;          /* merge limit in bytes */
	bool prp_limited;        /* NVMe PRPs: clamp max_req to STROM_CORE_MAX_REQ */
	bool file_contig;        /* merged requests must also be contiguous in the
				    file (userspace reads by file offset) */
	sc_u64 dest_segment;     /* no request crosses a multiple of this (0: none) */
	sc_u32 blkbits;          /* filesystem block bits, 9..12 */
	sc_u64 part_start_sect;  /* partition start on the volume */
	const struct strom_raid0 *raid0;   /* NULL: single device */
	/* fs block -> device block (both in fs blocks); holes and unwritten
	 * extents are the callback's -EIO */
	int (*bmap)(void *ctx, sc_u64 fblk, sc_u64 *dblk);
	void *bmap_ctx;
	int (*submit)(void *ctx, const struct strom_extent *e);
	void *submit_ctx;
	/* state */
	struct strom_extent cur;
	sc_u32 nr_submit;
	sc_u64 nr_sectors;
};

void strom_core_planner_init(struct strom_planner *p);
/* Map [fpos, fpos + len) page by page and merge into requests, submitting
 * each finished one.  fpos and len are 4 KiB aligned.  -EOPNOTSUPP when
 * a page is not contiguous on the device,
 * -ESPIPE / -ERANGE from the raid0 remap, or the callbacks' errors. */
int strom_core_plan_range(struct strom_planner *p, sc_u64 fpos, sc_u32 len, sc_u64 dest);
int strom_core_plan_flush(struct strom_planner *p);

/* ---- exact extent reads (MEMCPY_SSD2GPU_EXTENTS) ----------------------------
 * Layout-identical to uapi.h struct strom_file_extent (both providers assert
 * it): the caller's (file_off, len) in, dst_off out. */
struct strom_xfer_extent {
	sc_u64 file_off;
	sc_u64 dst_off;
	sc_u32 len;
	sc_u32 reserved;
};
/* n extents, sorted by file offset and disjoint, each ending at or before
 * isize, laid out for page-granular reads: an extent is widened to whole
 * 4 KiB pages; one whose first page starts at most gap_max bytes past the
 * current run's last page joins that run (the hole is read too), otherwise
 * it starts a new run.  Runs land back to back from destination 0, every
 * extent at the same distance from its run's start as in the file
 * (x[i].dst_off; 0 for an empty extent).  With a planner, every run goes to
 * strom_core_plan_range (its merge rules split it into requests; the caller
 * flushes); pages wholly past isize are not read.  *dst_bytes: destination
 * span; *read_bytes: bytes the requests read.  0, -EINVAL (unsorted or
 * overlapping), -ERANGE (past isize) or the planner's error. */
int strom_core_plan_xfer(struct strom_planner *p, struct strom_xfer_extent *x, sc_u32 n,
			 sc_u32 gap_max, sc_u64 isize, sc_u64 *dst_bytes, sc_u64 *read_bytes);

/* ---- bus addresses + PRPs ---------------------------------------------------- */
/* A dma-buf sg table flattened once at attach: segment k covers bytes
 * [start[k], start[k] + len[k]) of the buffer at bus address addr[k].
 * `hint` remembers the last segment found, so the sequential lookups of a
 * request cost O(1) instead of a walk from the first entry. */
struct strom_sgmap {
	sc_u32 nsegs;
	const sc_u64 *addr;
	const sc_u64 *len;
	const sc_u64 *start;
	sc_u32 hint;
};

/* Bus address of byte `off` and how many bytes follow contiguously. */
int strom_core_sg_lookup(struct strom_sgmap *m, sc_u64 off, sc_u64 *addr, sc_u64 *contig);

/* Bus address of the NVMe page at byte `off` of the destination (4 KiB
 * aligned, contiguous for 4 KiB or to the end of the request). */
typedef int (*strom_page_addr_fn)(void *ctx, sc_u64 off, sc_u32 need, sc_u64 *addr);
int strom_core_sg_page_addr(void *sgmap, sc_u64 off, sc_u32 need, sc_u64 *addr);

struct strom_prps {
	sc_u64 prp1, prp2;
	sc_u32 nlist;            /* entries written to the list page */
	bool uses_list;          /* prp2 is the list page's bus address */
};

/* Fill PRP1/PRP2 (+ list) for `len` bytes starting at destination byte
 * `off`.  off must be 4 KiB aligned (PRP2 and every list entry must be page
 * aligned, and a request that starts mid-page would need PRP1 offsets the
 * destination pages do not have), every page address 4 KiB aligned.  `list`
 * (cap entries) is written only when more than two pages are needed; its
 * bus address `list_dma` becomes PRP2.  -EINVAL misaligned or
 * discontiguous, -E2BIG more pages than the list holds. */
int strom_core_build_prps(strom_page_addr_fn page_addr, void *ctx, sc_u64 off, sc_u32 len,
			  sc_u64 *list, sc_u32 cap, sc_u64 list_dma, struct strom_prps *out);

/* NVMe READ fields for a merged request: starting LBA and 0-based block
 * count.  -EINVAL when the range is not LBA aligned or longer than 65536
 * blocks. */
int strom_core_nvme_rw(sc_u64 sect, sc_u32 len, sc_u32 lba_shift, sc_u64 *slba,
		       sc_u32 *nlb0);

/* Destination window check for SSD2GPU against a registered range:
 * -ERANGE when [offset, offset + bytes) leaves [0, length) (overflow-safe),
 * -EINVAL when base_off + offset is not 4 KiB aligned (PRP rule above). */
int strom_core_check_range(sc_u64 length, sc_u64 offset, sc_u64 bytes);
int strom_core_check_dest(sc_u64 length, sc_u64 base_off, sc_u64 offset, sc_u64 bytes);

#ifdef __cplusplus
}
#endif
#endif /* STROM_CORE_H */
