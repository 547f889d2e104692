// SPDX-License-Identifier: GPL-2.0
/*
 * strom_core.c — kernel-free planner, raid0 remap and PRP builder shared by
 * the kernel module and the userspace engine (see strom_core.h).
 */
#include "strom_core.h"

#define SC_MIN(a, b) ((a) < (b) ? (a) : (b))

/* ---- chunk position + landing ------------------------------------------------ */
int strom_core_chunk_fpos(sc_u32 cid, sc_u32 chunk_sz, sc_u32 relseg_sz, sc_u64 isize,
			  sc_u64 *fpos)
{
	const sc_u64 c = relseg_sz ? (sc_u64)(cid % relseg_sz) : (sc_u64)cid;

	*fpos = c * (sc_u64)chunk_sz;
	return *fpos >= isize ? -ERANGE : 0;
}

sc_u32 strom_core_land(struct strom_landing *l, sc_u32 i, bool cached)
{
	if (cached) {
		l->nr_ram++;
		return l->reorder ? l->nr_chunks - l->nr_ram : i;
	}
	return l->reorder ? l->nr_ssd++ : (l->nr_ssd++, i);
}

/* ---- raid0 ------------------------------------------------------------------------ */
int strom_core_raid0_check(const struct strom_raid0 *g)
{
	sc_u64 prev = 0;
	sc_u32 z, k;

	if (!g->chunk_sects || (g->chunk_sects & 7) || !g->nzones ||
	    g->nzones > STROM_RAID0_MAX_ZONES || !g->ndisks || g->ndisks > STROM_RAID0_MAX_DISKS)
		return -EINVAL;
	for (z = 0; z < g->nzones; z++) {
		const sc_u32 nb = g->zone_nb_dev[z];

		if (!nb || nb > g->ndisks || g->zone_end[z] <= prev)
			return -EINVAL;
		/* a zone is whole stripes: nb members x chunk */
		if ((g->zone_end[z] - prev) % ((sc_u64)nb * g->chunk_sects))
			return -EINVAL;
		for (k = 0; k < nb; k++)
			if (g->zone_devs[z][k] >= g->ndisks)
				return -EINVAL;
		prev = g->zone_end[z];
	}
	return 0;
}

int strom_core_raid0_map(const struct strom_raid0 *g, sc_u64 sector, sc_u32 nr, int *member,
			 sc_u64 *msector)
{
	sc_u64 zstart = 0, off, chunk_no, row, in_chunk;
	sc_u32 z, nb;

	if (!g->chunk_sects || !g->nzones)
		return -EINVAL;
	for (z = 0; z < g->nzones && sector >= g->zone_end[z]; z++)
		zstart = g->zone_end[z];
	if (z == g->nzones)
		return -ERANGE;
	in_chunk = sector % g->chunk_sects;
	if (in_chunk + nr > g->chunk_sects)
		return -ESPIPE;      /* the request straddles a stripe chunk */
	if (sector + nr > g->zone_end[z])
		return -ERANGE;
	nb = g->zone_nb_dev[z];
	off = sector - zstart;
	chunk_no = off / g->chunk_sects;     /* chunk index inside the zone */
	row = chunk_no / nb;
	*member = g->zone_devs[z][chunk_no % nb];
	*msector = g->zone_dev_start[z] + row * g->chunk_sects + in_chunk +
		   g->data_offset[*member];
	return 0;
}

/* ---- planner ---------------------------------------------------------------------- */
void strom_core_planner_init(struct strom_planner *p)
{
	if (!p->max_req || (p->prp_limited && p->max_req > STROM_CORE_MAX_REQ))
		p->max_req = STROM_CORE_MAX_REQ;
	p->max_req &= ~(STROM_CORE_PAGE - 1);
	if (p->max_req < STROM_CORE_PAGE)
		p->max_req = STROM_CORE_PAGE;
	if (p->blkbits < 9 || p->blkbits > STROM_CORE_PAGE_SHIFT)
		p->blkbits = STROM_CORE_PAGE_SHIFT;
	p->cur.len = 0;
	p->nr_submit = 0;
	p->nr_sectors = 0;
}

int strom_core_plan_flush(struct strom_planner *p)
{
	int rc;

	if (!p->cur.len)
		return 0;
	rc = p->submit(p->submit_ctx, &p->cur);
	p->nr_submit++;
	p->nr_sectors += p->cur.len >> 9;
	p->cur.len = 0;
	return rc;
}

/* device sector of the 4 KiB file page at fpos: every fs block of the page
 * must map, and map contiguously */
static int page_sector(struct strom_planner *p, sc_u64 fpos, sc_u64 *sect)
{
	const sc_u32 per = 1u << (STROM_CORE_PAGE_SHIFT - p->blkbits);
	const sc_u64 fblk = fpos >> p->blkbits;
	sc_u64 first = 0;
	sc_u32 k;

	for (k = 0; k < per; k++) {
		sc_u64 d = 0;
		int rc = p->bmap(p->bmap_ctx, fblk + k, &d);

		if (rc)
			return rc;
		if (k == 0)
			first = d;
		else if (d != first + k)
			return -EOPNOTSUPP;          /* page split on the device */
	}
	*sect = (first << (p->blkbits - 9)) + p->part_start_sect;
	return 0;
}

int strom_core_plan_range(struct strom_planner *p, sc_u64 fpos, sc_u32 len, sc_u64 dest)
{
	sc_u32 off;
	int rc;

	if ((fpos | len | dest) & (STROM_CORE_PAGE - 1))
		return -EINVAL;
	for (off = 0; off < len; off += STROM_CORE_PAGE) {
		const sc_u64 d = dest + off;
		sc_u64 sect;
		int member = -1;
		bool seg_ok = true;

		rc = page_sector(p, fpos + off, &sect);
		if (rc)
			return rc;
		if (p->raid0) {
			sc_u64 msect;

			rc = strom_core_raid0_map(p->raid0, sect, STROM_CORE_PAGE >> 9, &member, &msect);
			if (rc)
				return rc;
			sect = msect;
		}
		if (p->dest_segment && p->cur.len)
			seg_ok = p->cur.dest / p->dest_segment ==
				 (d + STROM_CORE_PAGE - 1) / p->dest_segment;
		if (p->cur.len && p->cur.member == member &&
		    p->cur.sect + (p->cur.len >> 9) == sect && p->cur.dest + p->cur.len == d &&
		    p->cur.len + STROM_CORE_PAGE <= p->max_req && seg_ok &&
		    (!p->file_contig || p->cur.file_off + p->cur.len == fpos + off)) {
			p->cur.len += STROM_CORE_PAGE;
			continue;
		}
		rc = strom_core_plan_flush(p);
		if (rc)
			return rc;
		p->cur.file_off = fpos + off;
		p->cur.sect = sect;
		p->cur.dest = d;
		p->cur.len = STROM_CORE_PAGE;
		p->cur.member = member;
	}
	return 0;
}

/* ---- exact extent reads -------------------------------------------------------------- */
/* one run [a, b) at destination d: the pages before EOF, in planner pieces
 * that fit plan_range's 32-bit length */
static int xfer_run(struct strom_planner *p, sc_u64 a, sc_u64 b, sc_u64 d, sc_u64 isize,
		    sc_u64 *read_bytes)
{
	const sc_u64 eof = (isize + STROM_CORE_PAGE - 1) & ~(sc_u64)(STROM_CORE_PAGE - 1);
	const sc_u64 end = b < eof ? b : eof;
	sc_u64 o;
	int rc;

	if (end <= a)
		return 0;
	*read_bytes += end - a;
	for (o = a; p && o < end; o += 1u << 30) {
		const sc_u64 piece = end - o < (1u << 30) ? end - o : (1u << 30);

		rc = strom_core_plan_range(p, o, (sc_u32)piece, d + (o - a));
		if (rc)
			return rc;
	}
	return 0;
}

int strom_core_plan_xfer(struct strom_planner *p, struct strom_xfer_extent *x, sc_u32 n,
			 sc_u32 gap_max, sc_u64 isize, sc_u64 *dst_bytes, sc_u64 *read_bytes)
{
	const sc_u64 mask = STROM_CORE_PAGE - 1;
	sc_u64 run_a = 0, run_b = 0, run_d = 0, d = 0, prev_end = 0;
	bool open = false;
	sc_u32 i;
	int rc;

	*dst_bytes = *read_bytes = 0;
	if (n && !x)
		return -EINVAL;
	for (i = 0; i < n; i++) {
		const sc_u64 o = x[i].file_off, e = o + x[i].len;
		sc_u64 a, b;

		if (!x[i].len) {                     /* nothing to read */
			x[i].dst_off = 0;
			continue;
		}
		if (e < o || e > isize)
			return -ERANGE;
		if (o < prev_end)
			return -EINVAL;              /* sorted and disjoint */
		prev_end = e;
		a = o & ~mask;
		b = (e + mask) & ~mask;
		if (open && a <= run_b + gap_max) {
			if (b > run_b)
				run_b = b;           /* sorted: a >= run_a */
		} else {
			if (open) {
				rc = xfer_run(p, run_a, run_b, run_d, isize, read_bytes);
				if (rc)
					return rc;
				d = run_d + (run_b - run_a);
			}
			run_a = a;
			run_b = b;
			run_d = d;
			open = true;
		}
		x[i].dst_off = run_d + (o - run_a);
	}
	if (open) {
		rc = xfer_run(p, run_a, run_b, run_d, isize, read_bytes);
		if (rc)
			return rc;
		d = run_d + (run_b - run_a);
	}
	*dst_bytes = d;
	return 0;
}

/* ---- bus addresses + PRPs ----------------------------------------------------------- */
int strom_core_sg_lookup(struct strom_sgmap *m, sc_u64 off, sc_u64 *addr, sc_u64 *contig)
{
	sc_u32 lo = 0, hi = m->nsegs, k = m->hint;

	if (!m->nsegs)
		return -ERANGE;
	/* sequential access: the hinted segment or the next one */
	if (k < m->nsegs && off >= m->start[k] && off - m->start[k] < m->len[k])
		goto found;
	if (k + 1 < m->nsegs && off >= m->start[k + 1] && off - m->start[k + 1] < m->len[k + 1]) {
		k++;
		goto found;
	}
	while (lo < hi) {                       /* first segment with start > off */
		const sc_u32 mid = lo + (hi - lo) / 2;

		if (m->start[mid] <= off)
			lo = mid + 1;
		else
			hi = mid;
	}
	if (!lo)
		return -ERANGE;
	k = lo - 1;
	if (off - m->start[k] >= m->len[k])
		return -ERANGE;
found:
	m->hint = k;
	*addr = m->addr[k] + (off - m->start[k]);
	*contig = m->len[k] - (off - m->start[k]);
	return 0;
}

int strom_core_sg_page_addr(void *sgmap, sc_u64 off, sc_u32 need, sc_u64 *addr)
{
	sc_u64 contig = 0;
	int rc = strom_core_sg_lookup((struct strom_sgmap *)sgmap, off, addr, &contig);

	if (rc)
		return rc;
	return contig < need ? -EINVAL : 0;
}

int strom_core_build_prps(strom_page_addr_fn page_addr, void *ctx, sc_u64 off, sc_u32 len,
			  sc_u64 *list, sc_u32 cap, sc_u64 list_dma, struct strom_prps *out)
{
	const sc_u32 npages = (len + STROM_CORE_PAGE - 1) >> STROM_CORE_PAGE_SHIFT;
	sc_u32 i;
	sc_u64 a;
	int rc;

	out->prp1 = out->prp2 = 0;
	out->nlist = 0;
	out->uses_list = false;
	if (!len || (off & (STROM_CORE_PAGE - 1)))
		return -EINVAL;
	if (npages > 2 && npages - 1 > cap)
		return -E2BIG;
	for (i = 0; i < npages; i++) {
		const sc_u32 need = SC_MIN(STROM_CORE_PAGE, len - i * STROM_CORE_PAGE);

		rc = page_addr(ctx, off + (sc_u64)i * STROM_CORE_PAGE, need, &a);
		if (rc)
			return rc;
		if (a & (STROM_CORE_PAGE - 1))
			return -EINVAL;
		if (i == 0)
			out->prp1 = a;
		else if (npages == 2)
			out->prp2 = a;
		else
			list[out->nlist++] = a;
	}
	if (npages > 2) {
		out->prp2 = list_dma;
		out->uses_list = true;
	}
	return 0;
}

int strom_core_nvme_rw(sc_u64 sect, sc_u32 len, sc_u32 lba_shift, sc_u64 *slba, sc_u32 *nlb0)
{
	const sc_u32 sh = lba_shift >= 9 ? lba_shift - 9 : 0;
	sc_u64 nlb;

	if (lba_shift < 9 || lba_shift > 16 || !len)
		return -EINVAL;
	if ((sect & ((1u << sh) - 1)) || (len & ((1u << lba_shift) - 1)))
		return -EINVAL;
	nlb = len >> lba_shift;
	if (nlb > 0x10000)
		return -EINVAL;
	*slba = sect >> sh;
	*nlb0 = (sc_u32)(nlb - 1);
	return 0;
}

int strom_core_check_range(sc_u64 length, sc_u64 offset, sc_u64 bytes)
{
	/* offset + bytes <= length, without the sum (it can wrap) */
	if (offset > length || bytes > length - offset)
		return -ERANGE;
	return 0;
}

int strom_core_check_dest(sc_u64 length, sc_u64 base_off, sc_u64 offset, sc_u64 bytes)
{
	if (strom_core_check_range(length, offset, bytes))
		return -ERANGE;
	if ((base_off + offset) & (STROM_CORE_PAGE - 1))
		return -EINVAL;
	return 0;
}
