"""Randomized HeapTupleSatisfiesMVCC fixtures shared by the host and device
tests: commit log, pg_subtrans and pg_multixact windows straddling the 2^32
wrap, snapshots (plain and suboverflowed, with the scanning transaction's
own xids and command id), and heap pages of tuples with random headers —
hint bits, multixact xmax, own xids, command ids, combo cids."""
import struct

import numpy as np

from nvme_strom_amd.utils import pgmvcc, pgpage
from nvme_strom_amd.utils.pgmvcc import (HEAP_COMBOCID, HEAP_XMAX_EXCL_LOCK, HEAP_XMAX_INVALID,
                                         HEAP_XMAX_IS_MULTI, HEAP_XMAX_LOCK_ONLY,
                                         HEAP_XMIN_COMMITTED, HEAP_XMIN_INVALID, CommitLog,
                                         MultiXact, Snapshot, SubTrans, XACT_ABORTED,
                                         XACT_COMMITTED, XACT_IN_PROGRESS, XACT_SUBCOMMITTED)

W = 1 << 32
HEAP_XMAX_COMMITTED = 0x0400


def header(xmin, xmax, mask, cid=0):
    return struct.pack("<IIIHHHHHB", xmin % W, xmax % W, cid, 0, 0, 0, 1, mask, 24)


def tuple_of(xmin, xmax, mask, cid, payload):
    return header(xmin, xmax, mask, cid) + b"\0" + payload


class World:
    """One randomized set of SLRU windows and a list of snapshots over it."""

    def __init__(self, seed=77, n=6000, wrap=True):
        rng = np.random.default_rng(seed)
        self.rng = rng
        base = (W - n // 2) if wrap else 100
        self.clog = CommitLog(n, base=base)
        self.sub = SubTrans(n, base=base)
        self.xs = [(base + i) % W for i in range(3, n)]
        for x in self.xs:
            st = int(rng.choice([XACT_COMMITTED] * 4 + [XACT_ABORTED, XACT_IN_PROGRESS,
                                                         XACT_SUBCOMMITTED]))
            self.clog.set(x, st)
            if st == XACT_SUBCOMMITTED or rng.random() < 0.2:
                self.sub.set(x, (x - int(rng.integers(1, 40))) % W)
        self.mx = MultiXact(base=(W - 20) if wrap else 10)
        self.multis = [self.mx.add([(int(rng.choice(self.xs)), int(rng.integers(0, 6)))
                                    for _ in range(int(rng.integers(1, 4)))]) for _ in range(60)]
        self.base = base
        self.n = n

    def pick(self):
        return int(self.rng.choice(self.xs))

    def snapshot(self, trial):
        rng = self.rng
        xmin = (self.base + int(rng.integers(self.n // 6, self.n // 2))) % W
        xmax = (xmin + int(rng.integers(10, self.n // 2))) % W
        xip = sorted({(xmin + int(rng.integers(0, 10))) % W for _ in range(int(rng.integers(0, 40)))})
        return Snapshot(xmin=xmin, xmax=xmax, xip=xip,
                        subxip=[self.pick() for _ in range(int(rng.integers(0, 12)))],
                        suboverflowed=bool(trial % 2),
                        curxids=[self.pick() for _ in range(int(rng.integers(0, 4)))],
                        curcid=int(rng.integers(0, 10)))

    def random_case(self, snap):
        rng = self.rng
        ismulti = rng.random() < 0.2
        xmax = int(rng.choice(self.multis)) if ismulti else int(rng.choice([0] + self.xs))
        mask = int(rng.choice([0, HEAP_XMIN_COMMITTED, HEAP_XMIN_INVALID,
                               HEAP_XMIN_COMMITTED | HEAP_XMIN_INVALID]))
        mask |= int(rng.choice([0, HEAP_XMAX_INVALID, HEAP_XMAX_COMMITTED, HEAP_XMAX_LOCK_ONLY,
                                HEAP_XMAX_EXCL_LOCK]))
        mask |= HEAP_XMAX_IS_MULTI if ismulti else 0
        mask |= HEAP_COMBOCID if rng.random() < 0.05 else 0
        cur = list(snap.curxids)
        xmin = int(rng.choice(cur)) if cur and rng.random() < 0.15 else self.pick()
        if cur and not ismulti and rng.random() < 0.1:
            xmax = int(rng.choice(cur))
        return xmin, xmax, mask, int(rng.integers(0, 10))

    def pages(self, snap, npages, per_page=200, all_visible_every=0):
        """(page bytes, cases per page); page p is PD_ALL_VISIBLE when
        all_visible_every divides p (its tuples then all count as visible)."""
        out, cases = [], []
        for p in range(npages):
            cs = [self.random_case(snap) for _ in range(per_page)]
            tuples = [tuple_of(a, b, m, c, struct.pack("<q", p * 1000 + i))
                      for i, (a, b, m, c) in enumerate(cs)]
            av = bool(all_visible_every) and p % all_visible_every == 0
            out.append(pgpage.build_page(tuples, blkno=p, all_visible=av))
            cases.append(cs)
        return b"".join(out), cases

    def expect(self, snap, cases, checked):
        """Per page: the (kept line numbers, removed count, recheck flag) the
        native check gives — undecided tuples are kept, their page flagged."""
        out = []
        for cs, chk in zip(cases, checked):
            if not chk:
                out.append(([i + 1 for i in range(len(cs))], 0, False))
                continue
            keep, removed, rc = [], 0, False
            for i, (a, b, m, c) in enumerate(cs):
                v = pgmvcc.native_visible(header(a, b, m, c), snap, self.clog, self.sub, self.mx)
                if v is False:
                    removed += 1
                else:
                    keep.append(i + 1)
                    rc |= v is None
            out.append((keep, removed, rc))
        return out
