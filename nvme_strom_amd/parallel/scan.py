"""Multi-GPU scans: one Arrow IPC file split over the ranks of a process
group, one process per GPU (PAR6 applied to the config-5 application).

The reference runs its scan in PostgreSQL parallel workers that share a
block cursor in DSM (pgsql/nvme_strom.c:708-780): every
worker drives the one GPU of the machine.  Here every rank owns a GPU and
its own engine, so the file is cut up front instead:

    plan:     record batches [0, nb) -> one contiguous range per rank, cut so
              every rank reads about the same number of STORED bytes of the
              referenced columns (compressed sizes from the footer walk —
              the read is the bound, not the row count)
    scan:     rank r: ArrowScan.scan_where(quals, project, batches=range_r)
              (storage -> HBM -> LZ4 decode -> qualifier bitmaps -> emit, all
              on its own GPU; row ids are file-global)
    combine:  selected counts all-gathered, then ids (+ projected values,
              validity) all-gathered padded to the largest count — RCCL over
              xGMI for device tensors, staged through the host with gloo —
              and concatenated in rank order = file order

Every rank returns the same result (``gather="all"``) or only its own part
(``gather="none"``: a consumer that keeps the data sharded, e.g. the next
operator of a distributed query).

``DistributedHeapScan`` does the same for a PostgreSQL relation, the way
the reference's parallel workers do it but with a GPU per process: every
rank's ``HeapRelationScan`` claims chunks from ONE cross-process block
cursor in shared memory (``SharedCursor``, the reference's DSM
``nsp_cblock``), so faster ranks take more chunks (dynamic balancing
instead of a static cut), and the item pointers are combined by the same
padded all-gather, then put in block order.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..models.arrow_scan import ArrowScan
from ..models import pg_scan


def partition(weights: np.ndarray, parts: int) -> List[Tuple[int, int]]:
    """Contiguous ranges of ``len(weights)`` items with about equal weight
    each (every item in exactly one range; ranges may be empty when there
    are fewer items than parts)."""
    w = np.asarray(weights, dtype=np.float64)
    n = len(w)
    if parts <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, parts - 1)
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    if total <= 0:
        cuts = [round(n * k / parts) for k in range(parts + 1)]
    else:
        targets = total * np.arange(1, parts) / parts
        # the cut after item i when cum[i + 1] first reaches the target
        inner = np.searchsorted(cum, targets, side="left").tolist()
        cuts = [0] + [min(n, max(0, c)) for c in inner] + [n]
        for k in range(1, len(cuts)):            # monotone
            cuts[k] = max(cuts[k], cuts[k - 1])
    return [(cuts[k], cuts[k + 1]) for k in range(parts)]


@dataclass
class DistScanOut:
    indices: torch.Tensor                 # selected row ids, file order
    values: Optional[torch.Tensor] = None
    valid: Optional[torch.Tensor] = None
    selected: int = 0
    per_rank: List[int] = field(default_factory=list)     # selected rows per rank
    ranges: List[Tuple[int, int]] = field(default_factory=list)
    seconds: Dict[str, float] = field(default_factory=dict)
    bytes_read: int = 0                   # this rank's storage -> HBM bytes


class DistributedArrowScan:
    """``ArrowScan`` over the ranks of ``group``: rank r scans its share of
    the record batches on its own device and the results are combined with
    collectives (see module docstring)."""

    def __init__(self, path: str, device: torch.device, group=None, **scan_kw):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.device = torch.device(device)
        self.scan = ArrowScan(path, self.device, **scan_kw)
        backend = dist.get_backend(group) if self.world > 1 else None
        # gloo cannot run collectives on device memory: stage through the host
        self.staged = self.device.type == "cuda" and backend == "gloo"
        self._cdev = torch.device("cpu") if (self.staged or self.device.type != "cuda") \
            else self.device
        self._ranges: Dict[tuple, List[Tuple[int, int]]] = {}

    def ranges(self, names: Sequence[str]) -> List[Tuple[int, int]]:
        """Per-rank record-batch ranges for a scan of ``names`` (same on
        every rank: computed from the file's own metadata)."""
        key = tuple(names)
        if key not in self._ranges:
            m = self.scan.meta
            w = np.zeros(m.nbatches, dtype=np.float64)
            for n in names:
                c = m.columns[m.column_index(n)]
                w += c.d_len + np.where(c.null_count > 0, c.v_len, 0)
            self._ranges[key] = partition(w, self.world)
        return self._ranges[key]

    # ---- collectives ------------------------------------------------------
    def _all_gather(self, t: torch.Tensor) -> List[torch.Tensor]:
        """All-gather equally sized 1-D tensors; list in rank order."""
        if self.world == 1:
            return [t]
        src = t.to(self._cdev) if t.device != self._cdev else t
        out = torch.empty(self.world * src.numel(), dtype=src.dtype, device=self._cdev)
        dist.all_gather_into_tensor(out, src.contiguous(), group=self.group)
        out = out.to(t.device) if out.device != t.device else out
        return list(out.view(self.world, -1))

    def _gather_var(self, t: torch.Tensor, counts: List[int]) -> torch.Tensor:
        """All-gather tensors of per-rank length ``counts`` (padded to the
        largest), concatenated in rank order."""
        mx = max(counts) if counts else 0
        if self.world == 1 or mx == 0:
            return t[:counts[self.rank]] if counts else t
        pad = torch.zeros(mx, dtype=t.dtype, device=t.device)
        pad[:t.numel()] = t
        parts = self._all_gather(pad)
        return torch.cat([p[:c] for p, c in zip(parts, counts)])

    # ---- scan -------------------------------------------------------------
    def scan_where(self, quals: Sequence[Tuple[str, object, object]],
                   project: Optional[str] = None, gather: str = "all") -> DistScanOut:
        if gather not in ("all", "none"):
            raise ValueError(f"gather {gather!r}")
        t0 = time.perf_counter()
        names: List[str] = []
        for n in [q[0] for q in quals] + ([project] if project else []):
            if n not in names:
                names.append(n)
        rngs = self.ranges(names)
        mine = rngs[self.rank]
        out = self.scan.scan_where(quals, project, batches=mine)
        t_scan = time.perf_counter()
        cnt = torch.tensor([out.selected], dtype=torch.int64, device=self.device)
        counts = [int(x) for x in torch.cat(self._all_gather(cnt)).tolist()]
        res = DistScanOut(out.indices, out.values, out.valid, sum(counts), counts, rngs,
                          bytes_read=out.bytes_read)
        if gather == "all" and self.world > 1:
            res.indices = self._gather_var(out.indices, counts)
            if out.values is not None:
                res.values = self._gather_var(out.values, counts)
            # validity: every rank must take part in the same collectives
            has_v = torch.tensor([1 if out.valid is not None else 0], dtype=torch.int64,
                                 device=self.device)
            if int(torch.cat(self._all_gather(has_v)).max()) and out.values is not None:
                v = out.valid if out.valid is not None else \
                    torch.ones(out.selected, dtype=torch.uint8, device=self.device)
                res.valid = self._gather_var(v, counts)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t_end = time.perf_counter()
        res.seconds = {"scan_s": t_scan - t0, "combine_s": t_end - t_scan,
                       "total_s": t_end - t0, **{f"local_{k}": v for k, v in out.seconds.items()}}
        return res

    def close(self) -> None:
        self.scan.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class _Combiner:
    """Padded variable-length all-gather over a group (device tensors with
    nccl, staged through host memory with gloo)."""

    def __init__(self, device: torch.device, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        backend = dist.get_backend(group) if self.world > 1 else None
        self.cdev = device if (device.type == "cuda" and backend != "gloo") else torch.device("cpu")

    def gather(self, t: torch.Tensor) -> Tuple[torch.Tensor, List[int]]:
        if self.world == 1:
            return t, [t.numel()]
        n = torch.tensor([t.numel()], dtype=torch.int64, device=self.cdev)
        ns = torch.empty(self.world, dtype=torch.int64, device=self.cdev)
        dist.all_gather_into_tensor(ns, n, group=self.group)
        counts = [int(x) for x in ns.tolist()]
        mx = max(counts)
        if mx == 0:
            return t[:0], counts
        pad = torch.zeros(mx, dtype=t.dtype, device=self.cdev)
        pad[:t.numel()] = t.to(self.cdev)
        out = torch.empty(self.world * mx, dtype=t.dtype, device=self.cdev)
        dist.all_gather_into_tensor(out, pad, group=self.group)
        out = out.view(self.world, mx)
        return torch.cat([out[r, :c] for r, c in enumerate(counts)]), counts


class DistributedHeapScan:
    """``HeapRelationScan`` over the ranks of ``group``, one GPU per rank,
    sharing one block cursor (see module docstring).  ``run()`` is
    collective; every rank returns the full, block-ordered result."""

    def __init__(self, rel: "pg_scan.Relation", cfg: Optional["pg_scan.ScanConfig"] = None,
                 device=None, group=None, **pred):
        self.rel = rel
        self.group = group
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.scan = pg_scan.HeapRelationScan(rel, cfg, self.device, **pred)
        self.comb = _Combiner(self.device, group)

    def _cursor(self, b0: int, b1: int):
        """Rank 0 creates the shared cursor, the others attach by name."""
        name = [None]
        if self.comb.rank == 0:
            name[0] = f"dist-{os.getpid()}-{time.monotonic_ns()}"
            cur = pg_scan.SharedCursor(name[0], nblocks=b1, start=b0, create=True)
        if self.comb.world > 1:
            dist.broadcast_object_list(name, src=0, group=self.group)
            if self.comb.rank != 0:
                cur = pg_scan.SharedCursor(name[0])
        return cur

    def run(self, workers: int = 1, blocks: Optional[Tuple[int, int]] = None) -> dict:
        b0, b1 = pg_scan._block_range(blocks, self.rel.nblocks)
        t0 = time.perf_counter()
        cur = self._cursor(b0, b1)
        try:
            r = self.scan.run(workers, cursor=cur)
            cur.add(r)
            t_scan = time.perf_counter()
            if self.comb.world == 1:
                items, counts = r.items, [len(r.items)]
            else:
                mine = torch.from_numpy(r.items.view(np.int64))
                allv, counts = self.comb.gather(mine)
                # every rank's part is in block order, interleaved chunk by
                # chunk with the others': one radix sort puts them together
                items = np.sort(allv.cpu().numpy().view(np.uint64), kind="stable")
            if self.comb.world > 1:
                dist.barrier(group=self.group)   # every rank has added its counters
            totals = cur.counters()
        finally:
            cur.close(unlink=False)
        if self.comb.world > 1:
            dist.barrier(group=self.group)       # everyone detached
        if self.comb.rank == 0:
            try:
                os.unlink(cur.path)
            except FileNotFoundError:
                pass
        t_end = time.perf_counter()
        return dict(items=items, per_rank_items=counts, pages=int(r.pages), totals=totals,
                    seconds={"scan_s": t_scan - t0, "combine_s": t_end - t_scan,
                             "total_s": t_end - t0})

    def close(self) -> None:
        self.scan.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
