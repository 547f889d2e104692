"""Tuple builder / deformer (utils.pgtuple) against PostgreSQL's on-disk rules."""
import struct

import numpy as np

import pytest

from nvme_strom_amd.utils import pgpage
from nvme_strom_amd.utils import pgtuple as T

import heapgen


def test_layout_by_hand():
    d = T.TupleDesc.of([("a", "int2"), ("b", "int8"), ("t", "text"), ("c", "int4")])
    t = T.heap_tuple([7, None, "hi", 9], d)
    infomask2, infomask, hoff = struct.unpack_from("<HHB", t, 18)
    assert infomask2 == 4 and infomask & T.HEAP_HASNULL
    assert t[23] == 0b1101 and hoff == 24            # bitmap: a, t, c present
    assert struct.unpack_from("<h", t, 24)[0] == 7
    # b is NULL (no storage); "hi" gets a 1-byte header right after a, unaligned
    assert t[26] == ((2 + 1) << 1) | 1 and t[27:29] == b"hi"
    # c is int4: aligned to 4 after the short varlena
    assert struct.unpack_from("<i", t, 32)[0] == 9 and len(t) == 36
    assert T.deform(t, d) == [7, None, b"hi", 9]


def test_long_varlena_is_aligned_4byte():
    d = T.TupleDesc.of([("x", "bool"), ("t", "text")])
    t = T.heap_tuple([1, "y" * 200], d)
    hoff = t[22]
    assert t[hoff] == 1 and t[hoff + 1:hoff + 4] == b"\0\0\0"   # pad to 4
    assert struct.unpack_from("<I", t, hoff + 4)[0] >> 2 == 204
    assert T.deform(t, d) == [1, b"y" * 200]


def test_toast_compressed_and_missing_attributes():
    d = T.TupleDesc.of([("t", "text"), ("u", "text"), ("v", "int4"), ("w", "int8")])
    t = T.heap_tuple([T.Toast(5), T.Compressed(), 3, 4], d, natts=3)
    assert T.deform(t, d) == [T.EXT, T.EXT, 3, None]
    assert d.cacheoff() == [-1, -1, -1, -1]
    assert T.TupleDesc.of([("a", "int2"), ("b", "int8"), ("t", "text")]).cacheoff() == [0, 8, -1]


def test_host_scan2_matches_row_model():
    rows = heapgen.rows(700, seed=3)
    data = T.build_pages(rows, heapgen.DESC, natts_of=heapgen.natts_of)
    for qs in heapgen.QUAL_SETS:
        items, status, proj = T.host_scan2(data, heapgen.DESC, qs, project="a")
        assert all(s & ~T.PAGE_RECHECK == 0 for s in status)
        # every item's row passes every qual (rows are packed in order)
        got = []
        per_page = {}
        for it in items:
            per_page.setdefault(it >> 16, []).append(it & 0xFFFF)
        assert len(items) == len(proj)
        n_pages = len(data) // 8192
        # rebuild row ids: count tuples per page
        row0, ids = 0, []
        for pg in range(n_pages):
            lower = struct.unpack_from("<H", data, pg * 8192 + 12)[0]
            nt = (lower - 24) // 4
            ids += [((pg << 16) | (j + 1), row0 + j) for j in range(nt)]
            row0 += nt
        rowof = dict(ids)
        for it in items:
            r = list(rows[rowof[it]])
            if heapgen.natts_of(rowof[it]) < 10:
                r[8:] = [None, None]
            for q in qs:
                k = heapgen.DESC.attno(q.col)
                v = r[k]
                if isinstance(v, str):
                    v = v.encode()
                elif isinstance(v, (T.Toast, T.Compressed)):
                    v = T.EXT
                assert q.test(v, heapgen.DESC.kinds[k]) is not False
        assert items == sorted(items)


def test_qual_struct_packing():
    pytest.importorskip("torch")
    from nvme_strom_amd.ops import heapscan as H
    qs = H.qual_structs(heapgen.DESC, heapgen.QUAL_SETS[5])
    assert [q.attno for q in qs] == [7, 8, 9]
    assert [q.kind for q in qs] == [4, 2, 1]
    with pytest.raises(ValueError):
        H.qual_structs(heapgen.DESC, [T.Qual("name", "between", (1, 2))])


def test_cpu_scan_with_qualifier_list(strom, tmp_path):
    """The reference-shaped host scan (SSD2RAM + host deformer) with a
    qualifier list and a projection equals host_scan2 over the same bytes,
    across segment files and chunks."""
    from nvme_strom_amd.models import pg_scan
    rows = heapgen.rows(3000, seed=5)
    data = T.build_pages(rows, heapgen.DESC, natts_of=heapgen.natts_of)
    rel = pg_scan.Relation.write(str(tmp_path / "24600"), data, relseg_size=16)
    cfg = pg_scan.ScanConfig(chunk_size=4 * 8192, buffer_size=16 * 8192)
    for qs, proj in ((heapgen.QUAL_SETS[1], "b"), (heapgen.QUAL_SETS[3], "note")):
        r = pg_scan.cpu_scan(rel, cfg, desc=heapgen.DESC, quals=qs, project=proj)
        want, status, vals = T.host_scan2(data, heapgen.DESC, qs, project=proj)
        assert r.items.tolist() == [((i >> 16) << 16) | (i & 0xFFFF) for i in want]
        assert r.recheck_blocks == [j for j, s in enumerate(status) if s & T.PAGE_RECHECK]
        if proj == "b":
            w = np.array([np.nan if v is None else v for v in vals])
            assert np.array_equal(r.valid, np.array([v is not None for v in vals], np.uint8))
            assert np.allclose(r.values[r.valid == 1], w[~np.isnan(w)])
        else:
            assert [v if ok == 1 else None for v, ok in zip(r.values, r.valid)] == \
                [v if isinstance(v, bytes) else None for v in vals]
