"""Tuple builder / deformer (utils.pgtuple) against PostgreSQL's on-disk rules."""
import collections
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


# ---- qualifier programs: numeric, CNF, constants of any size
def test_numeric_roundtrip_and_order():
    """numeric's on-disk form (NumericShort / NumericLong / specials) round-
    trips through the tuple deformer, and the order is PostgreSQL's
    (-inf < finite < +inf < NaN, NaN = NaN)."""
    import decimal
    D = decimal.Decimal
    desc = T.TupleDesc.of([("v", "numeric")])
    vals = [D("0"), D("1"), D("-1"), D("12345.678"), D("-0.00005"), D("1e-300"), D("NaN"),
            D("Infinity"), D("-Infinity"), D("123456789012345678901234567890.123456789"),
            D("99999999999999999999.5")]
    for v in vals:
        got = T.deform(T.heap_tuple([v], desc), desc)[0]
        assert (got.is_nan() and v.is_nan()) or got == v, (v, got)
    keys = sorted(vals, key=T.numeric_key)
    assert keys[0] == D("-Infinity") and keys[-1].is_nan() and keys[-2] == D("Infinity")


def test_program_compiles_cnf_and_exact_int_bounds():
    """Quals -> program: one clause per Qual / Or, constants in the pool;
    int bounds exact (a fractional lower bound rounds up, an upper one down,
    a fractional equality selects nothing, bounds clamp to the type) —
    ADVICE r4: the host twin and the device agree."""
    import ctypes as C
    from nvme_strom_amd.ops import heapscan as H
    desc, _ = heapgen.numeric_rel(10)
    qs = [T.Qual("x", "between", (1.5, 3)), T.Or(T.Qual("s", "eq", (2.5,)), T.Qual("x", "lt", (10**30,))),
          T.Qual("tag", "text_in", (["a" * 100, "b"],)), T.Qual("amt", "ge", (3,))]
    p = H.Program(desc, qs)
    cl = [q.clause for q in p.quals]
    assert cl == sorted(cl) and sorted(collections.Counter(cl).values()) == [1, 1, 1, 2]
    # clauses by first attribute (amt, tag, x, x|s), quals by attribute inside
    assert [q.attno for q in p.quals] == [1, 2, 3, 3, 6]
    x_between, x_lt, s_eq = p.quals[2], p.quals[3], p.quals[4]
    assert x_between.clause != x_lt.clause == s_eq.clause
    assert (x_between.lo, x_between.hi) == (2, 3)
    assert s_eq.flags & H.QUAL2_FALSE                         # s == 2.5: never
    assert x_lt.hi == (1 << 63) - 1                          # clamped to int8
    raw, pool = p.arrays()
    hp = np.frombuffer(raw, np.uint8)
    d = H.tupdesc_struct(desc)
    chk = H.lib().strom_heap_prog_check
    assert len(pool) % 8 == 0
    assert chk(C.byref(d), hp.ctypes.data, len(p.quals), pool, len(pool)) == 0
    assert chk(C.byref(d), hp.ctypes.data, len(p.quals), pool, 8) < 0
    assert chk(C.byref(d), hp.ctypes.data, len(p.quals), pool, len(pool) - 4) < 0   # unpadded
    # a text IN entry naming bytes past the pool's end
    tin = next(q for q in p.quals if q.kind == H.QUAL_TEXT_IN)
    bad = bytearray(pool)
    struct.pack_into("<I", bad, tin.coff + 4, len(pool) + 1)
    assert chk(C.byref(d), hp.ctypes.data, len(p.quals), bytes(bad), len(pool)) < 0
    # a numeric constant whose digit count runs past the pool's end
    pn = H.Program(desc, [T.Qual("amt", "ge", (3,))])
    raw2, pool2 = pn.arrays()
    h2 = np.frombuffer(raw2, np.uint8)
    assert chk(C.byref(d), h2.ctypes.data, 1, pool2, len(pool2)) == 0
    bad = bytearray(pool2)
    struct.pack_into("<H", bad, pn.quals[0].lo + 6, 999)
    assert chk(C.byref(d), h2.ctypes.data, 1, bytes(bad), len(pool2)) < 0
    # the host twin on the same fractional bounds
    assert T.Qual("x", "between", (1.5, 3)).test(1, "int") is False
    assert T.Qual("s", "eq", (2.5,)).test(2, "int") is False


def _brute(rows, desc, qs):
    """Independent CNF evaluation straight from the Python row values."""
    out = []
    for i, r in enumerate(rows):
        verdict = True
        for cl in T.clauses(qs):
            cv = False
            for q in cl:
                k = desc.attno(q.col)
                v = r[k]
                v = T.EXT if isinstance(v, (T.Toast, T.Compressed)) else (
                    T._b(v) if desc.kinds[k] == "text" and v is not None else v)
                t = q.test(v, desc.kinds[k])
                if t is True:
                    cv = True
                    break
                if t is None:
                    cv = None
            if cv is False:
                verdict = False
                break
            if cv is None:
                verdict = None
        out.append(verdict)
    return out


def test_host_scan2_cnf_matches_brute_force():
    """The host twin's CNF over deformed tuples equals a brute-force
    evaluation of the same quals over the Python row values (numeric,
    text IN / long constants, NULLs, TOAST / compressed -> undecidable)."""
    desc, rows = heapgen.numeric_rel(1500, seed=3)
    data = T.build_pages(rows, desc)
    rng = np.random.default_rng(8)
    for _ in range(25):
        qs = heapgen.random_cnf(rng, int(rng.integers(1, 12)))
        items, status, _ = T.host_scan2(data, desc, qs)
        want = _brute(rows, desc, qs)
        # rows -> (page, lineno) in insertion order
        ids, pg, ln, used = [], 0, 0, 24
        for r in rows:
            t = T.heap_tuple(r, desc)
            need = ((len(t) + 7) & ~7) + 4
            if ln and used + need > 8192:
                pg, ln, used = pg + 1, 0, 24
            ln += 1
            used += need
            ids.append((pg << 16) | ln)
        assert items == [i for i, w in zip(ids, want) if w is True]
        rech = {i >> 16 for i, w in zip(ids, want) if w is None}
        assert {p for p, s in enumerate(status) if s & T.PAGE_RECHECK} == rech


def test_program_rejects_kind_mismatches():
    """A qual whose op does not fit its column's type is refused at compile
    time (the device never sees it)."""
    from nvme_strom_amd.ops import heapscan as H
    desc, _ = heapgen.numeric_rel(4)
    for q in (T.Qual("amt", "prefix", ("1",)), T.Qual("tag", "between", (1, 2)),
              T.Qual("x", "text_eq", ("a",)), T.Qual("f", "text_in", (["a"],)),
              T.Qual("amt", "frobnicate", (1,))):
        with pytest.raises(ValueError):
            H.Program(desc, [q])
    # an empty IN is constant false, also under an Or
    p = H.Program(desc, [T.Or(T.Qual("amt", "in", ([],)), T.Qual("x", "in", ([],)))])
    assert all(q.flags & H.QUAL2_FALSE for q in p.quals)


def test_program_fixed_form():
    """A plain AND list of the fixed form's kinds goes in the kernel
    arguments (sorted by attribute, constants copied out of the pool); an OR,
    a numeric range, a constant-false qual, a long text constant or more than
    HEAP_MAX_QUALS quals keep the program mode."""
    import ctypes as C
    from nvme_strom_amd import _native as N
    from nvme_strom_amd.ops import heapscan as H
    desc, _ = heapgen.numeric_rel(4)
    fx = H.Program(desc, [T.Qual("x", "in", ([3, 1, 2],)), T.Qual("tag", "text_eq", ("abc",)),
                          T.Qual("f", "between", (0.5, 1.5))]).fixed()
    assert fx is not None and [q.attno for q in fx] == sorted(q.attno for q in fx)
    kinds = {q.kind: q for q in fx}
    assert set(kinds) == {2, 5, 7}
    assert kinds[7].nconst == 3 and bytes(kinds[7].cbytes)[:24] == struct.pack("<3q", 1, 2, 3)
    assert kinds[5].nconst == 3 and bytes(kinds[5].cbytes)[:3] == b"abc"
    assert C.sizeof(N.HeapQual) == 56
    for qs in ([T.Or(T.Qual("x", "eq", (1,)), T.Qual("s", "eq", (2,)))],
               [T.Qual("amt", "ge", (3,))],
               [T.Qual("s", "eq", (2.5,))],
               [T.Qual("tag", "text_eq", ("a" * 33,))],
               [T.Qual("x", "in", (list(range(5)),))],
               [T.Qual("x", "ge", (i,)) for i in range(N.HEAP_MAX_QUALS + 1)]):
        assert H.Program(desc, qs).fixed() is None, qs


def test_program_non_finite_int_constants():
    """inf / -inf / NaN constants against an int column compile
    to the range they mean (the type's limits, or a constant-false qual)
    instead of raising; IN lists drop them.  The host twin agrees."""
    from nvme_strom_amd.ops.heapscan import QUAL2_FALSE, Program
    from nvme_strom_amd.utils import pgtuple as T
    desc = T.TupleDesc.of([("a", "int4")])
    inf, nan = float("inf"), float("nan")
    lim = (-(1 << 31), (1 << 31) - 1)

    def one(q):
        p = Program(desc, [q])
        assert len(p.quals) == 1
        x = p.quals[0]
        return None if x.flags & QUAL2_FALSE else (x.kind, x.lo, x.hi, x.nconst)
    assert one(T.Qual("a", "lt", (inf,))) == (1, lim[0], lim[1], 0)
    assert one(T.Qual("a", "le", (-inf,))) is None
    assert one(T.Qual("a", "gt", (-inf,))) == (1, lim[0], lim[1], 0)
    assert one(T.Qual("a", "ge", (inf,))) is None
    assert one(T.Qual("a", "between", (-inf, 5.5))) == (1, lim[0], 5, 0)
    assert one(T.Qual("a", "between", (nan, 5))) is None
    assert one(T.Qual("a", "eq", (nan,))) is None
    assert one(T.Qual("a", "eq", (inf,))) is None
    assert one(T.Qual("a", "in", ([nan, inf, 3, 4.0, 4.5],))) == (7, 0, 0, 2)
    # the host evaluation of the same quals over a few values
    rows = [(v,) for v in (lim[0], -7, 0, 5, lim[1])]
    data = T.build_pages(rows, desc)
    for q, want in ((T.Qual("a", "lt", (inf,)), 5), (T.Qual("a", "le", (-inf,)), 0),
                    (T.Qual("a", "between", (-inf, 5.5)), 4), (T.Qual("a", "eq", (nan,)), 0)):
        items, _, _ = T.host_scan2(data, desc, [q])
        assert len(items) == want, (q, items)
