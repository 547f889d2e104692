"""GPU tuple deforming + qualifier lists (strom_heap_scan2 / strom_heap_project)
against the host deformer (utils.pgtuple.host_scan2): relations with NULLs
before the predicated columns, short and long text before and after them,
TOAST pointers, compressed datums and rows with fewer stored attributes."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import heapgen  # noqa: E402
from nvme_strom_amd.utils import pgtuple as T  # noqa: E402


@pytest.fixture(scope="module")
def rel():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rows = heapgen.rows(6000, seed=11)
    data = T.build_pages(rows, heapgen.DESC, natts_of=heapgen.natts_of)
    pages = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    return data, pages


@pytest.mark.parametrize("program", [False, True])
@pytest.mark.parametrize("qi", range(len(heapgen.QUAL_SETS)))
def test_scan2_matches_host(rel, qi, program):
    """Both kernels: the fixed AND list in the arguments (when the list fits
    it) and the device-memory program."""
    from nvme_strom_amd.ops import heapscan as H
    data, pages = rel
    qs = heapgen.QUAL_SETS[qi]
    want, wstatus, _ = T.host_scan2(data, heapgen.DESC, qs, verify_checksum=True)
    r = H.heap_scan2(pages, heapgen.DESC, qs, verify_checksum=True, program=program)
    got = r.sorted_items().tolist()
    assert got == want
    st = r.page_status.cpu().numpy().tolist()
    assert st == wstatus
    assert (r.recheck > 0) == any(s & T.PAGE_RECHECK for s in wstatus)


@pytest.mark.parametrize("col", ["a", "b", "name", "e", "tail"])
def test_project_matches_host(rel, col):
    from nvme_strom_amd.ops import heapscan as H
    data, pages = rel
    qs = heapgen.QUAL_SETS[1]
    want, _, wvals = T.host_scan2(data, heapgen.DESC, qs, project=col)
    r = H.heap_scan2(pages, heapgen.DESC, qs)
    cnt = torch.tensor([r.count], dtype=torch.int32, device=pages.device)
    vals, valid = H.heap_project(pages, r.items, cnt, heapgen.DESC, col, cap=r.count)
    order = torch.argsort(r.items[:r.count].to(torch.int64) & 0xFFFFFFFF)
    vals = vals[order].cpu().numpy()
    valid = valid[order].cpu().numpy()
    k = heapgen.DESC.attno(col)
    for v, ok, w in zip(vals.tolist(), valid.tolist(), wvals):
        if w is None:
            assert ok == 0
        elif w is T.EXT:
            assert ok == 2
        elif heapgen.DESC.attlen[k] == -1:
            assert ok == 1
            off, n = v >> 32, v & 0xFFFFFFFF
            assert data[off:off + n] == w
        elif heapgen.DESC.kinds[k] == "float":
            assert ok == 1 and (v == w or (v != v and w != w))
        else:
            assert ok == 1 and v == w


def test_scan2_rejects_bad_quals(rel):
    from nvme_strom_amd.api import StromError
    from nvme_strom_amd.ops import heapscan as H
    _, pages = rel
    d2 = T.TupleDesc.of([("t", "text"), ("i", "int4")])
    with pytest.raises((ValueError, StromError)):
        H.heap_scan2(pages, d2, [T.Qual("i", "text_eq", ("x" * 40,))])
    with pytest.raises((ValueError, StromError)):
        H.heap_scan2(pages, d2, [T.Qual("t", "between", (1, 2))])


def test_relation_scan_with_quals_and_projection(tmp_path):
    """HeapRelationScan in qualifier-list mode (engine reads into the HBM
    ring, GPU deform + quals + projection) equals the reference-shaped CPU
    scan with the host deformer, for 1 and 3 participants."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import nvme_strom_amd as S
    from nvme_strom_amd.models import pg_scan
    S.configure(gpu_emulation=0)
    rows = heapgen.rows(8000, seed=21)
    data = T.build_pages(rows, heapgen.DESC, natts_of=heapgen.natts_of)
    rel = pg_scan.Relation.write(str(tmp_path / "24700"), data, relseg_size=64)
    cfg = pg_scan.ScanConfig(chunk_size=16 * 8192, buffer_size=64 * 8192, verify_checksum=True)
    for qs, proj in ((heapgen.QUAL_SETS[1], "a"), (heapgen.QUAL_SETS[3], "note"),
                     (heapgen.QUAL_SETS[5], "e")):
        c = pg_scan.cpu_scan(rel, cfg, desc=heapgen.DESC, quals=qs, project=proj)
        for workers in (1, 3):
            with pg_scan.HeapRelationScan(rel, cfg, "cuda", desc=heapgen.DESC, quals=qs,
                                          project=proj) as hs:
                g = hs.run(workers)
            assert np.array_equal(g.items, c.items)
            assert g.recheck_blocks == c.recheck_blocks
            assert np.array_equal(g.valid, c.valid)
            if isinstance(c.values, list):
                assert [v for v, ok in zip(g.values, g.valid) if ok == 1] == \
                    [v for v, ok in zip(c.values, c.valid) if ok == 1]
            else:
                m = c.valid == 1
                assert np.array_equal(g.values[m], c.values[m])


# ---- qualifier programs: CNF, any number of quals, constants of any size,
# numeric ranges
@pytest.fixture(scope="module")
def nrel():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    desc, rows = heapgen.numeric_rel(5000, seed=5)
    data = T.build_pages(rows, desc)
    return desc, data, torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()


def test_scan2_random_cnf_matches_host(nrel):
    """Randomized CNF qualifier sets (1-14 clauses of 1-3 ORed quals: up to
    ~40 quals, numeric ranges / IN with NaN and infinities, text IN lists
    and constants longer than 32 bytes, int IN lists of up to 40 values,
    fractional int bounds) over a relation with NULLs, TOAST pointers and
    compressed values: GPU == host twin, items, page status and recheck."""
    from nvme_strom_amd.ops import heapscan as H
    desc, data, pages = nrel
    rng = np.random.default_rng(2024)
    nq_max = 0
    for trial in range(40):
        qs = heapgen.random_cnf(rng, int(rng.integers(1, 15)))
        nq_max = max(nq_max, sum(len(c) for c in T.clauses(qs)))
        want, wstatus, _ = T.host_scan2(data, desc, qs)
        r = H.heap_scan2(pages, desc, qs)
        assert r.sorted_items().tolist() == want, (trial, qs)
        assert r.page_status.cpu().numpy().tolist() == wstatus, (trial, qs)
        assert (r.recheck > 0) == any(x & T.PAGE_RECHECK for x in wstatus)
    assert nq_max > 8


def _same(a, b):
    import decimal
    if isinstance(a, decimal.Decimal) and isinstance(b, decimal.Decimal):
        return str(a) == str(b)
    return a == b or (a != a and b != b)


def test_project_many_matches_host(nrel):
    """Five columns (numeric, text, int8, float8, int2) in one projection
    launch equal the host deformer's values."""
    from nvme_strom_amd.ops import heapscan as H
    desc, data, pages = nrel
    qs = [T.Or(T.Qual("amt", "ge", (0,)), T.Qual("tag", "notnull")), T.Qual("s", "between", (-30, 40))]
    cols = ["amt", "tag", "x", "f", "s"]
    want, _, wvals = T.host_scan2(data, desc, qs, project=cols)
    r = H.heap_scan2(pages, desc, qs)
    cnt = torch.tensor([r.count], dtype=torch.int32, device=pages.device)
    got = H.heap_project_many(pages, r.items, cnt, desc, cols, cap=r.count)
    order = torch.argsort(r.items[:r.count].to(torch.int64) & 0xFFFFFFFF)
    assert r.sorted_items().tolist() == want
    for j, col in enumerate(cols):
        v, ok = got[col]
        v, ok = v[order].cpu().numpy().tolist(), ok[order].cpu().numpy().tolist()
        k = desc.attno(col)
        for x, f, w in zip(v, ok, (row[j] for row in wvals)):
            if w is None:
                assert f == 0
            elif w is T.EXT:
                assert f == 2
            elif desc.attlen[k] == -1:
                assert f == 1
                raw = data[x >> 32:(x >> 32) + (x & 0xFFFFFFFF)]
                assert _same(T.numeric_value(raw) if desc.kinds[k] == "numeric" else raw, w)
            else:
                assert f == 1 and _same(x, w)


def test_relation_scan_cnf_multi_projection(tmp_path):
    """HeapRelationScan with a CNF program and three projected columns
    equals cpu_scan (host deformer), numeric values decoded to Decimal."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import nvme_strom_amd as S
    from nvme_strom_amd.models import pg_scan
    S.configure(gpu_emulation=0)
    desc, rows = heapgen.numeric_rel(6000, seed=9)
    data = T.build_pages(rows, desc)
    rel = pg_scan.Relation.write(str(tmp_path / "24800"), data, relseg_size=64)
    cfg = pg_scan.ScanConfig(chunk_size=16 * 8192, buffer_size=64 * 8192, verify_checksum=True)
    rng = np.random.default_rng(77)
    cols = ["amt", "tag", "x"]
    for _ in range(3):
        qs = heapgen.random_cnf(rng, 3)
        c = pg_scan.cpu_scan(rel, cfg, desc=desc, quals=qs, project=cols)
        with pg_scan.HeapRelationScan(rel, cfg, "cuda", desc=desc, quals=qs, project=cols) as hs:
            g = hs.run(2)
        assert np.array_equal(g.items, c.items)
        assert g.recheck_blocks == c.recheck_blocks
        for col in cols:
            gv, gok = g.columns[col]
            cv, cok = c.columns[col]
            assert np.array_equal(gok, cok)
            for a, b, f in zip(list(gv), list(cv), cok.tolist()):
                if f == 1:
                    assert _same(a, b), (col, a, b)
