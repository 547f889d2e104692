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


@pytest.mark.parametrize("qi", range(len(heapgen.QUAL_SETS)))
def test_scan2_matches_host(rel, qi):
    from nvme_strom_amd.ops import heapscan as H
    data, pages = rel
    qs = heapgen.QUAL_SETS[qi]
    want, wstatus, _ = T.host_scan2(data, heapgen.DESC, qs, verify_checksum=True)
    r = H.heap_scan2(pages, heapgen.DESC, qs, verify_checksum=True)
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
    d2 = T.TupleDesc.of([("t", "text")])
    with pytest.raises((ValueError, StromError)):
        H.heap_scan2(pages, d2, [T.Qual("t", "text_eq", ("x" * 40,))])


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
