"""Arrow scan predicates on the CPU: every predicate kind on every column
kind, compiled by ops/colpred.py and evaluated by its numpy twin of the
GPU qualifier kernel over buffers our own metadata reader located and the
decoders' host twins decoded (models/arrow_scan.host_scan_where) — the
selected row ids must equal pyarrow.compute's (pc.filter of the row ids).
The GPU test (tests/test_gpu_models.py) runs the same cases through the
kernel."""
import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")

from arrowgen import cases, cnf_cases, expected_ids, table, write  # noqa: E402


@pytest.fixture(scope="module", params=[None, "lz4", "zstd"])
def arrow_file(request, tmp_path_factory):
    tbl = table()
    path = str(tmp_path_factory.mktemp("pred") / f"t_{request.param}.arrow")
    write(path, tbl, request.param)
    return path, tbl


def test_metadata_kinds(arrow_file):
    from nvme_strom_amd.utils.arrow_ipc import read_metadata
    path, tbl = arrow_file
    m = read_metadata(path)
    assert m == read_metadata(path, native=False)
    kinds = {c.name: (c.kind, c.storage, c.unit) for c in m.schema}
    assert kinds["d32"] == ("date", "i4", "d") and kinds["ts"] == ("timestamp", "i8", "us")
    assert kinds["t32"] == ("time", "i4", "ms") and kinds["dur"] == ("duration", "i8", "s")
    assert kinds["b"][1] == "b1" and kinds["s"] == ("utf8", "i4", "")
    assert kinds["ls"] == ("utf8", "i8", "") and kinds["bin"] == ("binary", "i4", "")
    assert kinds["dict"] == ("utf8", "i4", "") and m.schema[m.column_index("dict")].dictionary
    assert kinds["idict"] == ("int", "i1", "")
    assert kinds["dec"] == ("decimal", "d16", "")
    assert m.schema[m.column_index("dec")].scale == 4
    assert m.schema[m.column_index("ts")].tz == "UTC"
    assert all(c.supported for c in m.schema)


@pytest.mark.parametrize("case", range(len(cases())), ids=[c[0] for c in cases()])
def test_predicate_matches_pyarrow(arrow_file, case):
    from nvme_strom_amd.models.arrow_scan import host_scan_where
    path, tbl = arrow_file
    label, pred, ref = cases()[case]
    got = host_scan_where(path, [pred])
    want = expected_ids(tbl, ref)
    assert got.rows == tbl.num_rows
    assert np.array_equal(got.indices, want), (label, len(got.indices), len(want))


@pytest.mark.parametrize("case", range(len(cnf_cases())), ids=[c[0] for c in cnf_cases()])
def test_qualifier_list_matches_pyarrow(arrow_file, case):
    from nvme_strom_amd.models.arrow_scan import host_scan_where
    path, tbl = arrow_file
    label, quals, ref = cnf_cases()[case]
    got = host_scan_where(path, quals, project="ts", batches=(1, 4))
    want = expected_ids(tbl, ref)
    lo, hi = 700, 2800
    want = want[(want >= lo) & (want < hi)]
    assert np.array_equal(got.indices, want), label
    ts = tbl.column("ts").combine_chunks()
    ref_v = np.asarray(ts.cast("int64").fill_null(0))[want]
    assert np.array_equal(np.where(got.valid if got.valid is not None else True, got.values, 0),
                          np.where(np.asarray(ts.is_valid())[want], ref_v, 0))


def test_projection_of_strings_and_dictionary(arrow_file):
    from nvme_strom_amd.models.arrow_scan import host_scan_where
    from nvme_strom_amd.ops.colpred import P
    path, tbl = arrow_file
    got = host_scan_where(path, [P("i8") > 100], project="s")
    ids = got.indices
    s = tbl.column("s").combine_chunks()
    assert [v for v, ok in zip(got.values, got.valid if got.valid is not None else
                               [True] * len(ids)) if ok] == \
        [s[int(i)].as_py().encode() for i in ids if s[int(i)].is_valid]
    got = host_scan_where(path, [P("i8") > 100], project="dict")
    d = tbl.column("dict").combine_chunks()
    assert np.array_equal(np.asarray(got.values),
                          np.asarray(d.indices.fill_null(0))[ids] * np.asarray(d.is_valid())[ids]
                          + np.asarray(got.values) * ~np.asarray(d.is_valid())[ids])


def test_compile_exact_bounds():
    """Integer bounds in the column's own domain; float strictness by
    nextafter; empty and impossible predicates; the refusals."""
    import math

    from nvme_strom_amd.ops import colpred as CP
    from nvme_strom_amd.utils.arrow_ipc import Column
    i8 = Column("x", "int", 8, True)
    f8 = Column("y", "float", 64, True)
    u64 = Column("u", "int", 64, False)
    s = Column("s", "utf8", 0, False, nbuffers=3)
    r = lambda p, c: CP.compile_pred(p, c).ranges.tolist()
    assert r(CP.P("x") < 2.5, i8) == [[-128, 2]]
    assert r(CP.P("x") > 2.5, i8) == [[3, 127]]
    assert r(CP.P("x") == 2.5, i8) == []
    assert r(CP.P("x") > 1000, i8) == []
    assert r(CP.P("x").isin([1, 2, 3, 7]), i8) == [[1, 3], [7, 7]]
    assert r(CP.P("x") < float("inf"), i8) == [[-128, 127]]
    assert r(CP.P("x") == float("nan"), i8) == []
    assert r(CP.P("u") >= 2**63, u64) == [[2**63, 2**64 - 1]]
    assert r(CP.P("y") < 1.0, f8) == [[-math.inf, math.nextafter(1.0, -math.inf)]]
    q = CP.compile_pred(CP.P("y").isin([float("nan"), 2.0]), f8)
    assert q.flags & CP.FLAG_NAN and q.ranges.tolist() == [[2.0, 2.0]]
    q = CP.compile_pred(CP.P("s").isin(["b", "abc", "b"]), s)
    assert q.op == CP.QOP_STR_IN and q.nconst == 2
    assert np.frombuffer(q.offs, np.uint32).tolist() == [0, 3, 4, 1]
    q = CP.compile_pred(CP.P("s") < "b", s)
    assert q.op == CP.QOP_STR_RANGES and np.frombuffer(q.offs, np.uint32).tolist() == [0, 0, 0,
                                                                                       0, 1, 2]
    with pytest.raises(ValueError):
        CP.compile_pred(CP.P("x").startswith("a"), i8)
    with pytest.raises(ValueError):
        CP.Pred("x", "~=", 1)
    assert CP.clauses([("x", 1, 2), ("x", "in", [1]), CP.Or(("x", "==", 1), CP.P("y") > 0)]) == [
        [CP.Pred("x", "between", (1, 2))], [CP.Pred("x", "in", [1])],
        [CP.Pred("x", "==", 1), CP.Pred("y", ">", 0)]]


def test_dictionary_headers_malformed(tmp_path):
    """Corrupted DictionaryBatch headers end in a ValueError (or a file that
    still parses), never another exception type."""
    import pyarrow.ipc as ipc
    from nvme_strom_amd.utils.arrow_ipc import read_metadata
    tbl = pa.table({"d": pa.array(["x", "y", "z"] * 100).dictionary_encode(),
                    "i": np.arange(300)})
    path = str(tmp_path / "d.arrow")
    with ipc.new_file(path, tbl.schema) as w:
        w.write_table(tbl)
    m = read_metadata(path)
    blk = m.dicts[0][0].buffers[0].offset        # the dictionary batch body
    raw = bytearray(open(path, "rb").read())
    rng = np.random.default_rng(4)
    for trial in range(60):
        bad = bytearray(raw)
        pos = int(rng.integers(max(8, blk - 200), blk))
        bad[pos:pos + 4] = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        p = str(tmp_path / f"b{trial}.arrow")
        open(p, "wb").write(bad)
        try:
            read_metadata(p, native=False)
        except ValueError:
            pass


def test_scan_geometry_defaults_and_slots(arrow_file):
    """Codec-dependent defaults (ZSTD: 16 KiB chunks, 4 slots; else 64 KiB, 3)
    and the slot ring: one slot per group while it fits, never fewer than
    nslots, never more than the groups or MAX_SLOTS."""
    import torch
    from nvme_strom_amd.models.arrow_scan import ArrowScan
    path, _ = arrow_file
    sc = ArrowScan(path, torch.device("cpu"))
    zstd = set(sc.meta.codecs) - {None} == {"zstd"}
    assert sc.chunk_sz == (16 << 10 if zstd else 64 << 10)
    assert sc.nslots == (4 if zstd else 3)
    g = [object()] * 40
    assert sc._slot_count(g[:2], 1 << 20) == 2                 # never more than the groups
    assert sc._slot_count(g[:10], 1 << 20) == 10               # a slot per group
    assert sc._slot_count(g, 1 << 20) == ArrowScan.MAX_SLOTS
    assert sc._slot_count(g, 4 << 30) == sc.nslots             # the byte cap, floored at nslots
    assert ArrowScan(path, torch.device("cpu"), chunk_sz=8192, nslots=5).chunk_sz == 8192
