"""Synthetic Arrow IPC tables of every column kind the GPU scan takes, and
each predicate kind with its pyarrow.compute reference (shared by the CPU
parity test and the GPU test)."""
from __future__ import annotations

import datetime as dt
import decimal

import numpy as np

from nvme_strom_amd.ops.colpred import Or, P


def table(n: int = 3000, seed: int = 5):
    import pyarrow as pa
    rng = np.random.default_rng(seed)
    nulls = lambda p=0.07: rng.random(n) < p
    f32 = rng.normal(0, 10, n).astype(np.float32)
    f32[rng.random(n) < 0.03] = np.nan
    words = ["", "a", "ab", "abc", "abcd", "apple", "apricot", "banana", "band", "bandana",
             "cherry", "cherries", "日本語", "日本", "zz" * 13, "prefix-" + "x" * 30]
    s = [words[k] for k in rng.integers(0, len(words), n)]
    ts0 = np.datetime64("2024-01-01T00:00:00", "us").astype(np.int64)
    # decimal(18, 4) unscaled values; a fifth of them near 1.1 / 2.5, so float
    # constants (compared as float64, like pyarrow) select something
    dv = rng.integers(-10**9, 10**9, n)
    near = rng.random(n) < 0.2
    dv[near] = rng.choice([11000, 10999, 11001, -11000, 25000], int(near.sum()))
    cols = {
        "i8": pa.array(rng.integers(-128, 128, n).astype(np.int8), mask=nulls()),
        "u32": pa.array(rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)),
        "i64": pa.array(rng.integers(-10**12, 10**12, n), mask=nulls()),
        "f32": pa.array(f32, mask=nulls(0.05)),
        "f64": pa.array(rng.random(n)),
        "b": pa.array(rng.random(n) < 0.3, mask=nulls()),
        "d32": pa.array([dt.date(2020, 1, 1) + dt.timedelta(days=int(k))
                         for k in rng.integers(0, 2000, n)], pa.date32()),
        "ts": pa.array(ts0 + rng.integers(0, 86400 * 10**6 * 30, n), pa.timestamp("us", tz="UTC"),
                       mask=nulls()),
        "t32": pa.array(rng.integers(0, 86400 * 1000, n).astype(np.int32), pa.time32("ms")),
        "dur": pa.array(rng.integers(-1000, 1000, n), pa.duration("s")),
        "s": pa.array(s, mask=nulls()),
        "bin": pa.array([x.encode() for x in s], pa.binary()),
        "ls": pa.array(s, pa.large_string()),
        "dict": pa.array([words[k] for k in rng.integers(0, 9, n)], mask=nulls()).dictionary_encode(),
        "dec": pa.array([decimal.Decimal(int(v)).scaleb(-4) for v in dv], pa.decimal128(18, 4),
                        mask=nulls()),
        "idict": pa.DictionaryArray.from_arrays(
            pa.array(rng.integers(0, 20, n).astype(np.int8)),
            pa.array(np.arange(20, dtype=np.int64) * 1000 - 3000)),
    }
    return pa.table(cols)


def write(path: str, tbl, compression=None, batch_rows: int = 700) -> None:
    import pyarrow.ipc as ipc
    with ipc.new_file(path, tbl.schema,
                      options=ipc.IpcWriteOptions(compression=compression)) as w:
        for b0 in range(0, tbl.num_rows, batch_rows):
            for b in tbl.slice(b0, batch_rows).to_batches():
                w.write_batch(b)


D0 = dt.date(2021, 6, 1)
T0 = dt.datetime(2024, 1, 9, 12, 30, tzinfo=dt.timezone.utc)

# (label, predicate, pyarrow reference: table -> boolean mask)
def cases():
    import pyarrow as pa
    import pyarrow.compute as pc
    c = lambda t, n: t.column(n).combine_chunks()
    dec = lambda t, n: c(t, n).dictionary_decode()
    isin = lambda a, v: pc.and_(pc.is_in(a, value_set=pa.array(v, type=a.type)), pc.is_valid(a))
    notin = lambda a, v: pc.and_(pc.invert(pc.is_in(a, value_set=pa.array(v, type=a.type))),
                                 pc.is_valid(a))
    rng_ = lambda a, lo, hi: pc.and_(pc.greater_equal(a, lo), pc.less_equal(a, hi))
    return [
        ("i8 range (legacy)", ("i8", -20, 40), lambda t: rng_(c(t, "i8"), -20, 40)),
        ("i8 == ", P("i8") == 7, lambda t: pc.equal(c(t, "i8"), 7)),
        ("i8 != ", P("i8") != 7, lambda t: pc.not_equal(c(t, "i8"), 7)),
        ("i8 < 2.5", P("i8") < 2.5, lambda t: pc.less(c(t, "i8"), 2.5)),
        ("i8 > -300", P("i8") > -300, lambda t: pc.greater(c(t, "i8"), -300)),
        ("u32 >= 2^31", P("u32") >= 1 << 31, lambda t: pc.greater_equal(c(t, "u32"), 1 << 31)),
        ("u32 in", P("u32").isin([0, 5, 1 << 31]),
         lambda t: isin(c(t, "u32"), [0, 5, 1 << 31])),
        ("i64 between", P("i64").between(-10**11, 3 * 10**11),
         lambda t: rng_(c(t, "i64"), -10**11, 3 * 10**11)),
        ("i64 ranges", P("i64").ranges([(-10**12, -9 * 10**11), (0, 10**10), (5 * 10**11, 10**12)]),
         lambda t: pc.or_kleene(pc.or_kleene(rng_(c(t, "i64"), -10**12, -9 * 10**11),
                                 rng_(c(t, "i64"), 0, 10**10)),
                          rng_(c(t, "i64"), 5 * 10**11, 10**12))),
        ("f32 <= 0.1", P("f32") <= 0.1, lambda t: pc.less_equal(c(t, "f32"), 0.1)),
        ("f32 != 0", P("f32") != 0.0, lambda t: pc.not_equal(c(t, "f32"), 0.0)),
        ("f32 in NaN", P("f32").isin([float("nan"), 1.0]),
         lambda t: isin(c(t, "f32"), [float("nan"), 1.0])),
        ("f64 > 0.75", P("f64") > 0.75, lambda t: pc.greater(c(t, "f64"), 0.75)),
        ("b == True", P("b") == True,  # noqa: E712
         lambda t: pc.equal(c(t, "b"), True)),
        ("b is_null", P("b").is_null(), lambda t: pc.is_null(c(t, "b"))),
        ("d32 between", P("d32").between(D0, dt.date(2022, 1, 31)),
         lambda t: rng_(c(t, "d32"), pa.scalar(D0), pa.scalar(dt.date(2022, 1, 31)))),
        ("d32 in", P("d32").isin([dt.date(2020, 1, 5), D0]),
         lambda t: isin(c(t, "d32"), [dt.date(2020, 1, 5), D0])),
        ("ts < T0", P("ts") < T0, lambda t: pc.less(c(t, "ts"), pa.scalar(T0, pa.timestamp("us", "UTC")))),
        ("ts >= np64", P("ts") >= np.datetime64("2024-01-20T00:00:00.5"),
         lambda t: pc.greater_equal(c(t, "ts"), pa.scalar(
             dt.datetime(2024, 1, 20, 0, 0, 0, 500000, tzinfo=dt.timezone.utc),
             pa.timestamp("us", "UTC")))),
        ("t32 < 12:00", P("t32") < dt.time(12, 0), lambda t: pc.less(c(t, "t32"),
                                                                      pa.scalar(dt.time(12, 0), pa.time32("ms")))),
        ("dur > 1min", P("dur") > dt.timedelta(minutes=1),
         lambda t: pc.greater(c(t, "dur"), pa.scalar(dt.timedelta(minutes=1), pa.duration("s")))),
        ("s ==", P("s") == "apple", lambda t: pc.equal(c(t, "s"), "apple")),
        ("s == ''", P("s") == "", lambda t: pc.equal(c(t, "s"), "")),
        ("s != ", P("s") != "banana", lambda t: pc.not_equal(c(t, "s"), "banana")),
        ("s in", P("s").isin(["abc", "日本語", "zz" * 13]),
         lambda t: isin(c(t, "s"), ["abc", "日本語", "zz" * 13])),
        ("s not in", P("s").not_in(["abc", "band"]), lambda t: notin(c(t, "s"), ["abc", "band"])),
        ("s prefix", P("s").startswith("ban"), lambda t: pc.starts_with(c(t, "s"), "ban")),
        ("s prefix long", P("s").startswith("prefix-xxxxxxxxx"),
         lambda t: pc.starts_with(c(t, "s"), "prefix-xxxxxxxxx")),
        ("s prefix utf8", P("s").startswith("日本"), lambda t: pc.starts_with(c(t, "s"), "日本")),
        ("s range", P("s").between("ab", "apple"), lambda t: rng_(c(t, "s"), "ab", "apple")),
        ("s < ", P("s") < "b", lambda t: pc.less(c(t, "s"), "b")),
        ("s > utf8", P("s") > "日", lambda t: pc.greater(c(t, "s"), "日")),
        ("ls ranges", P("ls").ranges([("a", "abc"), ("cherry", "zz")]),
         lambda t: pc.or_kleene(rng_(c(t, "ls"), "a", "abc"), rng_(c(t, "ls"), "cherry", "zz"))),
        ("bin ==", P("bin") == b"cherry", lambda t: pc.equal(c(t, "bin"), pa.scalar(b"cherry"))),
        ("bin prefix", P("bin").startswith(b"ap"), lambda t: pc.starts_with(c(t, "bin"), b"ap")),
        ("ls ==", P("ls") == "bandana", lambda t: pc.equal(c(t, "ls"), "bandana")),
        ("ls prefix", P("ls").startswith("a"), lambda t: pc.starts_with(c(t, "ls"), "a")),
        ("dict ==", P("dict") == "apple", lambda t: pc.equal(dec(t, "dict"), "apple")),
        ("dict in", P("dict").isin(["a", "abcd", "nope"]),
         lambda t: isin(dec(t, "dict"), ["a", "abcd", "nope"])),
        ("dict prefix", P("dict").startswith("ab"), lambda t: pc.starts_with(dec(t, "dict"), "ab")),
        ("dict range", P("dict").between("ab", "apple"),
         lambda t: rng_(dec(t, "dict"), "ab", "apple")),
        ("dict is_null", P("dict").is_null(), lambda t: pc.is_null(c(t, "dict"))),
        ("idict >", P("idict") > 5000, lambda t: pc.greater(dec(t, "idict"), 5000)),
        ("dec > ", P("dec") > decimal.Decimal("12.3456"),
         lambda t: pc.greater(c(t, "dec"), pa.scalar(decimal.Decimal("12.3456"), pa.decimal128(18, 4)))),
        ("dec between", P("dec").between(-5, 7.25),
         lambda t: rng_(c(t, "dec"), pa.scalar(decimal.Decimal("-5"), pa.decimal128(18, 4)),
                        pa.scalar(decimal.Decimal("7.25"), pa.decimal128(18, 4)))),
        ("dec in", P("dec").isin([decimal.Decimal("0.0001"), 3]),
         lambda t: isin(c(t, "dec"), [decimal.Decimal("0.0001"), decimal.Decimal("3.0000")])),
        # float constants on a decimal column: compared in float64, as pyarrow does
        ("dec == 1.1", P("dec") == 1.1, lambda t: pc.equal(c(t, "dec"), 1.1)),
        ("dec >= 1.1", P("dec") >= 1.1, lambda t: pc.greater_equal(c(t, "dec"), 1.1)),
        ("dec < 1.1", P("dec") < 1.1, lambda t: pc.less(c(t, "dec"), 1.1)),
        ("dec > 2.5", P("dec") > 2.5, lambda t: pc.greater(c(t, "dec"), 2.5)),
        ("dec in floats", P("dec").isin([1.1, 2.5]),
         lambda t: pc.and_(pc.is_in(c(t, "dec"), value_set=pa.array([1.1, 2.5])),
                           pc.is_valid(c(t, "dec")))),
        ("or across columns", Or(P("i8") < -100, P("s") == "apple", P("b") == True),  # noqa: E712
         lambda t: pc.or_kleene(pc.or_kleene(pc.less(c(t, "i8"), -100), pc.equal(c(t, "s"), "apple")),
                          pc.equal(c(t, "b"), True))),
    ]


def cnf_cases():
    """Whole qualifier lists: AND of clauses, some of them ORs."""
    import pyarrow.compute as pc
    c = lambda t, n: t.column(n).combine_chunks()
    return [
        ("and3", [("i64", -5 * 10**11, 5 * 10**11), P("s").startswith("a"), P("f64") < 0.5],
         lambda t: pc.and_(pc.and_(pc.and_(pc.greater_equal(c(t, "i64"), -5 * 10**11),
                                           pc.less_equal(c(t, "i64"), 5 * 10**11)),
                                   pc.starts_with(c(t, "s"), "a")),
                           pc.less(c(t, "f64"), 0.5))),
        ("or then and", [Or(P("i8") < 0, P("dict") == "apple"), P("d32") >= D0,
                         Or(P("b").is_null(), P("f64") > 0.9)],
         lambda t: pc.and_(pc.and_(
             pc.or_kleene(pc.less(c(t, "i8"), 0), pc.equal(c(t, "dict").dictionary_decode(), "apple")),
             pc.greater_equal(c(t, "d32"), D0)),
             pc.or_kleene(pc.is_null(c(t, "b")), pc.greater(c(t, "f64"), 0.9)))),
    ]


def expected_ids(tbl, mask_fn):
    import pyarrow as pa
    import pyarrow.compute as pc
    m = mask_fn(tbl)
    m = m.combine_chunks() if hasattr(m, "combine_chunks") else m
    ids = pa.array(np.arange(tbl.num_rows, dtype=np.int64))
    return np.asarray(pc.filter(ids, m.fill_null(False)))
