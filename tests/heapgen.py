"""Random heap relations with real tuple descriptors (shared by the CPU and
GPU heap-scan tests): utils.pgtuple.synthetic's 10-column relation."""
from nvme_strom_amd.utils import pgtuple as T

DESC = T.synthetic(1)[0]


def rows(n: int, seed: int = 0):
    return T.synthetic(n, seed)[1]


def natts_of(i: int) -> int:
    # every 13th row was written before the last two columns were added
    return 8 if i % 13 == 5 else 10


QUAL_SETS = [
    [T.Qual("a", "between", (-200_000, 300_000))],
    [T.Qual("a", "between", (-500_000, 200_000)), T.Qual("b", "between", (0.1, 0.6))],
    [T.Qual("name", "text_eq", ("k17",))],
    [T.Qual("note", "prefix", ("ab",)), T.Qual("c", "in", ([1, 2, 3],))],
    [T.Qual("flag", "eq", (1,)), T.Qual("b", "isnull")],
    [T.Qual("e", "between", (-0.5, 0.5)), T.Qual("d", "notnull"), T.Qual("tail", "between", (0, 50))],
    [T.Qual("tail", "isnull")],
    [T.Qual("id", "between", (100, 4000)), T.Qual("name", "notnull"), T.Qual("note", "text_eq", ("zzzz",))],
]


# ---- general qualifier programs: CNF, IN lists / text of any size, numeric
def numeric_rel(n: int, seed: int = 0):
    """A relation with numeric and text columns (NULLs, long values, TOAST
    pointers and compressed datums) for qualifier-program tests."""
    import decimal

    import numpy as np
    desc = T.TupleDesc.of([("id", "int4"), ("amt", "numeric"), ("tag", "text"), ("x", "int8"),
                           ("big", "numeric"), ("f", "float8"), ("s", "int2")])
    rng = np.random.default_rng(seed)
    words = ["alpha", "beta", "gamma", "delta", "x" * 40, "y" * 130, "prefix-" + "p" * 50, ""]
    rows = []
    for i in range(n):
        r = rng.random()
        amt = (None if r < 0.08 else decimal.Decimal("NaN") if r < 0.1 else
               decimal.Decimal("Infinity") if r < 0.11 else decimal.Decimal("-Infinity") if r < 0.12
               else decimal.Decimal(int(rng.integers(-10**7, 10**7))).scaleb(-int(rng.integers(0, 5))))
        tr = rng.random()
        tag = (None if tr < 0.1 else T.Toast(i) if tr < 0.13 else T.Compressed() if tr < 0.16
               else words[int(rng.integers(0, len(words)))])
        big = decimal.Decimal(int(rng.integers(0, 10**9))) * (decimal.Decimal(10) ** int(rng.integers(-30, 30)))
        rows.append([i, amt, tag, None if rng.random() < 0.1 else int(rng.integers(-1000, 1000)),
                     None if rng.random() < 0.05 else big, float(rng.normal()),
                     int(rng.integers(-50, 50))])
    return desc, rows


def random_cnf(rng, nclauses: int):
    """A random qualifier list over numeric_rel's columns: clauses of 1-3
    ORed quals of every kind."""
    import decimal
    D = decimal.Decimal
    words = ["alpha", "beta", "gamma", "delta", "x" * 40, "y" * 130, "none", "prefix-" + "p" * 50]

    def one():
        k = int(rng.integers(0, 12))
        if k == 0:
            a = D(int(rng.integers(-10**7, 10**7))).scaleb(-int(rng.integers(0, 4)))
            return T.Qual("amt", "between", (a, a + D(int(rng.integers(0, 10**6)))))
        if k == 1:
            return T.Qual("amt", ["lt", "le", "gt", "ge", "eq"][int(rng.integers(0, 5))],
                          (D(int(rng.integers(-10**6, 10**6))).scaleb(-2),))
        if k == 2:
            return T.Qual("amt", "in", ([D("NaN"), D("Infinity"), D(int(rng.integers(-5, 5)))],))
        if k == 3:
            return T.Qual("tag", "text_in", ([words[int(j)] for j in rng.integers(0, len(words), 5)],))
        if k == 4:
            return T.Qual("tag", "text_eq", (words[int(rng.integers(0, len(words)))],))
        if k == 5:
            return T.Qual("tag", "prefix", (["prefix-" + "p" * 40, "x" * 35, "al", ""][int(rng.integers(0, 4))],))
        if k == 6:
            return T.Qual("x", "in", ([int(v) for v in rng.integers(-1000, 1000, int(rng.integers(1, 40)))],))
        if k == 7:
            lo = float(rng.integers(-1000, 1000)) + 0.5
            return T.Qual("x", "between", (lo, lo + float(rng.integers(0, 500))))
        if k == 8:
            return T.Qual("big", ["gt", "lt"][int(rng.integers(0, 2))],
                          (D(int(rng.integers(0, 10**9))) * D(10) ** int(rng.integers(-30, 30)),))
        if k == 9:
            return T.Qual("f", ["lt", "ge"][int(rng.integers(0, 2))], (float(rng.normal()),))
        if k == 10:
            return T.Qual(["amt", "tag", "x", "big"][int(rng.integers(0, 4))],
                          ["isnull", "notnull"][int(rng.integers(0, 2))])
        return T.Qual("s", "eq", (float(rng.integers(-50, 50)) + (0.5 if rng.random() < 0.3 else 0.0),))
    out = []
    for _ in range(nclauses):
        m = int(rng.integers(1, 4))
        out.append(one() if m == 1 else T.Or(*[one() for _ in range(m)]))
    return out
