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
