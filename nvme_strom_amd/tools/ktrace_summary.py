"""Per-kernel device time from a rocprofv3 ``--kernel-trace`` CSV.

``python -m nvme_strom_amd.tools.ktrace_summary trace_kernel_trace.csv [--md out.md]``

Groups dispatches by kernel name (template arguments kept, argument lists
dropped) and prints calls, median / min device microseconds and, for the
kernels whose traffic kbench knows (``--bytes name=N`` or the defaults
for a ``kbench --gib G`` run), TB/s at the median.
"""
from __future__ import annotations

import argparse
import csv
import re
import statistics
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    depth, out = 0, []
    for ch in name:                     # drop the parameter list, keep template args
        if ch == "(" and depth == 0 and out:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).replace("void ", "").strip()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--bytes", action="append", default=[],
                    help="kernel-substring=bytes per call (for TB/s)")
    ap.add_argument("--md", default="")
    a = ap.parse_args(argv)
    per = {}
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per.setdefault(short(r["Kernel_Name"]), []).append(d)
    nbytes = {}
    for kv in a.bytes:
        k, v = kv.rsplit("=", 1)
        nbytes[k] = float(v)
    rows = ["| kernel | calls | median us | min us | TB/s at median |", "|---|---|---|---|---|"]
    for k, ds in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        med = statistics.median(ds)
        tb = next((f"{b / med / 1e6:.2f}" for s, b in nbytes.items() if s in k), "")
        rows.append(f"| `{k[:90]}` | {len(ds)} | {med:.1f} | {min(ds):.1f} | {tb} |")
    text = "\n".join(rows)
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
