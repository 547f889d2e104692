"""Per-kernel summary of rocprofv3 ``--pmc`` CSVs (one or more passes).

``python -m nvme_strom_amd.tools.pmc_summary DIR_OR_CSV... [--match REGEX] [--out F.json]``

Counters are summed per kernel (short name) over its dispatches, then:
  issue     SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES   (a wave issuing, per wave-cycle)
  wait      SQ_WAIT_ANY / SQ_WAVE_CYCLES          (a wave waiting on anything)
  wait_inst SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES     (waiting for an instruction slot)
  lds_active / lds_wait: SQ_ACTIVE_INST_LDS, SQ_WAIT_INST_LDS per wave-cycle
  bank_conflict_per_lds_inst: SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (cycles per LDS instruction)
  *_per_wave: instruction counts per wave (VALU, SALU, LDS, VMEM rd/wr, SMEM, branch)
Passes are joined by kernel name (each pass profiles the same program), so
ratios across passes use the same dispatches.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    """Kernel name without return type, namespaces and argument list, with
    its template arguments (the instances differ by them)."""
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    depth, cut = 0, len(n)
    for k, ch in enumerate(n):            # the argument list: the first
        if ch == "<":                     # "(" outside template brackets
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = k
            break
    n = re.sub(r"\s+", " ", n[:cut]).strip()
    n = re.sub(r"^[\w:]*::(?=\w+(<|$))", "", n)
    return n[-90:]


def load(paths, match):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for p in paths:
        files = glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True) \
            if os.path.isdir(p) else [p]
        for f in files:
            with open(f, newline="") as fh:
                for row in csv.DictReader(fh):
                    k = short(row["Kernel_Name"])
                    if match and not re.search(match, row["Kernel_Name"]):
                        continue
                    tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[k].add((f, row["Dispatch_Id"]))
                    tot[k]["_vgpr"] = float(row.get("VGPR_Count") or 0)
                    tot[k]["_lds"] = float(row.get("LDS_Block_Size") or 0)
    return tot, disp


def summarize(tot, disp):
    out = {}
    for k, c in tot.items():
        r = {"dispatches": len(disp[k]), "vgpr": c.get("_vgpr"), "lds_bytes": c.get("_lds")}
        wc = c.get("SQ_WAVE_CYCLES")
        waves = c.get("SQ_WAVES")
        if wc:
            for name, ctr in (("issue", "SQ_ACTIVE_INST_ANY"), ("wait", "SQ_WAIT_ANY"),
                              ("wait_inst", "SQ_WAIT_INST_ANY"), ("lds_active", "SQ_ACTIVE_INST_LDS"),
                              ("lds_wait", "SQ_WAIT_INST_LDS"), ("valu_active", "SQ_ACTIVE_INST_VALU"),
                              ("scalar_active", "SQ_ACTIVE_INST_SCA")):
                if ctr in c:
                    r[name] = round(c[ctr] / wc, 3)
        if c.get("SQ_INSTS_LDS"):
            r["bank_conflict_per_lds_inst"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"], 3)
        if waves:
            r["waves"] = int(waves)
            for name, ctr in (("valu", "SQ_INSTS_VALU"), ("salu", "SQ_INSTS_SALU"),
                              ("lds", "SQ_INSTS_LDS"), ("vmem_rd", "SQ_INSTS_VMEM_RD"),
                              ("vmem_wr", "SQ_INSTS_VMEM_WR"), ("smem", "SQ_INSTS_SMEM"),
                              ("branch", "SQ_INSTS_BRANCH")):
                if ctr in c:
                    r[f"{name}_per_wave"] = round(c[ctr] / waves, 1)
            if wc:
                r["cycles_per_wave"] = round(wc / waves, 1)
        for ctr in ("TCC_HIT_sum", "TCC_MISS_sum", "FETCH_SIZE", "WRITE_SIZE"):
            if ctr in c:
                r[ctr] = c[ctr]
        out[k] = r
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    tot, disp = load(a.paths, a.match)
    res = summarize(tot, disp)
    js = json.dumps(res, indent=1, sort_keys=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js)
    print(js)
    return 0


if __name__ == "__main__":
    sys.exit(main())
