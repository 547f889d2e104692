"""Diagnostic: the cold-then-warm Arrow scan with the BAR mapping off
(tests/test_gpu_models.py::test_arrow_scan_bar_refused_after_cold_scan),
with a watchdog that dumps the Python stacks and the ingest grid's counters
if a step stalls."""
import faulthandler
import os
import sys
import threading
import time

import numpy as np
import pyarrow as pa
import pyarrow.ipc as ipc
import torch

import nvme_strom_amd as S
from nvme_strom_amd.models.arrow_scan import ArrowScan

faulthandler.dump_traceback_later(40, exit=True)
step = ["start"]


def watch():
    while True:
        time.sleep(10)
        print("watchdog", step[0], S.ingest_info(0), file=sys.stderr, flush=True)


threading.Thread(target=watch, daemon=True).start()
d = sys.argv[1] if len(sys.argv) > 1 else "/tmp/arrow_diag"
os.makedirs(d, exist_ok=True)
rng = np.random.default_rng(7)
n, nb = 200_000, 4
a = rng.integers(-10**6, 10**6, n * nb)
b = rng.integers(-10**6, 10**6, n * nb)
tbl = pa.table({"a": pa.array(a, type=pa.int64()), "b": pa.array(b, type=pa.int64())})
path = os.path.join(d, "w.arrow")
with ipc.new_file(path, tbl.schema) as w:
    for k in range(nb):
        w.write_batch(tbl.slice(k * n, n).to_batches()[0])
S.configure(gpu_emulation=0, bar_map=int(os.environ.get("BAR", "0")))
fd = os.open(path, os.O_RDONLY)
S.evict_file(fd)
os.close(fd)
sc = ArrowScan(path, "cuda")
step[0] = "filter"
out = sc.filter("a", -1000, 5000)
print("filter ok", out.selected, S.ingest_info(0), flush=True)
with open(path, "rb") as f:
    f.read()
step[0] = "scan_where"
out = sc.scan_where([("a", -500_000, 200_000), ("b", 0, 700_000)], project="b")
sel = (a >= -500_000) & (a <= 200_000) & (b >= 0) & (b <= 700_000)
print("scan_where ok", out.selected, int(sel.sum()), S.ingest_info(0), flush=True)
