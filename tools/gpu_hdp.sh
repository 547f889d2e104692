#!/bin/bash
# HDP-flush BAR path: GPU tests, register discovery log, flagship bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_h.log 2>&1
step hdp timeout -k 10 120 env STROM_VERBOSE=1 python -c "
import torch
from nvme_strom_amd.tensor import HbmBuffer
with HbmBuffer(64 << 20, 'cuda') as hb:
    pass
" > gpurun_out/hdp.log 2>&1
grep -i "hdp\|bar_map" gpurun_out/hdp.log
step bench timeout -k 10 300 python bench.py --lat-samples 1000 > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err
cat gpurun_out/bench_h.json
