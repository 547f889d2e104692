#!/bin/bash
# Decoder / verify iteration: kernel tests, kernel bench, kernel trace, and
# the BAR-map phase timings (STROM_VERBOSE=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/pytest_k.log 2>&1
step kbench timeout -k 10 240 python -m nvme_strom_amd.tools.kbench --gib 1 --only crc,verify,lz4,snappy --out gpurun_out/kbench_d.json > gpurun_out/kbench_d.log 2>&1
cat gpurun_out/kbench_d.json
step barmap timeout -k 10 120 env STROM_VERBOSE=1 python -c "
import torch
from nvme_strom_amd.tensor import HbmBuffer
for mib in (64, 1024, 4096):
    with HbmBuffer(mib << 20, 'cuda') as hb:
        pass
" > gpurun_out/barmap.log 2>&1
cd /tmp
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_d" -o k -- python3 -m nvme_strom_amd.tools.kbench --gib 0.5 --only verify,lz4,snappy > "$R/gpurun_out/prof_d.log" 2>&1
