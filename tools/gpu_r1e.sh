#!/bin/bash
# Engine hand-off/staging changes + verify-kernel reduction: tests, bench,
# block-size sweep, kernel bench and its kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_e.log 2>&1
step bench timeout -k 10 300 python bench.py > gpurun_out/bench_e.json 2> gpurun_out/bench_e.err
cat gpurun_out/bench_e.json
step sweep timeout -k 10 400 python -m nvme_strom_amd.tools.sweep --out gpurun_out/sweep_e.json > gpurun_out/sweep_e.log 2>&1
step kbench timeout -k 10 240 python -m nvme_strom_amd.tools.kbench --gib 1 --out gpurun_out/kbench_e.json > gpurun_out/kbench_e.log 2>&1
cd /tmp
step kprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kprof_e" -o k -- python3 -m nvme_strom_amd.tools.kbench --gib 0.5 > "$R/gpurun_out/kprof_e.log" 2>&1
