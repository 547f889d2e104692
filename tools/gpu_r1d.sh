#!/bin/bash
# Evidence pass: GPU tests, flagship bench, block-size sweep, kernel bench,
# kernel trace of the kernel bench, kernel+copy+marker trace of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_d.log 2>&1
step bench timeout -k 10 300 python bench.py > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err
cat gpurun_out/bench_d.json
step sweep timeout -k 10 400 python -m nvme_strom_amd.tools.sweep --out gpurun_out/sweep_d.json > gpurun_out/sweep_d.log 2>&1
step kbench timeout -k 10 240 python -m nvme_strom_amd.tools.kbench --gib 1 --out gpurun_out/kbench_full_d.json > gpurun_out/kbench_full_d.log 2>&1
cd /tmp
step kprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kprof_d" -o k -- python3 -m nvme_strom_amd.tools.kbench --gib 0.5 > "$R/gpurun_out/kprof_d.log" 2>&1
export STROM_TRACE=1
step bprof timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --stats --output-format csv \
  -d "$R/gpurun_out/bprof_d" -o bench -- python3 "$R/bench.py" --steps 3 --warmup 1 --file-gib 2 --lat-samples 200 \
  > "$R/gpurun_out/bprof_d.log" 2>&1
