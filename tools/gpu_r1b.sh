#!/bin/bash
# Round-1 checkpoint: GPU tests, kernel bench (incl. contiguous verify), flagship
# bench, and a kernel+copy+roctx-marker trace of the bench.  Each GPU step has
# its own time limit; the script stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_r1b.log 2>&1
step kbench timeout -k 10 240 python -m nvme_strom_amd.tools.kbench --gib 1 --out gpurun_out/kbench_r1b.json > gpurun_out/kbench_r1b.log 2>&1
step bench timeout -k 10 300 python bench.py > gpurun_out/bench_r1b.json 2> gpurun_out/bench_r1b.err
cat gpurun_out/bench_r1b.json
cd /tmp
export STROM_TRACE=1
step prof timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --stats --output-format csv \
  -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r1b" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --file-gib 2 --lat-samples 200 \
  > "$GRAFT_REPO_ROOT/gpurun_out/prof_r1b.log" 2>&1
