#!/bin/bash
# First GPU pass: tests, smoke, short bench, kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" 
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --file-gib 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"
cat gpurun_out/bench1.json
