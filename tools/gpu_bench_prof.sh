#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --file-gib 4 > gpurun_out/bench2.json 2> gpurun_out/bench2.err
echo "bench rc=$?"; cat gpurun_out/bench2.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 3 --warmup 1 --file-gib 2 --lat-samples 200 > gpurun_out/prof_bench.log 2>&1
echo "prof rc=$?"
