#!/bin/bash
# Kernel throughput + rocprofv3 kernel stats + counters for the post-read kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m nvme_strom_amd.tools.kbench --gib 1 --out gpurun_out/kbench.json > gpurun_out/kbench.log 2>&1
echo "kbench rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_k -o k -- python3 -m nvme_strom_amd.tools.kbench --gib 0.5 > gpurun_out/prof_k.log 2>&1
echo "prof rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT FETCH_SIZE WRITE_SIZE --output-format csv -d gpurun_out/pmc_k -o k -- python3 -m nvme_strom_amd.tools.kbench --gib 0.25 > gpurun_out/pmc_k.log 2>&1
echo "pmc rc=$?"
