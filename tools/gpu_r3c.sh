set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_models.py > gpurun_out/r3c/gpu_models.log 2>&1 && \
timeout -k 10 600 python -u -m nvme_strom_amd.tools.arrow_bench --reps 4 --out gpurun_out/r3c/arrow.json > gpurun_out/r3c/arrow.log 2>&1 && \
timeout -k 10 500 python -u -m nvme_strom_amd.tools.sweep --engine-only --ab fixed_bufs --reps 3 --blocks 4K,16K,64K,256K,1M --no-raw --out gpurun_out/r3c/sweep_cache_ab.json > gpurun_out/r3c/sweep_cache.log 2>&1
