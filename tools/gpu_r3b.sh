set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
ulimit -l > gpurun_out/r3b/memlock.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r3b/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u -m nvme_strom_amd.tools.sweep --engine-only --ab fixed_bufs --out gpurun_out/r3b/sweep_cache_ab.json > gpurun_out/r3b/sweep_cache.log 2>&1 && \
timeout -k 10 400 python -u -m nvme_strom_amd.tools.sweep --ab fixed_bufs --blocks 4K,16K,64K,256K,1M --out gpurun_out/r3b/sweep_storage_ab.json > gpurun_out/r3b/sweep_storage.log 2>&1
