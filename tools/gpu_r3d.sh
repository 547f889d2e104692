set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_models.py > gpurun_out/r3d/gpu_models.log 2>&1 && \
timeout -k 10 600 python -u -m nvme_strom_amd.tools.arrow_bench --reps 4 --out gpurun_out/r3d/arrow.json > gpurun_out/r3d/arrow.log 2>&1 && \
timeout -k 10 600 python -u -m nvme_strom_amd.tools.sweep --ab fixed_bufs --reps 3 --blocks 4K,16K,64K,256K,1M --no-raw --out gpurun_out/r3d/sweep_storage_ab.json > gpurun_out/r3d/sweep_storage.log 2>&1
