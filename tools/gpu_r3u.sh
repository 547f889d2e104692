set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3u
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_models.py tests/test_gpu_kernels.py > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 600 python -u -m nvme_strom_amd.tools.arrow_bench --reps 6 --out $OUT/arrow.json > $OUT/arrow.log 2>&1
