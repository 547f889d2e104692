set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3j
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_models.py > gpurun_out/r3j/gpu_tests.log 2>&1 && \
timeout -k 10 600 python -u -m nvme_strom_amd.tools.arrow_bench --reps 5 --out gpurun_out/r3j/arrow.json > gpurun_out/r3j/arrow.log 2>&1
