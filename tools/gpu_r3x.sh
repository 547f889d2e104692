set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3x
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_models.py > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 512,768,1024,2048,4096 --distinct 32 --iters 5 --out $OUT/lz4par.json > $OUT/lz4par.log 2>&1 && \
timeout -k 10 500 python -u -m nvme_strom_amd.tools.arrow_bench --reps 5 --out $OUT/arrow.json > $OUT/arrow.log 2>&1
