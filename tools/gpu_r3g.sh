set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3g
timeout -k 10 300 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 256,2048 --distinct 32 --iters 3 --prof --out gpurun_out/r3g/lz4par_prof.json > gpurun_out/r3g/lz4par.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_models.py > gpurun_out/r3g/gpu_tests.log 2>&1 && \
timeout -k 10 600 python -u -m nvme_strom_amd.tools.arrow_bench --reps 4 --out gpurun_out/r3g/arrow.json > gpurun_out/r3g/arrow.log 2>&1
