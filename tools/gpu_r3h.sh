set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3h
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "lz4 or decomp or codec" > gpurun_out/r3h/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 512,2048 --distinct 32 --iters 5 --prof --variants ob4096_hr32768,ob4096_hr8192,ob4096_hr0,ob2048_hr8192 --out gpurun_out/r3h/lz4par.json > gpurun_out/r3h/lz4par.log 2>&1
