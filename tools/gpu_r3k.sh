set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3k
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py > gpurun_out/r3k/gpu_kernels.log 2>&1 && \
timeout -k 10 300 python -u -m nvme_strom_amd.tools.decomp_ab nvme_strom_amd/lib/ab/r3cur.so --streams 16384 --distinct 61 --rounds 3 --out gpurun_out/r3k/decomp_16k_diverging.json > gpurun_out/r3k/decomp_ab.log 2>&1 && \
timeout -k 10 500 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 4096,8192,16384 --distinct 32 --iters 3 --out gpurun_out/r3k/lz4par_threshold.json > gpurun_out/r3k/lz4par.log 2>&1
