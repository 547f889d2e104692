set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3i
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "lz4 or decomp or codec" > gpurun_out/r3i/gpu_tests.log 2>&1 && \
timeout -k 10 500 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 512,1024,2048,4096 --distinct 32 --iters 5 --no-lanes --variants pw16384_ob4096_hr0_lb512,pw8192_ob4096_hr0_lb256,pw8192_ob4096_hr0_lb512,pw8192_ob2048_hr0_lb256,pw16384_ob2048_hr0_lb512 --out gpurun_out/r3i/lz4par.json > gpurun_out/r3i/lz4par.log 2>&1
