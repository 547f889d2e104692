set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3t
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "lz4 or decomp or codec or geometr or malformed" > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 500 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 256,512,640,768,1024,1536,2048 --distinct 32 --iters 5 --no-lanes --out $OUT/lz4par_nt.json > $OUT/lz4par.log 2>&1
