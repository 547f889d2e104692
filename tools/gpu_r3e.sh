set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3e
timeout -k 10 400 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 256,2048,8192 --distinct 32 --iters 3 --out gpurun_out/r3e/lz4par.json > gpurun_out/r3e/lz4par.log 2>&1
