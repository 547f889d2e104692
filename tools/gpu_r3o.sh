set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3o
mkdir -p $OUT
timeout -k 10 400 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 512,2048 --distinct 32 --iters 5 --no-lanes --variants d0r0,d0r1,d1r0,d1r1 --out $OUT/lz4par.json > $OUT/lz4par.log 2>&1
