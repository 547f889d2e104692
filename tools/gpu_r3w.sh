set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3w
mkdir -p $OUT
timeout -k 10 500 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 512,768,1024,2048 --distinct 32 --iters 5 --no-lanes --variants n256u16,n256u8,n512u16,n512u8,n512u8w6 --out $OUT/lz4par.json > $OUT/lz4par.log 2>&1
