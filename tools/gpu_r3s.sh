set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3s
mkdir -p $OUT
timeout -k 10 400 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 512,2048,8192 --distinct 32 --iters 5 --no-lanes --variants base,lb384,nt512,nt512ob2k,nt512lb384 --out $OUT/lz4par.json > $OUT/lz4par.log 2>&1
