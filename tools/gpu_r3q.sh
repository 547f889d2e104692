set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3q
mkdir -p $OUT
timeout -k 10 500 python -u -m nvme_strom_amd.tools.sweep --blocks 4K,16K,64K,1M --ab workers=4,8 --reps 2 --lat-samples 100 --out $OUT/sweep_storage_workers.json > $OUT/sweep.log 2>&1 && \
for w in 4 8 4 8; do
  STROM_WORKERS=$w timeout -k 10 300 python bench.py > $OUT/bench_w$w.log 2>&1 || exit 1
  grep '^{' $OUT/bench_w$w.log | tail -1 >> $OUT/bench_w$w.jsonl
done
