set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3v
mkdir -p $OUT
for r in 2 0 4 2 0 4; do
  STROM_ARROW_ROUND_PER_CU=$r timeout -k 10 400 python -u -m nvme_strom_amd.tools.arrow_bench --reps 4 --out $OUT/arrow_r$r.json > $OUT/arrow_r$r.log 2>&1 || exit 1
  cat $OUT/arrow_r$r.json >> $OUT/arrow_r$r.jsonl; echo >> $OUT/arrow_r$r.jsonl
done
