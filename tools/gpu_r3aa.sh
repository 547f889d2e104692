set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/r3aa
mkdir -p $OUT
export TMPDIR=/tmp
export PYTHONPATH=$ROOT
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
   -- python3 -m nvme_strom_amd.tools.arrow_bench --reps 3 --no-qual2 --out $OUT/arrow.json > $OUT/arrow.log 2>&1)
