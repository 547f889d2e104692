set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3p
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && \
timeout -k 10 400 python -u -m nvme_strom_amd.tools.sweep --engine-only --out $OUT/sweep_cache.json > $OUT/sweep_cache.log 2>&1 && \
timeout -k 10 400 python -u -m nvme_strom_amd.tools.sweep --engine-only --blocks 4K,16K,64K --ab workers=4,8,16 --reps 2 --lat-samples 100 --out $OUT/sweep_cache_workers.json > $OUT/sweep_workers.log 2>&1 && \
timeout -k 10 500 python -u -m nvme_strom_amd.tools.pg_bench --out $OUT/pg.json > $OUT/pg.log 2>&1 && \
timeout -k 10 500 python -u -m nvme_strom_amd.tools.arrow_bench --reps 5 --out $OUT/arrow.json > $OUT/arrow.log 2>&1
