export TMPDIR=/tmp; mkdir -p gpurun_out/r2c
for w in 4 6 8 12; do
  STROM_WORKERS=$w timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lat-samples 0 > gpurun_out/r2c/bench_w$w.json 2> gpurun_out/r2c/bench_w$w.err || exit 1
done
for g in 8 32; do
  STROM_INGEST_GRID=$g timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --lat-samples 0 > gpurun_out/r2c/bench_g$g.json 2> gpurun_out/r2c/bench_g$g.err || exit 1
done
