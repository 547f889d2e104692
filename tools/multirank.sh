#!/bin/bash
# Multi-rank rehearsal on a one-GPU box: bench.py with 4 gloo ranks sharing
# the card (RCCL refuses two ranks on one GPU) — self-launched child
# torchrun, all-gather staged through host memory, per-slice CRC verify.
#   gpurun -- bash tools/multirank.sh TAG
set -o pipefail
TAG=${1:?tag}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python bench.py --gpus 4 --backend gloo --steps 3 --warmup 1 \
  --window-mib 256 --file-gib 1 --lat-samples 200 > "$OUT/bench_4rank_gloo.log" 2>&1 || { tail -30 "$OUT/bench_4rank_gloo.log"; exit 1; }
grep '^{' "$OUT/bench_4rank_gloo.log" | tail -1 > "$OUT/bench_4rank_gloo.json"
python -c "import json;r=json.load(open('$OUT/bench_4rank_gloo.json'));print({k:r[k] for k in ('value','n_gpus','ms_per_step')}, r['rccl'], r['per_rank'])"
