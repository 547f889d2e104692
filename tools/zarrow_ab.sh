#!/bin/bash
# A/B of the ZSTD Arrow scan's group size (STROM_ARROW_ZSTD_DIV), arms
# interleaved in one box call: gpurun -- bash tools/zarrow_ab.sh TAG
set -o pipefail
TAG=${1:?tag}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONPATH=$PWD
for rep in 1 2; do
  for div in 1 4 8; do
    STROM_ARROW_ZSTD_DIV=$div timeout -k 10 300 python -u -m nvme_strom_amd.tools.arrow_bench --codec zstd \
      --no-qual2 --out "$OUT/zdiv${div}_rep${rep}.json" > "$OUT/zdiv${div}_rep${rep}.log" 2>&1 || exit $?
    python -c "import json;r=json.load(open('$OUT/zdiv${div}_rep${rep}.json'));print('div $div rep $rep', {k:(v['column_GBps'],v['cold_ms'],v['verified']) for k,v in r['columns'].items()})"
  done
done
