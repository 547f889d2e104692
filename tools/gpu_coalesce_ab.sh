#!/bin/bash
# A/B on one box: worker copy coalescing and staging depth, block sweep.
# Usage: tools/gpu_coalesce_ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/ab}
mkdir -p $OUT
export TMPDIR=/tmp
for v in "c0_s0" "c1_s0" "c1_s4" "c1_s8" "c0_s0b" "c1_s4b"; do
  c=${v:1:1}; s=${v#*_s}; s=${s%b}
  STROM_COALESCE=$c STROM_STAGING_BYTES=$((s << 20)) timeout -k 10 200 \
    python -u -m nvme_strom_amd.tools.sweep --blocks 4K,32K,64K,128K,256K,512K,1M \
    --out $OUT/sweep_$v.json > $OUT/sweep_$v.log 2>&1
  rc=$?; echo "sweep $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
