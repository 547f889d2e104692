#!/bin/bash
# A/B of engine knobs on the flagship bench + block sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for v in "SPIN=20" "SPIN=0" "STAGE=16777216"; do
  case $v in
    SPIN=*) export STROM_SPIN_US=${v#SPIN=}; unset STROM_STAGING_BYTES;;
    STAGE=*) export STROM_SPIN_US=20; export STROM_STAGING_BYTES=${v#STAGE=};;
  esac
  step "bench $v" timeout -k 10 300 python bench.py --lat-samples 500 > gpurun_out/ab_bench_$v.json 2> gpurun_out/ab_bench_$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab_bench_$v.json'));print('$v', d['value'], d['vfs_control_GiBps'], d['p50_4k_lat_us'])"
done
unset STROM_STAGING_BYTES; export STROM_SPIN_US=20
step sweep timeout -k 10 400 python -m nvme_strom_amd.tools.sweep --out gpurun_out/sweep_f.json > gpurun_out/sweep_f.log 2>&1
