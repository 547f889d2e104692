#!/bin/bash
# Storage facts of the box + per-kernel trace and PMC counters for every
# CDNA4 kernel (kbench at 0.25 GiB).  Two counter passes (TCC: FETCH_SIZE
# takes 3 of 4 counters, WRITE_SIZE 2, so they go in separate passes).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step sysprobe timeout -k 10 400 bash tools/sysprobe.sh
cd /tmp
K="-m nvme_strom_amd.tools.kbench --gib 0.25"
step ktrace timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pmc" -o trace -- python3 $K > "$R/gpurun_out/pmc_trace.log" 2>&1
step pmc1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc" -o p1 -- python3 $K > "$R/gpurun_out/pmc_p1.log" 2>&1
step pmc2 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/pmc" -o p2 -- python3 $K > "$R/gpurun_out/pmc_p2.log" 2>&1
find "$R/gpurun_out/pmc" -name "*.csv" | head -20
