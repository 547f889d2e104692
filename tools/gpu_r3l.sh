# PMC passes + kernel stats of the block-parallel LZ4 decoder (2,048 config-5 frames)
set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/r3l
mkdir -p $OUT
export TMPDIR=/tmp
export PYTHONPATH=$ROOT
BENCH="-m nvme_strom_amd.tools.lz4par_bench --kinds val --streams 2048 --distinct 32 --iters 2 --no-lanes"
n=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA" \
            "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "WRITE_SIZE SQ_BUSY_CYCLES SQ_INSTS_SMEM"; do
  n=$((n + 1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pmc$n" -o pmc \
     -- python3 $BENCH > "$OUT/pmc$n.log" 2>&1) || exit 1
done
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
   -- python3 $BENCH > "$OUT/trace.log" 2>&1)
