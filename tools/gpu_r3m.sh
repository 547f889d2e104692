set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/r3m
mkdir -p $OUT
export TMPDIR=/tmp
export PYTHONPATH=$ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "lz4 or decomp or codec or geometr or malformed" > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds val,ids,text --streams 512,2048,8192 --distinct 32 --iters 5 --no-lanes --variants pw16384_ob4096_hr0_lb512,pw8192_ob4096_hr0_lb256,pw16384_ob4096_hr0_lb384 --out $OUT/lz4par.json > $OUT/lz4par.log 2>&1 && \
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$OUT/pmc" -o pmc \
     -- python3 -m nvme_strom_amd.tools.lz4par_bench --kinds val --streams 2048 --distinct 32 --iters 2 --no-lanes > "$OUT/pmc.log" 2>&1)
