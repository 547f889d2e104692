set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3y
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_models.py > $OUT/gpu_models.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29561 -m nvme_strom_amd.tools.dist_scan_bench --rows 134217728 --reps 3 --out $OUT/dist1.json > $OUT/dist1.log 2>&1 && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29562 -m nvme_strom_amd.tools.dist_scan_bench --rows 134217728 --reps 3 --backend gloo --out $OUT/dist2_gloo.json > $OUT/dist2.log 2>&1
