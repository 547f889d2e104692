set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3z
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_models.py > $OUT/gpu_models.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29571 -m nvme_strom_amd.tools.dist_scan_bench --kind pg --pg-mib 2048 --reps 3 --out $OUT/dist_pg1.json > $OUT/dist_pg1.log 2>&1 && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29572 -m nvme_strom_amd.tools.dist_scan_bench --kind pg --pg-mib 2048 --reps 3 --backend gloo --out $OUT/dist_pg2_gloo.json > $OUT/dist_pg2.log 2>&1
