"""Probe: can two RCCL ranks share one GPU on this pool box?  (If yes, the
multi-rank nccl path of bench.py / ShardedLoader can be rehearsed on a
1-GPU box.)  torchrun --nproc-per-node 2 tools/probe/rccl_same_gpu.py"""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.full((1 << 20,), rank + 1, dtype=torch.int32, device="cuda:0")
out = torch.empty(world << 20, dtype=torch.int32, device="cuda:0")
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
ok = all(int(out[i << 20]) == i + 1 for i in range(world))
print(f"rank {rank}: all_gather ok={ok}", flush=True)
dist.destroy_process_group()
sys.exit(0 if ok else 3)
