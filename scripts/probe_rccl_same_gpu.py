"""Probe: can two ranks share one GPU through RCCL (torch 'nccl' backend)?

Run: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
     --master-port 29512 scripts/probe_rccl_same_gpu.py
"""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    x = torch.full((4,), float(rank + 1), device="cuda:0")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce ok {x.tolist()}", flush=True)
    y = torch.arange(4, device="cuda:0", dtype=torch.int64) + 10 * rank
    z = torch.empty_like(y)
    dist.all_to_all_single(z, y)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_to_all ok {z.tolist()}", flush=True)
    dist.destroy_process_group()
except Exception as e:  # report and exit non-zero
    print(f"rank {rank}: FAILED {type(e).__name__}: {e}", flush=True)
    sys.exit(3)
