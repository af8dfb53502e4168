"""Probe: torch imported (and gloo initialised) before libgcz -> one HIP runtime in the process."""
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("gloo", rank=0, world_size=1)
import __graft_entry__ as g  # noqa: E402

g.smoke()
print("torch.cuda.is_available:", torch.cuda.is_available())
dist.destroy_process_group()
