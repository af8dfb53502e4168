#!/usr/bin/env python3
"""World-1 RCCL group lifecycle probe: which librccl copies the process maps, and
whether create -> build -> close -> exit completes (usage: rccl_probe.py [torch|notorch|late] [dist])."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "genome-compression_amd"))
mode = sys.argv[1] if len(sys.argv) > 1 else "torch"
if mode == "torch":
    import torch  # noqa: F401
if len(sys.argv) > 2 and sys.argv[2] == "dist":
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("gloo", rank=0, world_size=1)
import numpy as np  # noqa: E402
import gcz  # noqa: E402


def maps():
    with open("/proc/self/maps") as f:
        return sorted({ln.split()[-1] for ln in f if "rccl" in ln})


print("before:", maps(), file=sys.stderr, flush=True)
ctx = gcz.Context(0)
g = gcz.Group.rccl(ctx, 0, 1, gcz.dist_unique_id())
if mode == "late":   # torch (and its own librccl) arrives after ours
    import torch  # noqa: F401,F811
print("after create:", maps(), file=sys.stderr, flush=True)
rng = np.random.default_rng(1)
S, L = 1 << 14, 16
bases = rng.integers(0, 4, S * L, dtype=np.uint8)
buf = ctx.upload(np.frombuffer(b"ACGT", dtype=np.uint8)[bases])
g.build_device_bases([buf.ptr], S, L)
print("built", gcz.digest(g.tree()) is not None, file=sys.stderr, flush=True)
buf.free()
g.close()
print("closed group", file=sys.stderr, flush=True)
ctx.close()
print("closed ctx", file=sys.stderr, flush=True)
