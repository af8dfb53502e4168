"""Probe: where does the RCCL world-1 bench path abort at teardown?"""
import faulthandler
import importlib.util
import os
import sys

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("gcz", os.path.join(REPO, "genome-compression_amd", "gcz.py"))
gcz = importlib.util.module_from_spec(spec)
sys.modules["gcz"] = gcz
spec.loader.exec_module(gcz)


def step(msg):
    print("STEP", msg, flush=True)


profile = "--profile" in sys.argv
n = 12_000_000
ctx = gcz.Context(0)
host = gcz.synth(0, n)
dev = ctx.upload(host)
step("uploaded")
g = gcz.Group.rccl(ctx, 0, 1, gcz.dist_unique_id())
step("group")
for i in range(3):
    g.build_device_bases([dev.ptr], n // 12, 12)
step("built")
if profile:
    ctx.profile(True)
    ctx.profile_reset()
    g.build_device_bases([dev.ptr], n // 12, 12)
    print(ctx.profile_table(), flush=True)
    ctx.profile(False)
    step("profiled")
for layer in range(-1, g.info()["n_layers"]):
    g.copy_slice(0, layer)
step("copied slices")
dev.free()
step("dev freed")
g.close()
step("group closed")
ctx.close()
step("ctx closed")
