"""The N > 1 bench path as real processes on one GPU.

`python -m torch.distributed.run --nproc-per-node N bench.py` is exactly what the
driver runs on an 8-GPU node; here every rank shares GPU 0 and the exchanges go
through the host-staged shared-memory transport (--transport shm; RCCL refuses two
ranks on one device).  Everything else is the production multi-rank path: one
process and context per rank, the strong-scaled headline (uniform_100m split over
the ranks), the per-level owner exchange, the streamed rank-slice parity digest
over gloo, and the weak-scaled timing (N x uniform_100m) on the same group.  Both
must match the reference goldens (synth/uniform_100000003 and
uniform_{200000006,300000009}).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_bench_multiprocess_shm(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--transport", "shm", "--shm-region-mb", "256", "--config", "uniform_100m", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-4000:]
    d = json.loads(lines[-1])
    assert d["n_gpus"] == world and d["scaling"] == "strong" and d["value"] > 0
    assert d["config"]["nbases"] == 100_000_003
    par = d["parity"]
    assert par["golden"] == "synth/uniform_100000003"
    for k in ("layers_sha256_match", "leaves_sha256_match", "root_match", "layer_sizes_match"):
        assert par[k] is True, (k, par)
    wk = d["weak_scaling"]
    assert "error" not in wk, wk
    assert wk["golden"] == f"synth/uniform_{world * 100_000_003}"
    assert wk["nbases"] == world * 100_000_003 // 12 * 12
    assert wk["layer_sizes_match"] and wk["root_match"], wk


@pytest.mark.gpu
def test_bench_rccl_world1():
    """The RCCL group path in one process (bench.py --rccl-world1): our librccl is
    dlopen'd before torch loads its own copy; the process must also EXIT cleanly
    (both copies resident: RTLD_GLOBAL once made their destructors double-free)."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--rccl-world1", "--config", "uniform_100m",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-4000:]
    d = json.loads(lines[-1])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["config"]["parallelism"].endswith("over rccl"), d["config"]["parallelism"]
    par = d["parity"]
    for k in ("layers_sha256_match", "leaves_sha256_match", "root_match", "layer_sizes_match"):
        assert par[k] is True, (k, par)
    assert d["weak_scaling"] is None


@pytest.mark.gpu
def test_bench_multiprocess_stalled_rank_is_bounded():
    """A rank that stalls before an exchange (GCZ_DIST_STALL = rank:seq:seconds) must not hold
    the job: its peer leaves that exchange after GCZ_DIST_TIMEOUT_S, the run exits non-zero and
    the error names the exchange (sequence number and name) -- the diagnosis an 8-GPU run that
    hangs in RCCL gets from the watchdog (same exchange numbering, gcz_group::Watch)."""
    import time
    env = dict(os.environ, GCZ_DIST_STALL="1:2:60", GCZ_DIST_TIMEOUT_S="6")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--transport", "shm", "--shm-region-mb", "256", "--config", "uniform_100m", "--steps", "1",
           "--warmup", "0", "--no-cpu-baseline", "--no-parity", "--no-weak"]
    t0 = time.monotonic()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=200, cwd=REPO, env=env)
    dt = time.monotonic() - t0
    out = p.stdout + p.stderr
    assert p.returncode != 0, out[-3000:]
    assert dt < 150, dt
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, out[-3000:]
    err = json.loads(lines[-1]).get("error", "")
    assert "collective #2" in err and "R1b leaf presence bitmaps" in err, err
    assert "no peer arrived within 6 s" in err, err
