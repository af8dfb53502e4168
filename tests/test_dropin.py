"""The rebuilt C++ surface (include/dna.h, fasta_reader.h, shared_tree.h) and the
compress CLI, compiled against libgcz like a reference user's code would be."""
import hashlib
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, PKG, REPO, load_gcz

BIN = os.path.join(REPO, "tests", "cxx", "test_dropin")


def build_test_binary():
    load_gcz()   # makes sure libgcz.so exists
    src = os.path.join(REPO, "tests", "cxx", "test_dropin.cpp")
    deps = [src, os.path.join(PKG, "libgcz.so")] + [os.path.join(REPO, "include", h)
                                                    for h in ("dna.h", "fasta_reader.h", "shared_tree.h", "gcz.h")]
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(d) for d in deps):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-I" + os.path.join(REPO, "include"), src,
                        "-o", BIN, "-L" + PKG, "-lgcz", "-Wl,-rpath," + PKG], check=True)
    return BIN


def test_dropin_host_groups():
    r = subprocess.run([build_test_binary(), GOLDEN], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_dropin_gpu_groups():
    r = subprocess.run([build_test_binary(), GOLDEN, "gpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def _compress(args, cwd):
    exe = os.path.join(PKG, "compress")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", PKG], check=True)
    return subprocess.run([exe] + args, capture_output=True, text=True, cwd=cwd)


def test_compress_cli_usage(tmp_path):
    r = _compress([], str(tmp_path))
    assert r.returncode == 2 and "argument <file> required" in r.stdout
    r = _compress(["--help"], str(tmp_path))
    assert r.returncode == 0 and r.stdout.startswith("Usage: compress")
    r = _compress(["--verbose", "--statistics", "x"], str(tmp_path))
    assert r.returncode == 2 and "mutually exclusive" in r.stdout
    r = _compress(["a", "b"], str(tmp_path))
    assert r.returncode == 1 and "multiple files" in r.stdout
    r = _compress([str(tmp_path / "missing")], str(tmp_path))
    assert r.returncode == 2 and "Invalid filename" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["chmpxx", "edited", "hehcmv", "merged", "humdyst"])
def test_compress_cli_matches_reference(name, tmp_path, manifest):
    exp = manifest[f"corpus/{name}"]["expect"]
    src = os.path.join(GOLDEN, "data", name)
    out = tmp_path / f"{name}.dag"
    r = _compress(["--statistics", f"--output={out}", src], str(tmp_path))
    assert r.returncode == 0, r.stderr
    f = r.stdout.strip().split(",")
    # dna_size,width,ratio,original,compressed,t_build,t_sort,t_total (compress.cpp:71-79)
    assert f[0] == "12" and int(f[1]) == exp["width"] and f[2] == exp["ratio"]
    assert int(f[3]) == exp["file_size"] and int(f[4]) == exp["bytes"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == exp["sha_dag"]


@pytest.mark.gpu
def test_compress_cli_errors(tmp_path, manifest):
    exp = manifest["fasta/crlf"]["expect"]
    r = _compress(["--no-save", os.path.join(GOLDEN, "fasta", "crlf.fa")], str(tmp_path))
    assert r.returncode == 1 and r.stderr.strip() == exp["stderr"]


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [2, 3])
@pytest.mark.parametrize("name", ["chmpxx", "merged"])
def test_compress_cli_gpus(name, gpus, tmp_path, manifest):
    """compress --gpus=N (shared_tree_on_gpus): N processes, one rank each; on the one-GPU
    box every rank shares the device and exchanges host-staged (GCZ_MULTI_TRANSPORT=shm).
    Same .dag and statistics as the reference."""
    exp = manifest[f"corpus/{name}"]["expect"]
    out = tmp_path / f"{name}.dag"
    env = dict(os.environ, GCZ_MULTI_TRANSPORT="shm")
    exe = os.path.join(PKG, "compress")
    r = subprocess.run([exe, "--statistics", f"--gpus={gpus}", f"--output={out}", os.path.join(GOLDEN, "data", name)],
                       capture_output=True, text=True, cwd=str(tmp_path), env=env, timeout=240)
    assert r.returncode == 0, r.stderr
    f = r.stdout.strip().split(",")
    assert int(f[1]) == exp["width"] and f[2] == exp["ratio"] and int(f[4]) == exp["bytes"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == exp["sha_dag"]


@pytest.mark.gpu
def test_compress_cli_gpus_errors(tmp_path, manifest):
    exp = manifest["fasta/bad_symbol"]["expect"]
    env = dict(os.environ, GCZ_MULTI_TRANSPORT="shm")
    r = subprocess.run([os.path.join(PKG, "compress"), "--no-save", "--gpus=2",
                        os.path.join(GOLDEN, "fasta", "bad_symbol.fa")], capture_output=True, text=True,
                       cwd=str(tmp_path), env=env, timeout=240)
    assert r.returncode == 1 and r.stderr.strip() == exp["stderr"]
