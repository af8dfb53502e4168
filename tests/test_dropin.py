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


@pytest.mark.gpu
def test_dropin_reader_exhausted():
    """tree_constructor::reduce on a reader whose every buffer was read: libgcz's error, exit 1."""
    r = subprocess.run([build_test_binary(), GOLDEN, "exhausted"], capture_output=True, text=True)
    assert r.returncode == 1, r.stdout + r.stderr
    assert "every reader buffer was already read" in r.stderr


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
    Same .dag and statistics as the reference; the tree is gathered device to device into rank
    0's context (gcz_group_assemble), so the frequency sort runs on the GPU (GCZ_TIMING phase)."""
    exp = manifest[f"corpus/{name}"]["expect"]
    out = tmp_path / f"{name}.dag"
    env = dict(os.environ, GCZ_MULTI_TRANSPORT="shm", GCZ_TIMING="1")
    exe = os.path.join(PKG, "compress")
    r = subprocess.run([exe, "--statistics", f"--gpus={gpus}", f"--output={out}", os.path.join(GOLDEN, "data", name)],
                       capture_output=True, text=True, cwd=str(tmp_path), env=env, timeout=240)
    assert r.returncode == 0, r.stderr
    f = r.stdout.strip().split(",")
    assert int(f[1]) == exp["width"] and f[2] == exp["ratio"] and int(f[4]) == exp["bytes"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == exp["sha_dag"]
    assert "gcz-time device-sort" in r.stderr, r.stderr


@pytest.mark.gpu
def test_compress_cli_gpus_errors(tmp_path, manifest):
    exp = manifest["fasta/bad_symbol"]["expect"]
    env = dict(os.environ, GCZ_MULTI_TRANSPORT="shm")
    r = subprocess.run([os.path.join(PKG, "compress"), "--no-save", "--gpus=2",
                        os.path.join(GOLDEN, "fasta", "bad_symbol.fa")], capture_output=True, text=True,
                       cwd=str(tmp_path), env=env, timeout=240)
    assert r.returncode == 1 and r.stderr.strip() == exp["stderr"]


# ---- the reference's own callers on the drop-in (include/utility.h, oracle/Makefile dropin) ----

REF = "/root/reference"
DROPIN_COMPRESS = os.path.join(REPO, "oracle", "_ref", "dropin_compress")
DROPIN_TEST = os.path.join(REPO, "oracle", "_ref", "dropin_test")


def test_utility_matches_reference(tmp_path):
    """include/utility.h (our restatement) gives the reference utility.h's results on every
    helper: compiled against both when /root/reference exists, otherwise against the output
    the reference's header produced (tests/golden/utility_check.txt, same program)."""
    src = os.path.join(REPO, "tests", "cxx", "utility_check.cpp")

    def run(inc, name):
        exe = str(tmp_path / name)
        subprocess.run(["g++", "-std=c++17", "-O1", "-w", "-I" + inc, src, "-o", exe], check=True)
        return subprocess.run([exe], capture_output=True, text=True, check=True).stdout

    ours = run(os.path.join(REPO, "include"), "ours")
    with open(os.path.join(GOLDEN, "utility_check.txt")) as f:
        assert ours == f.read()
    if os.path.isdir(os.path.join(REF, "include")):
        assert ours == run(os.path.join(REF, "include"), "ref")


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference sources")
def test_reference_callers_compile():
    """The reference's unmodified compress.cpp and tests/test.cpp compile against include/
    and link to libgcz.so; the CLI's host-only paths behave."""
    load_gcz()
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "dropin"], check=True)
    r = subprocess.run([DROPIN_COMPRESS, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("Usage: compress")
    r = subprocess.run([DROPIN_COMPRESS], capture_output=True, text=True)
    assert r.returncode == 2 and "argument <file> required" in r.stdout
    r = subprocess.run([DROPIN_COMPRESS, "/nonexistent/x"], capture_output=True, text=True)
    assert r.returncode == 2 and "Invalid filename" in r.stdout


@pytest.mark.gpu
def test_reference_test_program_on_dropin():
    """The reference's own test program (tests/test.cpp, every group) built on the drop-in
    runs green on the GPU (it reads data/edited and data/chmpxx relative to its cwd)."""
    if not os.path.exists(DROPIN_TEST):
        pytest.skip("oracle/_ref/dropin_test not built (needs /root/reference at build time)")
    r = subprocess.run([DROPIN_TEST], capture_output=True, text=True, cwd=GOLDEN, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    assert out.count("Finished without errors") == 10 and "error" not in out.replace("without errors", ""), out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["chmpxx", "merged"])
def test_reference_compress_on_dropin(name, tmp_path, manifest):
    """The reference's own compress.cpp on the drop-in: same statistics and .dag bytes."""
    if not os.path.exists(DROPIN_COMPRESS):
        pytest.skip("oracle/_ref/dropin_compress not built (needs /root/reference at build time)")
    exp = manifest[f"corpus/{name}"]["expect"]
    out = tmp_path / f"{name}.dag"
    r = subprocess.run([DROPIN_COMPRESS, "--statistics", f"--output={out}", os.path.join(GOLDEN, "data", name)],
                       capture_output=True, text=True, cwd=str(tmp_path), timeout=300)
    assert r.returncode == 0, r.stderr
    f = r.stdout.strip().split(",")
    assert f[0] == "12" and int(f[1]) == exp["width"] and f[2] == exp["ratio"] and int(f[4]) == exp["bytes"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == exp["sha_dag"]


def test_compress_cli_gpus_over_rank_limit(tmp_path):
    """--gpus beyond the multi-rank build's 31 ranks is refused up front (no device touched)."""
    r = _compress(["--no-save", "--gpus=40", os.path.join(GOLDEN, "data", "chmpxx")], str(tmp_path))
    assert r.returncode == 1 and "more than the 31 ranks" in r.stderr


@pytest.mark.gpu
def test_compress_cli_gpus_failing_rank_ends_job(tmp_path):
    """A rank that cannot start (here: a device index past the box's GPUs, RCCL transport) ends
    the whole job with exit 1 instead of leaving the other ranks blocked in RCCL."""
    import time
    env = dict(os.environ, GCZ_DEVICE="0", HIP_VISIBLE_DEVICES="0")   # one visible GPU: rank 1 has none
    env.pop("GCZ_MULTI_TRANSPORT", None)
    t0 = time.time()
    r = subprocess.run([os.path.join(PKG, "compress"), "--no-save", "--gpus=2",
                        os.path.join(GOLDEN, "data", "chmpxx")], capture_output=True, text=True,
                       cwd=str(tmp_path), env=env, timeout=180)
    assert r.returncode == 1, r.stderr
    assert "failed" in r.stderr
    assert time.time() - t0 < 170
