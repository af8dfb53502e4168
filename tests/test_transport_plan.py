"""The RCCL transport's point-to-point arithmetic (gcz_dist_p2p_plan / gcz_dist_gather_plan:
the exact offsets and byte counts RcclTransport passes to ncclSend / ncclRecv) at world > 1,
on the CPU.  Each rank's plan is executed as matched point-to-point copies between simulated
rank buffers and the result must equal the transport contract every transport implements
(gcz_dist.hip Transport: rank d's receive buffer holds rank s's segment for d at its receive
displacement) -- the layout the virtual-rank and shm transports, which the GPU parity tests
run, produce.  RCCL itself has never run at world > 1 on this project's one-GPU test boxes;
this pins everything of it but the library calls."""
import numpy as np
import pytest


def _contract(M, R, rev, elem, send, sd, rd, rsize):
    """recv[d][rd(d,s)] = send[s][sd(s,d)], count(s,d) elements; Python restatement."""
    cnt = (lambda s, d: M[d, s]) if rev else (lambda s, d: M[s, d])
    if sd is None:
        sd = np.zeros((R, R), np.uint64)
        for s in range(R):
            o = 0
            for d in range(R):
                sd[s, d] = o
                o += cnt(s, d)
    if rd is None:
        rd = np.zeros((R, R), np.uint64)
        for d in range(R):
            o = 0
            for s in range(R):
                rd[d, s] = o
                o += cnt(s, d)
    recv = [np.zeros(rsize[d], np.uint8) for d in range(R)]
    for s in range(R):
        for d in range(R):
            n = int(cnt(s, d)) * elem
            a, b = int(sd[s, d]) * elem, int(rd[d, s]) * elem
            recv[d][b:b + n] = send[s][a:a + n]
    return recv


def _execute(gcz, M, R, rev, elem, send, sd, rd, rsize):
    """Every rank's plan as matched point-to-point transfers."""
    plans = [gcz.p2p_plan(R, me, M, rev, elem, sd, rd) for me in range(R)]
    recv = [np.zeros(rsize[d], np.uint8) for d in range(R)]
    for me in range(R):
        for q in range(R):
            so, sb, _, _, peer = (int(x) for x in plans[me][q])
            assert peer == q
            ro, rb = int(plans[q][me][2]), int(plans[q][me][3])
            assert sb == rb, (me, q, sb, rb)          # what me sends to q is what q expects from me
            recv[q][ro:ro + rb] = send[me][so:so + sb]
    return recv


@pytest.mark.parametrize("R", [2, 3, 5, 8, 16, 31])
@pytest.mark.parametrize("rev", [False, True])
@pytest.mark.parametrize("explicit", [False, True])
def test_p2p_plan_matches_transport_contract(gcz, R, rev, explicit):
    rng = np.random.default_rng(R * 4 + 2 * rev + explicit)
    for elem in (1, 4, 8):
        M = rng.integers(0, 50, size=(R, R)).astype(np.uint64)
        M[rng.random((R, R)) < 0.3] = 0                        # empty segments, incl. self ones
        cnt = M.T if rev else M                                # cnt[s, d]
        sd = rd = None
        ssize = [int(cnt[s].sum()) * elem for s in range(R)]
        rsize = [int(cnt[:, d].sum()) * elem for d in range(R)]
        if explicit:                                           # segments at shuffled places, with gaps
            sd = np.zeros((R, R), np.uint64)
            rd = np.zeros((R, R), np.uint64)
            for s in range(R):
                o = 0
                for d in rng.permutation(R):
                    o += int(rng.integers(0, 5))
                    sd[s, d] = o
                    o += int(cnt[s, d])
                ssize[s] = (o + 3) * elem
            for d in range(R):
                o = 0
                for s in rng.permutation(R):
                    o += int(rng.integers(0, 5))
                    rd[d, s] = o
                    o += int(cnt[s, d])
                rsize[d] = (o + 3) * elem
        send = [rng.integers(0, 256, size=ssize[s], dtype=np.uint8) for s in range(R)]
        want = _contract(M, R, rev, elem, send, sd, rd, rsize)
        got = _execute(gcz, M, R, rev, elem, send, sd, rd, rsize)
        for d in range(R):
            assert np.array_equal(got[d], want[d]), (R, rev, explicit, elem, d)


@pytest.mark.parametrize("R", [2, 4, 8, 31])
def test_gather_plan_concatenates_in_rank_order(gcz, R):
    rng = np.random.default_rng(R)
    elem = 4
    cnt = rng.integers(0, 100, size=R).astype(np.uint64)
    cnt[rng.random(R) < 0.25] = 0
    send = [rng.integers(0, 256, size=int(cnt[s]) * elem, dtype=np.uint8) for s in range(R)]
    recv0 = np.zeros(int(cnt.sum()) * elem, np.uint8)
    plans = [gcz.gather_plan(R, me, cnt, elem) for me in range(R)]
    for me in range(R):
        for q in range(R):
            so, sb, _, rb_me, _ = (int(x) for x in plans[me][q])
            if me != 0:
                assert rb_me == 0                               # only rank 0 receives
            if sb:
                assert q == 0                                   # everything goes to rank 0
                ro, rb = int(plans[0][me][2]), int(plans[0][me][3])
                assert sb == rb
                recv0[ro:ro + rb] = send[me][so:so + sb]
    assert np.array_equal(recv0, np.concatenate(send))


def test_plan_rejects_bad_arguments(gcz):
    with pytest.raises(gcz.GczError):
        gcz.p2p_plan(2, 2, np.zeros(4), False, 1)
    with pytest.raises(gcz.GczError):
        gcz.p2p_plan(40, 0, np.zeros(1600), False, 1)


def _watch_run(build_returns):
    """gcz_dist_watch_selftest in a child process: (exit code, stderr)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = (
        "import ctypes, sys\n"
        f"lib = ctypes.CDLL({os.path.join(here, '..', 'genome-compression_amd', 'libgcz.so')!r})\n"
        f"sys.exit(lib.gcz_dist_watch_selftest(1, 2, {int(build_returns)}))\n")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    return p.returncode, p.stderr


def test_watchdog_spares_a_build_that_returned():
    """after the watchdog fired and the build returned its error (gcz_group::fail),
    the process must outlive the watchdog's grace period and keep its own exit code."""
    rc, err = _watch_run(True)
    assert rc == 0, err
    assert "has not completed within 1 s" in err and "collective #0 selftest" in err
    assert "did not return after the abort" not in err


def test_watchdog_ends_a_build_that_never_returns():
    rc, err = _watch_run(False)
    assert rc == 70, (rc, err)
    assert "did not return after the abort; exiting" in err
