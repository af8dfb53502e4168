#!/usr/bin/env python3
"""Exchange budget of the multi-rank build from a virtual-rank bench line.

    python scripts/budget.py <bench --virtual R json> [single-GPU ms per Gbase] [--weak] [--link GB/s ...]

(--weak: the line is a weak-scaled probe, e.g. uniform_8g over 8 ranks = 1 Gbase per rank; the
projected speedup is then genome Gbase x single-GPU ms / T_R, else single-GPU ms / T_R.)

A `bench.py --virtual R` line carries each rank's kernel time (`rank_kernel_ms`, the device
work of that rank alone -- on R GPUs the ranks run concurrently) and its exchange log
(`rank_timeline[r].exchange_log`: every collective's name and the bytes the rank sent /
received).  Two projections for R GPUs of one node:

additive (every schedule): nothing overlaps --

    T_R = max_r kernel_ms_r  +  sum over collectives (latency + bytes over the busiest link / B)
          + host syncs x t_sync

overlap (the fused schedule, gcz_group::build_fast): the line also carries each rank's compute
segments (`rank_timeline[r].segments_ms`, kernel time between the schedule's fl_mark points
C1 .. C8 and the tail after C8), and the model replays the schedule's dependencies:

    C1 C2 [bulk mark] | R1a | C3 | (host: R1a + t_sync) R1b | C4 | R2 | (wait K2) C5 | R3 | C6 | R4 |
    C7 | R5 | C8 tail | top gather | final vectors | t_sync

A collective starts when every rank has reached it (its end is common to all ranks); K2, the
layer-0 keys' all-to-all, runs on the bulk stream from max(every rank's C2 end, the host's
read of R1a) and shares the links with whatever collective is moving bytes at the same time
(processor sharing: two transfers in flight get B / 2 each).  Compute of one rank is not slowed
by RCCL's kernels in this model.

The busiest link's bytes = max over ranks of max(sent, received) / (R - 1) (every pair of GPUs
has its own xGMI link; all-to-alls and allgathers spread evenly over the R - 1 links; the gather
to rank 0 loads rank 0's links).  Latency and t_sync are assumed, not measured (RCCL at
world > 1 has not run on this project's one-GPU boxes): 25 us per collective and 15 us per host
round trip; link bandwidths 50 and 100 GB/s per direction are shown."""
import json
import sys

LAT_US, SYNC_US = 25.0, 15.0
FUSED = ["R1a", "K2", "R1b", "R2", "R3", "R4", "R5", "top words to rank 0", "final vectors"]


def busiest_bytes(logs, R):
    n = len(logs[0])
    return [max(max(lg[k][2], lg[k][3]) for lg in logs) / max(1, R - 1) for k in range(n)]


class Bulk:
    """The one transfer on the bulk stream (K2): latency, then bytes at the link's rate, shared
    equally with a concurrent transfer on the build's stream."""

    def __init__(self, start_s, lat_s, nbytes):
        self.t = start_s + lat_s   # bytes start moving here
        self.rem = nbytes
        self.end = start_s + lat_s if nbytes == 0 else None

    def alone(self, until, B):
        """Progress with the links to itself up to time `until`."""
        if self.end is not None or until <= self.t:
            return
        dt = until - self.t
        if self.rem <= dt * B:
            self.end = self.t + self.rem / B
            self.rem = 0.0
        else:
            self.rem -= dt * B
        self.t = until

    def finish(self, B):
        if self.end is None:
            self.alone(float("inf"), B)
        return self.end


def transfer(t0, lat_s, nbytes, B, bulk):
    """A build-stream collective from t0; returns its end (sharing the links with `bulk`)."""
    t = t0 + lat_s
    rem = nbytes
    if bulk is not None:
        bulk.alone(t, B)
    while rem > 1e-9:
        if bulk is not None and bulk.end is None and bulk.t <= t:
            dt = min(rem / (B / 2), bulk.rem / (B / 2))
            rem -= dt * B / 2
            bulk.rem -= dt * B / 2
            t += dt
            bulk.t = t
            if bulk.rem <= 1e-9:
                bulk.end = t
                bulk.rem = 0.0
        elif bulk is not None and bulk.end is None:   # bulk not moving bytes yet
            dt = min(rem / B, bulk.t - t)
            rem -= dt * B
            t += dt
        else:
            t += rem / B
            rem = 0.0
    return t


def overlap_model(segs, names, xb, B, verbose=False):
    """Replay the fused schedule; returns (T seconds, event list)."""
    R = len(segs)
    idx = {}
    for k, nm in enumerate(names):
        for f in FUSED:
            if nm == f or nm.startswith(f + " "):
                idx[f] = k
    lat, sync = LAT_US * 1e-6, SYNC_US * 1e-6
    ready = [0.0] * R
    ev = []

    def comp(i):
        for r in range(R):
            ready[r] += segs[r][i] * 1e-3

    def coll(f, bulk, not_before=0.0):
        t0 = max(max(ready), not_before)
        t1 = transfer(t0, lat, xb[idx[f]], B, bulk)
        ev.append((f, t0, t1))
        for r in range(R):
            ready[r] = t1
        return t1

    comp(0)
    comp(1)
    c2_end = max(ready)
    r1a = coll("R1a", None)
    host = r1a + sync                      # the mid-build read
    bulk = Bulk(max(c2_end, host), lat, xb[idx["K2"]])
    comp(2)
    coll("R1b", bulk, host)
    comp(3)
    coll("R2", bulk)
    k2 = bulk.finish(B)
    ev.append(("K2 (bulk)", max(c2_end, host), k2))
    for r in range(R):
        ready[r] = max(ready[r], k2)
    comp(4)
    coll("R3", None)
    comp(5)
    coll("R4", None)
    comp(6)
    coll("R5", None)
    comp(7)
    comp(8)
    coll("top words to rank 0", None)
    t = coll("final vectors", None) + sync
    return t, ev


def main():
    args = sys.argv[1:]
    weak = "--weak" in args
    args = [a for a in args if a != "--weak"]
    links = [50.0, 100.0]
    if "--link" in args:
        i = args.index("--link")
        links = [float(x) for x in args[i + 1:]]
        args = args[:i]
    d = json.loads(open(args[0]).read().strip().splitlines()[-1])
    single = float(args[1]) if len(args) > 1 else None
    tl = d["rank_timeline"]
    R = len(tl)
    kern = max(d["rank_kernel_ms"])
    logs = [r.get("exchange_log") or [] for r in tl]
    n = len(logs[0])
    syncs = {"leaf r-first counts + bucket prefixes", "owner counts", "leaf owner counts", "first counts + C/D sizes",
             "final vectors", "leaf dictionary size"}
    # the fused schedule: its mid-build read waits on an event behind R1a
    is_sync = lambda name: name in syncs or name.startswith("R1a ")  # noqa: E731
    xb = busiest_bytes(logs, R)
    names = [logs[0][k][1] for k in range(n)]
    print(f"R = {R}, config {d['config']['workload']}: slowest rank's kernels {kern:.3f} ms "
          f"(ranks {min(d['rank_kernel_ms']):.3f}-{kern:.3f})")
    print(f"{'#':>2} {'collective':64s} {'busiest link MB':>16s} {'host sync':>9s}")
    for k in range(n):
        print(f"{k:2d} {names[k]:64s} {xb[k] / 1e6:16.3f} {'yes' if is_sync(names[k]) else '':>9s}")
    nsync = sum(1 for nm in names if is_sync(nm))

    def speedup(T):
        if not single:
            return ""
        gb = d["config"]["nbases"] / 1e9
        return (f" -> {single * gb / T:.2f}x ({gb:.0f} Gbase at {single} ms per Gbase on one GPU)" if weak
                else f" -> {single / T:.2f}x of {single} ms on one GPU")

    for B in links:
        xfer = sum(xb) / (B * 1e9) * 1e3
        lat = n * LAT_US / 1e3 + nsync * SYNC_US / 1e3
        T = kern + xfer + lat
        print(f"additive, B = {B:.0f} GB/s: kernels {kern:.3f} + transfers {xfer:.3f} + {n} collectives / {nsync} syncs "
              f"{lat:.3f} = {T:.3f} ms" + speedup(T))
    segs = [r.get("segments_ms") for r in tl]
    fused = all(s is not None and len(s) == 9 for s in segs) and all(
        any(nm == f or nm.startswith(f + " ") for nm in names) for f in FUSED)
    if not fused:
        return
    print("segments (ms) per rank, C1 .. C8, tail:")
    for r, s in enumerate(segs):
        print(f"  rank {r}: " + " ".join(f"{x:.3f}" for x in s))
    for B in links:
        T, ev = overlap_model(segs, names, xb, B * 1e9)
        print(f"overlap, B = {B:.0f} GB/s: {T * 1e3:.3f} ms" + speedup(T * 1e3))
        print("   " + ", ".join(f"{f.split(' ')[0]} {t0 * 1e3:.3f}-{t1 * 1e3:.3f}" for f, t0, t1 in ev))


if __name__ == "__main__":
    main()
