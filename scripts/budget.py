#!/usr/bin/env python3
"""Exchange budget of the multi-rank build from a virtual-rank bench line.

    python scripts/budget.py <bench --virtual R json> [single-GPU ms per Gbase] [--weak] [--link GB/s ...]

(--weak: the line is a weak-scaled probe, e.g. uniform_8g over 8 ranks = 1 Gbase per rank; the
projected speedup is then genome Gbase x single-GPU ms / T_R, else single-GPU ms / T_R.)

A `bench.py --virtual R` line carries each rank's kernel time (`rank_kernel_ms`, the device
work of that rank alone -- on R GPUs the ranks run concurrently) and its exchange log
(`rank_timeline[r].exchange_log`: every collective's name and the bytes the rank sent /
received).  The projection for R GPUs of one node:

    T_R = max_r kernel_ms_r  +  sum over collectives (latency + bytes over the busiest link / B)
          + host syncs x t_sync

with the busiest link's bytes = max over ranks of max(sent, received) / (R - 1) (every pair
of GPUs has its own xGMI link; all-to-alls and allgathers spread evenly over the R - 1 links;
the gather to rank 0 loads rank 0's links).  Latency and t_sync are assumed, not measured
(RCCL at world > 1 has not run on this project's one-GPU boxes): 25 us per collective and
15 us per host round trip; link bandwidths 50 and 100 GB/s per direction are shown."""
import json
import sys


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
    lat_us, sync_us = 25.0, 15.0
    syncs = {"leaf r-first counts + bucket prefixes", "owner counts", "leaf owner counts", "first counts + C/D sizes",
             "final vectors", "leaf dictionary size"}
    # the fused schedule (gcz_dist_fast.h): one collective group per row; its mid-build read
    # waits on an event behind R1 (the r-first work stays queued behind it) -- counted as a sync
    is_sync = lambda name: name in syncs or name.startswith("R1a ")  # noqa: E731
    rows = []
    for k in range(n):
        name = logs[0][k][1]
        busiest = max(max(lg[k][2], lg[k][3]) for lg in logs) / max(1, R - 1)
        rows.append((k, name, busiest, is_sync(name)))
    print(f"R = {R}, config {d['config']['workload']}: slowest rank's kernels {kern:.3f} ms "
          f"(ranks {min(d['rank_kernel_ms']):.3f}-{kern:.3f})")
    print(f"{'#':>2} {'collective':60s} {'busiest link MB':>16s} {'host sync':>9s}")
    for k, name, b, s in rows:
        print(f"{k:2d} {name:60s} {b / 1e6:16.3f} {'yes' if s else '':>9s}")
    nsync = sum(1 for r in rows if r[3])
    for B in links:
        xfer = sum(b for _, _, b, _ in rows) / (B * 1e9) * 1e3
        lat = n * lat_us / 1e3 + nsync * sync_us / 1e3
        T = kern + xfer + lat
        line = (f"B = {B:.0f} GB/s: kernels {kern:.3f} + transfers {xfer:.3f} + {n} collectives / {nsync} syncs "
                f"{lat:.3f} = {T:.3f} ms")
        if single:
            gb = d["config"]["nbases"] / 1e9
            line += (f" -> {single * gb / T:.2f}x ({gb:.0f} Gbase at {single} ms per Gbase on one GPU)" if weak
                     else f" -> {single / T:.2f}x of {single} ms on one GPU")
        print(line)


if __name__ == "__main__":
    main()
