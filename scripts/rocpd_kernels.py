#!/usr/bin/env python3
"""Per-kernel dispatch list from a rocprofv3 SQLite database (rocprofv3 -o x -> x_results.db):
   python scripts/rocpd_kernels.py <db> [--build N] [--stats]
--stats: kernel name, calls, total/avg us (like --stats' kernel_stats.csv); default: the dispatch
sequence (start offset us, duration us, name) of the last N dispatches."""
import sqlite3
import sys


def main():
    args = sys.argv[1:]
    db = sqlite3.connect(args[0])
    rows = db.execute("select start, end, name from kernels order by start").fetchall()
    if "--stats" in args:
        agg = {}
        for s, e, n in rows:
            a = agg.setdefault(n, [0, 0])
            a[0] += 1
            a[1] += (e - s) / 1e3
        for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{c:6d} {t:12.1f} {t / c:10.2f}  {n[:110]}")
        return
    n = int(args[args.index("--build") + 1]) if "--build" in args else len(rows)
    rows = rows[-n:]
    t0 = rows[0][0]
    for s, e, name in rows:
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.2f}  {name[:100]}")


if __name__ == "__main__":
    main()
