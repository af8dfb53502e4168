"""Per-kernel durations of one build from a rocprofv3 --kernel-trace CSV (the second-last
build in the file): python scripts/trace_build.py <kernel_trace.csv>."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_build_init" in r["Kernel_Name"]]
b = starts[-2]
end = next(i for i in range(b, len(rows)) if any(x in rows[i]["Kernel_Name"] for x in ("k_tail", "k_build_finish")))
tot = 0
for r in rows[b:end + 1]:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot += d
    print(f"{d / 1000:7.2f} us  {r['Kernel_Name'].replace('gcz_dev::', '')[:80]}")
print(f"sum of kernel durations: {tot / 1000:.2f} us over {end + 1 - b} kernels")
