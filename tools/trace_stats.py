#!/usr/bin/env python3
"""Per (kernel, grid) launch statistics from a rocprofv3 --kernel-trace CSV:
calls, average / median / min duration. The search kernel runs once per level
with a different grid per level, so rocprof's per-name --stats average mixes
levels; this table separates them (the bench roofline's finest-level launch is
the k_search8 row with the largest grid)."""
import collections
import csv
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        d[(r["Kernel_Name"], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for (name, grid), v in d.items():
        v.sort()
        rows.append((name, grid, len(v), sum(v) / len(v), v[len(v) // 2], v[0], sum(v)))
    rows.sort(key=lambda r: -r[6])
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Grid_Threads", "Calls", "Average_us", "Median_us", "Min_us", "Total_us"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], f"{r[3]:.1f}", f"{r[4]:.1f}", f"{r[5]:.1f}", f"{r[6]:.1f}"])
            print(f"{r[0][:48]:48s} grid {r[1]:9d} calls {r[2]:4d} avg {r[3]:8.1f} us  median {r[4]:8.1f} us")


if __name__ == "__main__":
    main()
