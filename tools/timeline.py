#!/usr/bin/env python3
"""Print the kernel timeline of one step from a rocprofv3 kernel-trace CSV
(step = the launches from the K-th pyramid launch of queue-order), relative
to that step's first launch: name, grid, queue, start, end, duration (us)."""
import csv
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 24
    rows = [r for r in csv.DictReader(open(path)) if "copyBuffer" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    pyr = [i for i, r in enumerate(rows) if "pyramid" in r["Kernel_Name"] or "k_pyr12" in r["Kernel_Name"]]
    i0 = pyr[min(k, len(pyr) - 1)]
    t0 = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:i0 + n]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        print(f"{r['Kernel_Name'][10:28]:18s} grid {g:8d} q{r['Queue_Id']:>3s} {s:8.1f} -> {e:8.1f} ({e - s:7.1f})")


if __name__ == "__main__":
    main()
