#!/usr/bin/env python3
"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes of a bench.py run into HBM
bytes per launch per kernel (and launch grid), and write the finest-level
search launch's figure (the k_search8 launch with the largest grid) to
profiles/traffic.json (read by bench.py as `roofline.traffic`).

Correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE on gfx950 counts
half the bytes read; calibrated here with tools/pmc_calib for 1-, 4- and 16-B
loads alike (r01: 262150 KiB reported for a 524288 KiB read), so bytes =
2 * FETCH_SIZE * 1024; WRITE_SIZE is exact (524288 KiB for 524288 KiB).
"""
import argparse
import collections
import csv
import json


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = f'{r["Kernel_Name"]} grid={r["Grid_Size"]}'
        tot[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: (tot[k] / len(disp[k]), len(disp[k])) for k in tot}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--out", required=True)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--preset", default="medium")
    a = ap.parse_args()
    f = per_kernel(a.fetch_csv, "FETCH_SIZE")
    w = per_kernel(a.write_csv, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        fk, n = f.get(k, (0.0, 0))
        wk, _ = w.get(k, (0.0, 0))
        kernels[k] = {"launches": n, "fetch_kib": fk, "write_kib": wk,
                      "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024}
    search = sorted((k for k in kernels if "k_search8" in k), key=lambda k: -int(k.rsplit("=", 1)[1]))
    out = {"batch": a.batch, "width": a.width, "height": a.height, "preset": a.preset,
           "kernel": (search[0] + " (finest level)") if search else None,
           "hbm_bytes_per_launch": kernels[search[0]]["hbm_bytes_per_launch"] if search else None,
           "correction": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE counts half the bytes; "
                         "calibrated with tools/pmc_calib for 1/4/16-B loads)",
           "kernels": kernels}
    json.dump(out, open(a.out, "w"), indent=1)
    for k, v in kernels.items():
        print(f"{k[:72]:72s} launches {v['launches']:3d}  HBM MB/launch {v['hbm_bytes_per_launch'] / 1e6:9.2f}")


if __name__ == "__main__":
    main()
