#!/usr/bin/env python3
"""Per-(kernel, grid) summary of rocprofv3 --pmc CSVs: SQ counters (VALU
instructions per wave, cycles per VALU instruction per SIMD, average resident
waves as a fraction of the 16-per-CU slots, wait fractions) and, given the
FETCH_SIZE / WRITE_SIZE passes, HBM bytes per launch.

  pmc_summary.py SQ.csv [--fetch F.csv --write W.csv] [--match k_vr] [--top N]

Units (MI355X, rocprofv3 on gfx950): GRBM_GUI_ACTIVE sums the 8 XCDs' busy
cycles; SQ_WAVE_CYCLES counts resident wave-cycles in units of 4 cycles; so
the average resident waves = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8), out
of 4096 slots (256 CUs x 16). FETCH_SIZE is in KiB with the gfx950 x2
correction of profiles/traffic.json (tools/pmc_traffic.py), WRITE_SIZE in KiB."""
import argparse
import collections
import csv


def load(path, match):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ids = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if match and match not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"], int(r["Grid_Size"]))
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ids[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(ids[k]) for c, v in d.items()} | {"_n": len(ids[k])} for k, d in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    sq = load(a.sq, a.match)
    fe = load(a.fetch, a.match) if a.fetch else {}
    wr = load(a.write, a.match) if a.write else {}
    rows = sorted(sq.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))[: a.top]
    for (name, grid), d in rows:
        g = d.get("GRBM_GUI_ACTIVE", 0) / 8
        w = max(d.get("SQ_WAVES", 1), 1)
        line = f"{name[:58]:58s} grid {grid:9d} n {d['_n']:3d}"
        if g:
            line += f"  cyc {g:9.0f}"
            if d.get("SQ_INSTS_VALU"):
                line += f"  VALU/wave {d['SQ_INSTS_VALU'] / w:7.0f}  cyc/VALU/SIMD {g / (d['SQ_INSTS_VALU'] / 1024):6.2f}"
            if d.get("SQ_WAVE_CYCLES"):
                occ = 4 * d["SQ_WAVE_CYCLES"] / g / 4096
                line += f"  occ {occ:5.2f}"
                line += f"  waitany {d.get('SQ_WAIT_ANY', 0) / d['SQ_WAVE_CYCLES']:4.2f}"
                line += f"  waitinst {d.get('SQ_WAIT_INST_ANY', 0) / d['SQ_WAVE_CYCLES']:4.2f}"
            if d.get("SQ_INSTS_LDS"):
                line += f"  LDS/wave {d['SQ_INSTS_LDS'] / w:6.0f}"
            if d.get("SQ_INSTS_SALU"):
                line += f"  SALU/wave {d['SQ_INSTS_SALU'] / w:6.0f}"
        k = (name, grid)
        if k in fe and k in wr:
            rd = fe[k].get("FETCH_SIZE", 0) * 2 * 1024  # gfx950 correction (profiles/traffic.json)
            wb = wr[k].get("WRITE_SIZE", 0) * 1024
            line += f"  HBM read {rd / 1e6:8.2f} MB write {wb / 1e6:8.2f} MB"
        print(line)


if __name__ == "__main__":
    main()
