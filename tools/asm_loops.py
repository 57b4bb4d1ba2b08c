#!/usr/bin/env python3
"""Per-loop instruction counts of one kernel in a hipcc -S listing, from the
compiler's block comments ("Loop Header" / "in Loop: Header=BBx_y"): VALU / DS /
SALU instructions per loop (its own blocks and the header), to compare kernel
variants without a GPU.  usage: asm_loops.py file.s kernel_symbol_substring"""
import re
import sys
from collections import defaultdict


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l)
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    loops = defaultdict(lambda: [0, 0, 0, 0])
    cur = None
    for l in lines[start:end]:
        if re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:)", l):
            m = re.search(r"Header=BB(\d+_\d+)", l)
            h = re.match(r"^\.LBB(\d+_\d+):.*Loop Header", l)
            cur = h.group(1) if h else (m.group(1) if m else None)
            continue
        t = l.strip()
        if cur is None or not l.startswith("\t") or t.startswith(";") or t.startswith("."):
            continue
        c = loops[cur]
        c[3] += 1
        if t.startswith("v_"):
            c[0] += 1
        elif t.startswith("ds_"):
            c[1] += 1
        elif t.startswith("s_"):
            c[2] += 1
    for h, (v, d, s, n) in loops.items():
        print(f"loop BB{h:10s} VALU {v:4d}  DS {d:3d}  SALU {s:3d}  total {n}")
    meta = [l.strip() for l in lines[end:end + 200] if "next_free_vgpr" in l or "next_free_sgpr" in l]
    print(" ".join(meta[:2]))


if __name__ == "__main__":
    main()
