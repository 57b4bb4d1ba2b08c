#!/usr/bin/env python3
"""Per-workgroup timeline of the r06 coarse-head experiment (k_search8_head) from a
library built with timestamps (STAMPS=1 tools/build_head_variant.sh, which exports
dis_head_stamps: per workgroup its level, s_memrealtime at its ticket, after
its wait, and before its publish; 100 MHz). Prints, per sub-batch and head
level, when its blocks took tickets, were released and finished, in us from
the sub-batch's first ticket.
  python3 tools/head_probe.py <lib> [--batch 32] [--streams 2]"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import torch  # noqa: E402

import disflow  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--calls", type=int, default=3)
    a = ap.parse_args()
    disflow.LIB_PATH = a.lib if os.path.isabs(a.lib) else os.path.join(ROOT, a.lib)
    L = disflow.lib()
    L.dis_head_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    W, H, B = 1920, 1080, a.batch
    dev = torch.device("cuda", 0)
    pairs = [disflow.synth_pair(k, W, H) for k in range(B)]
    d0 = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
    d1 = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
    eng = disflow.DenseInverseSearch(disflow.preset_params(disflow.Preset.MEDIUM, W, H), W, H, max_batch=B)
    eng.set_concurrency(a.streams)
    out = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
    buf = np.zeros((16384, 4), dtype=np.uint64)
    for call in range(a.calls + 2):
        L.dis_head_stamps(buf.ctypes.data_as(ctypes.c_void_p), 16384)  # reset
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        n = L.dis_head_stamps(buf.ctypes.data_as(ctypes.c_void_p), 16384)
        if call < 2:
            continue
        s = buf[:n]
        print(f"call {call}: {n} workgroups")
        t00 = int(s[:, 1].min())
        for sub in sorted(set(int(x) >> 8 for x in s[:, 0])):
            ss = s[(s[:, 0] >> 8).astype(int) == sub]
            t0 = int(ss[:, 1].min())
            print(f"  sub key {sub}: first ticket at {(t0 - t00) / 100:.2f} us")
            for j in sorted(set(int(x) & 255 for x in ss[:, 0])):
                r = ss[(ss[:, 0] & 255).astype(int) == j]
                f = lambda col: (r[:, col].astype(np.int64) - t0) / 100.0  # noqa: E731
                print(f"    level {j}: {len(r):4d} wgs  ticket {f(1).min():7.2f}..{f(1).max():7.2f}  "
                      f"released {f(2).min():7.2f}..{f(2).max():7.2f}  done {f(3).min():7.2f}..{f(3).max():7.2f}  "
                      f"run after release med {np.median(f(3) - f(2)):6.2f} us")


if __name__ == "__main__":
    main()
