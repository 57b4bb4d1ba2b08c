#!/usr/bin/env python3
"""Per-call timeline of the sub-batch streams without a profiler attached.

Needs the diagnostic build (tools/build_variants.sh stamp:"-DDIS_STAMP") and
DIS_STAMP=1: k_pyr12 of each sub-batch records its start clock and every
k_output workgroup its end clock (s_memrealtime, 100 MHz) per call. Runs the
bench configuration (32 x 1920x1080 MEDIUM, inputs in HBM, graphs on) for
--steps back-to-back calls and prints, per call: the sub-batches' start
offsets, their ends, and the idle time before the next call's first start.

usage: DIS_STAMP=1 DISFLOW_LIB=.../libdis_hip_stamp.so tools/stamp_probe.py [--steps N] [--streams S]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "optical-flow-using-dense-inverse-search_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))

K_STAMP_N = 4096
K_MAX_SUB = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--streams", type=int, default=0)
    ap.add_argument("--no-graphs", action="store_true")
    a = ap.parse_args()
    assert os.environ.get("DIS_STAMP"), "set DIS_STAMP=1"
    import torch
    import disflow
    from bench import make_pairs

    W, H, B = 1920, 1080, 32
    p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
    I0, I1 = make_pairs(list(range(B)), W, H)
    dev = torch.device("cuda", 0)
    d0 = torch.from_numpy(I0).to(dev)
    d1 = torch.from_numpy(I1).to(dev)
    out = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
    eng = disflow.DenseInverseSearch(p, W, H, max_batch=B)
    if a.streams:
        eng.set_concurrency(a.streams)
    if a.no_graphs:
        eng.set_graphs(False)
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(a.warmup):
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s)
    torch.cuda.synchronize(dev)
    lib = disflow.lib()
    lib.dis_stamp_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    n = K_MAX_SUB * (1 + 2 * K_STAMP_N)
    buf = np.zeros(n, np.uint64)
    assert lib.dis_stamp_read(eng._ctx, buf.ctypes.data, n) == 0
    base = buf.reshape(K_MAX_SUB, 1 + 2 * K_STAMP_N)
    c0 = [int(base[k, 0]) for k in range(K_MAX_SUB)]
    for _ in range(a.steps):
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s)
    torch.cuda.synchronize(dev)
    assert lib.dis_stamp_read(eng._ctx, buf.ctypes.data, n) == 0
    base = buf.reshape(K_MAX_SUB, 1 + 2 * K_STAMP_N)
    subs = [k for k in range(K_MAX_SUB) if int(base[k, 0]) > c0[k]]
    st = {k: [int(base[k, 1 + (i % K_STAMP_N)]) for i in range(c0[k], c0[k] + a.steps)] for k in subs}
    en = {k: [int(base[k, 1 + K_STAMP_N + (i % K_STAMP_N)]) for i in range(c0[k], c0[k] + a.steps)] for k in subs}
    us = 0.01  # 100 MHz ticks -> us
    rows = []
    for i in range(a.steps - 1):
        t0 = min(st[k][i] for k in subs)
        end = max(en[k][i] for k in subs)
        nxt = min(st[k][i + 1] for k in subs)
        rows.append([(st[k][i] - t0) * us for k in subs] + [(en[k][i] - t0) * us for k in subs] +
                    [(nxt - end) * us, (nxt - t0) * us])
    r = np.array(rows)
    ns = len(subs)
    print(f"sub-batch streams {ns}, calls {a.steps}, graphs {not a.no_graphs}")
    print("median  starts " + " ".join(f"{v:7.1f}" for v in np.median(r[:, :ns], 0)) +
          "  ends " + " ".join(f"{v:7.1f}" for v in np.median(r[:, ns:2 * ns], 0)) +
          f"  idle before next {np.median(r[:, 2 * ns]):6.1f}  call {np.median(r[:, 2 * ns + 1]):7.1f} us")
    for row in rows[:8]:
        print("        starts " + " ".join(f"{v:7.1f}" for v in row[:ns]) + "  ends " +
              " ".join(f"{v:7.1f}" for v in row[ns:2 * ns]) + f"  idle {row[2 * ns]:6.1f}  call {row[2 * ns + 1]:7.1f}")


if __name__ == "__main__":
    main()
