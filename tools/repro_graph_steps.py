#!/usr/bin/env python3
"""Step-selectable copy of test_graph_replay_matches_eager_and_tracks_its_key
(bisecting a host crash): repro_graph_steps.py <steps>, steps a subset of
  E  an eager (graphs off) context's host call first
  K  device calls over 2 buffer sets x n in (B, 2), 3 rounds (4 graph keys)
  S  concurrency 1 then 3, capture + replay each
  F  FMA precision, one device call
  H  the graph context's host call (where the crash was)
  D  a device call on a new buffer set (a new graph key) instead
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import disflow as d  # noqa: E402


def main():
    steps = sys.argv[1] if len(sys.argv) > 1 else "EKSFH"
    W, H, B = 640, 480, 4
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    pairs = [d.synth_pair(70 + k, W, H) for k in range(B)]
    X0 = np.stack([a for a, _ in pairs])
    X1 = np.stack([b for _, b in pairs])
    if "E" in steps:
        eager = d.DenseInverseSearch(p, W, H, max_batch=B)
        eager.set_graphs(False)
        eager.calc_batch(X0, X1)
        print("E ok", flush=True)
    eng = d.DenseInverseSearch(p, W, H, max_batch=B)
    s = torch.cuda.current_stream()
    bufs = [(torch.from_numpy(X0).cuda(), torch.from_numpy(X1).cuda(),
             torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")) for _ in range(2)]
    if "K" in steps:
        for rep in range(3):
            for k, (d0, d1, out) in enumerate(bufs):
                for n in (B, 2):
                    out.fill_(float("nan"))
                    eng.calc_device(n, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
                    torch.cuda.synchronize()
        print("K ok", flush=True)
    d0, d1, out = bufs[0]
    if "S" in steps:
        for streams in (1, 3):
            eng.set_concurrency(streams)
            for _ in range(2):
                eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
                torch.cuda.synchronize()
        print("S ok", flush=True)
    if "F" in steps:
        eng.set_precision(d.PRECISION_FMA)
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        print("F ok", flush=True)
    if "D" in steps:
        e0, e1 = torch.from_numpy(X0).cuda(), torch.from_numpy(X1).cuda()
        o2 = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
        eng.calc_device(B, e0.data_ptr(), e1.data_ptr(), o2.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        print("D ok", flush=True)
    if "H" in steps:
        eng.calc_batch(X0, X1)
        print("H ok", flush=True)
    print("done", steps, flush=True)


if __name__ == "__main__":
    main()
