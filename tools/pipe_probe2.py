#!/usr/bin/env python3
"""Probe (r03): batches of 32 1080p MEDIUM pairs (inputs in HBM) issued in
serving patterns, each after >= 1 s of untimed warm-up (clock ramp), in one
process, interleaved over --rounds:
  one       one engine, 2 sub-batch streams, graphs (bench.py's `value`)
  two-g     two engines, 1 sub-batch stream each, graphs, calls alternating on
            two caller streams (two batches in flight, no fork/join per call)
  two-g2    the same with 2 sub-batch streams per engine
  linked    two engines linked with dis_pipeline_link (eager by construction)
Prints pairs/s per pattern (median over rounds) and checks every output."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import disflow  # noqa: E402
from bench import make_pairs  # noqa: E402

W, H, B = 1920, 1080, 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
    I0, I1 = make_pairs(list(range(B)), W, H)
    d0 = torch.from_numpy(I0).to(dev)
    d1 = torch.from_numpy(I1).to(dev)
    outs = [torch.empty((B, H, W, 2), dtype=torch.float32, device=dev) for _ in range(2)]

    one = disflow.DenseInverseSearch(p, W, H, max_batch=B)
    ea = disflow.DenseInverseSearch(p, W, H, max_batch=B)
    eb = disflow.DenseInverseSearch(p, W, H, max_batch=B)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def setup(mode):
        if mode == "one":
            return [one], [main_s]
        ea.pipeline_link(None)
        c = 2 if mode == "two-g2" else 1
        for e in (ea, eb):
            e.set_concurrency(c)
        if mode == "linked":
            ea.pipeline_link(eb)
        return [ea, eb], [sa, sb]

    def run(engs, strs, calls):
        for k in range(calls):
            e = k % len(engs)
            engs[e].calc_device(B, d0.data_ptr(), d1.data_ptr(), outs[e].data_ptr(), strs[e].cuda_stream)

    modes = ["one", "two-g", "two-g2", "linked"]
    res = {m: [] for m in modes}
    for r in range(a.rounds):
        for m in modes:
            engs, strs = setup(m)
            t = time.perf_counter()
            while time.perf_counter() - t < 1.0:
                run(engs, strs, 8)
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(engs, strs, a.calls)
            torch.cuda.synchronize()
            res[m].append(B * a.calls / (time.perf_counter() - t0))
    ref = one.calc_batch(I0[:4], I1[:4])
    for o in outs:
        assert np.array_equal(o[:4].cpu().numpy().view(np.uint32), ref.view(np.uint32))
    for m in modes:
        print(f"{m:8s} median {np.median(res[m]):9.0f} pairs/s   rounds " + " ".join(f"{v:.0f}" for v in res[m]))
    print("outputs identical")


if __name__ == "__main__":
    main()
