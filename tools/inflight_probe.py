#!/usr/bin/env python3
"""Batches in flight (bench.py's `pipelined` line, generalised): N contexts,
one sub-batch stream each (set_concurrency(1): the context runs on the caller's
stream), steps issued round-robin to N caller streams, every flow written.
Prints pairs/s per N next to the one-context two-sub-batch step (the headline
form). 1080p MEDIUM, 32 pairs per step.
  python3 tools/inflight_probe.py [--steps 60] [--ns 1,2,3,4]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import torch  # noqa: E402

import disflow  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--ns", default="1,2,3,4")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    W, H, B = 1920, 1080, 32
    dev = torch.device("cuda", 0)
    pairs = [disflow.synth_pair(k, W, H) for k in range(B)]
    d0 = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
    d1 = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
    params = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
    nmax = max(int(x) for x in a.ns.split(","))
    engs = [disflow.DenseInverseSearch(params, W, H, max_batch=B) for _ in range(nmax)]
    strs = [torch.cuda.Stream(dev) for _ in range(nmax)]
    outs = [torch.empty((B, H, W, 2), dtype=torch.float32, device=dev) for _ in range(nmax)]

    def run(n, steps):
        if n == 0:  # the headline form: one context, two sub-batch streams, one caller stream
            engs[0].set_concurrency(2)
            for _ in range(steps):
                engs[0].calc_device(B, d0.data_ptr(), d1.data_ptr(), outs[0].data_ptr(), strs[0].cuda_stream)
            return
        for e in engs[:n]:
            e.set_concurrency(1)
        for k in range(steps):
            engs[k % n].calc_device(B, d0.data_ptr(), d1.data_ptr(), outs[k % n].data_ptr(), strs[k % n].cuda_stream)

    forms = [0] + [int(x) for x in a.ns.split(",")]
    res = {f: [] for f in forms}
    for r in range(a.rounds + 1):
        for f in forms:
            run(f, 8)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            run(f, a.steps)
            torch.cuda.synchronize(dev)
            if r:
                res[f].append(B * a.steps / (time.perf_counter() - t0))
    ref = outs[0].view(torch.int32)
    same = all(torch.equal(o.view(torch.int32), ref) for o in outs)
    for f in forms:
        name = "one context, 2 sub-batch streams" if f == 0 else f"{f} context(s) in flight, 1 stream each"
        print(f"{name:40s} pairs/s median {np.median(res[f]):8.0f}  max {max(res[f]):8.0f}")
    print("outputs identical:", same)


if __name__ == "__main__":
    main()
