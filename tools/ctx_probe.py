#!/usr/bin/env python3
"""Diagnostic: throughput of successive contexts in one process (1080p MEDIUM,
batch 32) -- does a context created after others run slower (HIP stream ->
hardware-queue mapping), and does the sub-batch stream count matter?"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import disflow  # noqa: E402

W, H, B = 1920, 1080, 32
dev = torch.device("cuda", 0)
p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
pairs = [disflow.synth_pair(k, W, H) for k in range(B)]
d0 = torch.from_numpy(np.stack([a for a, _ in pairs])).to(dev)
d1 = torch.from_numpy(np.stack([b for _, b in pairs])).to(dev)
out = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
s = torch.cuda.current_stream(dev)


def timeit(eng, label, steps=40):
    for _ in range(10):
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    print(f"{label:40s} {B * steps / (time.perf_counter() - t):8.0f} pairs/s", flush=True)


for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    eng = disflow.DenseInverseSearch(p, W, H, max_batch=B)
    timeit(eng, f"ctx {rnd}: 2 streams")
    eng.set_concurrency(1)
    timeit(eng, f"ctx {rnd}: 1 stream")
    eng.set_concurrency(2)
    timeit(eng, f"ctx {rnd}: 2 streams again")
    eng.close()
