#!/usr/bin/env python3
"""Trace probe for the two-in-flight serving pattern: K batches of B 1080p
MEDIUM pairs alternating between two engines on two caller streams (one
sub-batch stream each), under rocprofv3 --kernel-trace; tools/timeline.py then
shows which hardware queue each launch ran on and how the batches overlap.
--mode one: the headline loop (one engine, one caller stream) instead."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import disflow  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="two")
ap.add_argument("--steps", type=int, default=12)
ap.add_argument("--nsub", type=int, default=1)
ap.add_argument("--graphs", type=int, default=1)
ap.add_argument("--link", type=int, default=0)
a = ap.parse_args()
W, H, B = 1920, 1080, 32
dev = torch.device("cuda", 0)
p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
pairs = [disflow.synth_pair(k, W, H) for k in range(B)]
d0 = torch.from_numpy(np.stack([x for x, _ in pairs])).to(dev)
d1 = torch.from_numpy(np.stack([y for _, y in pairs])).to(dev)
n_eng = 1 if a.mode == "one" else 2
engs = [disflow.DenseInverseSearch(p, W, H, max_batch=B) for _ in range(n_eng)]
strs = [torch.cuda.Stream() for _ in range(n_eng)]
outs = [torch.empty((B, H, W, 2), dtype=torch.float32, device=dev) for _ in range(n_eng)]
for e in engs:
    e.set_concurrency(a.nsub)
    e.set_graphs(bool(a.graphs))
if a.link and n_eng == 2:
    engs[0].pipeline_link(engs[1])
for k in range(a.steps):
    i = k % n_eng
    engs[i].calc_device(B, d0.data_ptr(), d1.data_ptr(), outs[i].data_ptr(), strs[i].cuda_stream)
torch.cuda.synchronize()
print("done")
