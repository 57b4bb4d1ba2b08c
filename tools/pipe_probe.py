#!/usr/bin/env python3
"""Probe: K batches of B 1080p MEDIUM pairs issued (a) one after another on one
stream (the bench's loop) and (b) alternating between two engines on two
streams (two batches in flight, each engine with one sub-batch stream), every
batch written in full. Prints pairs/s for each schedule."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import disflow  # noqa: E402

W, H, B, K = 1920, 1080, 32, 20
dev = torch.device("cuda", 0)
p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
pairs = [disflow.synth_pair(k, W, H) for k in range(B)]
d0 = torch.from_numpy(np.stack([a for a, _ in pairs])).to(dev)
d1 = torch.from_numpy(np.stack([b for _, b in pairs])).to(dev)
outs = [torch.empty((B, H, W, 2), dtype=torch.float32, device=dev) for _ in range(2)]


def run(engs, streams, K):
    for k in range(4):
        e = k % len(engs)
        engs[e].calc_device(B, d0.data_ptr(), d1.data_ptr(), outs[e].data_ptr(), streams[e].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        e = k % len(engs)
        engs[e].calc_device(B, d0.data_ptr(), d1.data_ptr(), outs[e].data_ptr(), streams[e].cuda_stream)
    torch.cuda.synchronize()
    return B * K / (time.perf_counter() - t0)


one = disflow.DenseInverseSearch(p, W, H, max_batch=B)
print("one engine, 2 sub-batch streams:", round(run([one], [torch.cuda.current_stream()], K)))
ea = disflow.DenseInverseSearch(p, W, H, max_batch=B)
eb = disflow.DenseInverseSearch(p, W, H, max_batch=B)
for e in (ea, eb):
    e.set_concurrency(1)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
print("two engines on two streams, 1 sub-batch each:", round(run([ea, eb], [sa, sb], K)))
ea.pipeline_link(eb)
print("  linked (dis_pipeline_link):", round(run([ea, eb], [sa, sb], K)))
print("  linked, 40 batches:", round(run([ea, eb], [sa, sb], 40)))
ea.pipeline_link(None)
for e in (ea, eb):
    e.set_concurrency(2)
print("two engines on two streams, 2 sub-batches each:", round(run([ea, eb], [sa, sb], K)))
outs += [torch.empty((B, H, W, 2), dtype=torch.float32, device=dev) for _ in range(2)]
engs = [disflow.DenseInverseSearch(p, W, H, max_batch=B) for _ in range(4)]
strs = [torch.cuda.Stream() for _ in range(4)]
for e in engs:
    e.set_concurrency(1)
print("three engines on three streams:", round(run(engs[:3], strs[:3], 21)))
print("four engines on four streams:", round(run(engs, strs, K)))
ref = one.calc_batch(d0.cpu().numpy(), d1.cpu().numpy())
for o in outs:
    assert np.array_equal(o.cpu().numpy().view(np.uint32), ref.view(np.uint32))
print("outputs identical")
