#!/usr/bin/env python3
"""Interleaved A/B timing of library builds in ONE process (cdna guide §5.4
rule 24): each variant = path to a libdis_hip*.so [+ ":streams=N"]; rounds
alternate variants; prints median/min ms per step and pairs/s per variant.

--spawn N: instead, N rounds of one child process per variant (interleaved),
for variants whose streams would interfere inside one process (several
contexts' streams share the process's hardware queues)."""
import argparse
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import disflow  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--preset", default="medium")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spawn", type=int, default=0)
    a = ap.parse_args()
    if a.spawn:
        return spawn(a)
    W, H, B = a.width, a.height, a.batch
    dev = torch.device("cuda", 0)
    pairs = [disflow.synth_pair(k, W, H) for k in range(B)]
    d0 = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
    d1 = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
    outs, engines = [], []
    for v in a.variants:
        path, _, opt = v.partition(":")
        disflow._lib = None
        disflow.LIB_PATH = os.path.join(ROOT, path) if not os.path.isabs(path) else path
        L = disflow.lib()
        p = disflow.preset_params(disflow.Preset[a.preset.upper()], W, H)
        opts = dict(kv.partition("=")[::2] for kv in filter(None, opt.split(",")))
        if "iters" in opts:
            p.iterations = int(opts.pop("iters"))
        if "vr" in opts:
            p.var_refine_iters = int(opts.pop("vr"))
        if "paper" in opts:
            p.paper_mode = int(opts.pop("paper"))
        eng = disflow.DenseInverseSearch(p, W, H, max_batch=B)
        for k, val in opts.items():
            if k == "streams":
                eng.set_concurrency(int(val))
            elif k == "variant":
                eng.set_variant(int(val))
            elif k == "graphs":
                eng.set_graphs(bool(int(val)))
            elif k == "fma":
                eng.set_precision(int(val))
            else:
                raise SystemExit(f"unknown option {k}")
        engines.append((v, L, eng))
        outs.append(torch.empty((B, H, W, 2), dtype=torch.float32, device=dev))
    s = torch.cuda.current_stream(dev)
    times = {v: [] for v in a.variants}
    for r in range(a.rounds + 1):
        for (v, L, eng), out in zip(engines, outs):
            disflow._lib = L
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            if r:  # round 0 is warm-up
                times[v].append((time.perf_counter() - t0) / a.steps * 1e3)
    ref = outs[0].cpu().numpy().view(np.uint32)
    for (v, _, _), out in zip(engines, outs):
        same = np.array_equal(out.cpu().numpy().view(np.uint32), ref)
        t = times[v]
        print(f"{v:70s} median {statistics.median(t):.3f} ms  min {min(t):.3f} ms  "
              f"pairs/s {B / statistics.median(t) * 1e3:.0f}  same_as_first={same}")
    # each context is destroyed by the library that created it (a context
    # handed to another build's dis_destroy crashed the process at exit)
    torch.cuda.synchronize()
    for v, L, eng in engines:
        disflow._lib = L
        eng.close()


def spawn(a):
    import re
    import subprocess
    res = {v: [] for v in a.variants}
    for _ in range(a.spawn):
        for v in a.variants:
            cmd = [sys.executable, os.path.abspath(__file__), v, "--rounds", str(a.rounds), "--steps", str(a.steps),
                   "--batch", str(a.batch), "--preset", a.preset, "--width", str(a.width), "--height", str(a.height)]
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stdout, out.stderr, file=sys.stderr)
                raise SystemExit(f"child failed: {v}")
            m = re.search(r"median ([0-9.]+) ms", out.stdout)
            res[v].append(float(m.group(1)))
    for v, t in res.items():
        print(f"{v:70s} median-of-process-medians {statistics.median(t):.3f} ms  min {min(t):.3f} ms  "
              f"pairs/s {a.batch / statistics.median(t) * 1e3:.0f}  ({len(t)} processes)")


if __name__ == "__main__":
    main()
