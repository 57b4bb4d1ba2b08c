#!/usr/bin/env python3
"""Host<->device transfer rates and per-batch compute latency on this box:
what bounds the host-frame path (dis_calc_batch_u8 with DIS_MEM_HOST, the
reference's own call pattern src/main.cpp:115-116,184-189 -- host frames in,
host flow out). Prints one JSON line.

  pinned / pageable H2D and D2H (torch copies, 16.6 MB = one 1080p flow)
  device-resident calc latency per batch size (1080p MEDIUM)
  host-mode calc throughput per batch size (numpy in / numpy out)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import disflow  # noqa: E402


def rate(fn, nbytes, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    out = {}
    nb = W * H * 8
    d = torch.empty(nb, dtype=torch.uint8, device=dev)
    hp = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    hq = torch.empty(nb, dtype=torch.uint8)
    hq.fill_(1)
    lib = os.environ.get("DISFLOW_LIB")
    out["lib"] = os.path.basename(lib) if lib else "libdis_hip.so"
    for k, fn in (("pinned_d2h_GBps", lambda: hp.copy_(d, non_blocking=True)),
                  ("pinned_h2d_GBps", lambda: d.copy_(hp, non_blocking=True)),
                  ("pageable_d2h_GBps", lambda: hq.copy_(d)),
                  ("pageable_h2d_GBps", lambda: d.copy_(hq))):
        out[k] = rate(fn, nb)
    big = 8 * nb
    d8 = torch.empty(big, dtype=torch.uint8, device=dev)
    hp8 = torch.empty(big, dtype=torch.uint8, pin_memory=True)
    out["pinned_d2h_8x_GBps"] = rate(lambda: hp8.copy_(d8, non_blocking=True), big, 10)
    t0 = time.perf_counter()
    for _ in range(10):
        np.copyto(hq.numpy(), hp.numpy())
    out["host_memcpy_1thread_GBps"] = 10 * nb / (time.perf_counter() - t0) / 1e9
    del d8, hp8
    p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
    Bmax = 32
    pairs = [disflow.synth_pair(k, W, H) for k in range(Bmax)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    eng = disflow.DenseInverseSearch(p, W, H, max_batch=Bmax)
    d0 = torch.from_numpy(I0).to(dev)
    d1 = torch.from_numpy(I1).to(dev)
    fo = torch.empty((Bmax, H, W, 2), dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev)
    lat = {}
    for B in (1, 2, 4, 8, 16, 32):
        for _ in range(3):
            eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), fo.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 20
        for _ in range(reps):
            eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), fo.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        lat[B] = (time.perf_counter() - t0) / reps * 1e3
    out["device_ms_per_call"] = lat
    host = {}
    for B in (1, 4, 8, 32):
        flow = np.empty((B, H, W, 2), np.float32)
        L = disflow.lib()

        def call():
            disflow._check(L.dis_calc_batch_u8(eng._ctx, B, I0.ctypes.data, I1.ctypes.data, W, W * H,
                                                flow.ctypes.data, disflow.MEM_HOST, None))
        call()
        t0 = time.perf_counter()
        reps = max(2, 32 // B)
        for _ in range(reps):
            call()
        host[B] = B * reps / (time.perf_counter() - t0)
    out["host_mode_pairs_per_s"] = host
    # pinned destination (page-locked by torch's host allocator)
    pf = torch.empty((Bmax, H, W, 2), dtype=torch.float32, pin_memory=True)
    pi0 = torch.from_numpy(I0).pin_memory()
    pi1 = torch.from_numpy(I1).pin_memory()
    hostp = {}
    for B in (1, 4, 8, 32):
        L = disflow.lib()

        def callp():
            disflow._check(L.dis_calc_batch_u8(eng._ctx, B, pi0.data_ptr(), pi1.data_ptr(), W, W * H,
                                                pf.data_ptr(), disflow.MEM_HOST, None))
        callp()
        t0 = time.perf_counter()
        reps = max(2, 32 // B)
        for _ in range(reps):
            callp()
        hostp[B] = B * reps / (time.perf_counter() - t0)
    out["host_mode_pinned_pairs_per_s"] = hostp
    # chunk sizes at B = 32, pageable buffers (the library default: 0 = auto)
    sweep = {}
    flow = np.empty((Bmax, H, W, 2), np.float32)
    for chunk in (1, 2, 4, 8, 0):
        try:
            eng.set_host_pipeline(chunk)
        except Exception as e:  # (an A/B library with another setter)
            sweep[f"chunk{chunk}"] = repr(e)[:60]
            continue
        eng.calc_batch_host(Bmax, I0.ctypes.data, I1.ctypes.data, flow.ctypes.data)
        t0 = time.perf_counter()
        for _ in range(3):
            eng.calc_batch_host(Bmax, I0.ctypes.data, I1.ctypes.data, flow.ctypes.data)
        sweep[f"chunk{chunk}"] = 3 * Bmax / (time.perf_counter() - t0)
    out["host_mode_sweep_B32"] = sweep
    out["d2h_bound_pairs_per_s"] = out["pinned_d2h_GBps"] * 1e9 / nb
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
