#!/usr/bin/env python3
"""Throughput of the BASELINE.json configs beyond the headline bench line
(bench.py measures config 2): one JSON line per config, inputs and outputs
resident in HBM, batch per call as given, `steps` timed calls after warmup.

  config 1  640x480    ULTRAFAST
  1cpu      config 1's reference CPU path (BASELINE config 1): the C restatement
            (oracle/dis_oracle.c at -O3, one pair at a time per process, like
            src/main.cpp:102-206) on one core and on the job's 16-CPU share --
            run first, before the GPU is initialised (forked workers)
  config 2  1920x1080  MEDIUM            (as bench.py)
  config 3  3840x2160  MEDIUM
  config 5  3840x2160  SLOW + variational refinement (3 fixed-point iterations per level)
  2p        1920x1080  MEDIUM in paper mode
  2f / 3f   configs 2 / 3 with DIS_PRECISION_FMA (contracted search arithmetic,
            within the stated tolerance; tests/test_gpu_tolerance.py)
  colour    1920x1080  Middlebury colour coding of 32 flow fields (dis_flow_color)
  compat    1920x1080  MEDIUM through the reference-interface entry (dis_flow_from_pyramids,
            OpticalFlowClass semantics: host padded pyramids in, finest-level flow out,
            synchronous) beside dis_calc_u8 on host frames, one pair per call
  host      1920x1080  MEDIUM host-frame path (dis_calc_batch_u8 with DIS_MEM_HOST: host
            frames in, host flow out, synchronous) at batches 1, 4 and 32, pageable and
            page-locked buffers, beside the box's measured D2H rate and the pairs/s that
            rate allows for 16.6 MB of flow per pair
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import disflow  # noqa: E402

CONFIGS = {
    "1": ("640x480 ULTRAFAST", 640, 480, "ULTRAFAST", 64),
    "2": ("1920x1080 MEDIUM", 1920, 1080, "MEDIUM", 32),
    "3": ("3840x2160 MEDIUM", 3840, 2160, "MEDIUM", 8),
    "5": ("3840x2160 SLOW + variational refinement", 3840, 2160, "SLOW", 2),
    "2p": ("1920x1080 MEDIUM paper mode", 1920, 1080, "MEDIUM", 32, 1),
    "2f": ("1920x1080 MEDIUM, DIS_PRECISION_FMA", 1920, 1080, "MEDIUM", 32, 0, 1),
    "3f": ("3840x2160 MEDIUM, DIS_PRECISION_FMA", 3840, 2160, "MEDIUM", 8, 0, 1),
}
FMA_PEAK = 157.3  # TFLOP/s, vector f32 with FMA counted as 2 (MI355X_MICROARCH.md)
EXACT_PEAK = 78.6  # non-FMA f32 issue peak (one op per lane per instruction)


def run(name, W, H, preset, B, steps, warmup, paper=0, fma=0):
    dev = torch.device("cuda", 0)
    p = disflow.preset_params(disflow.Preset[preset], W, H)
    p.paper_mode = paper
    pairs = [disflow.synth_pair(k, W, H) for k in range(B)]
    d0 = torch.from_numpy(np.stack([a for a, _ in pairs])).to(dev)
    d1 = torch.from_numpy(np.stack([b for _, b in pairs])).to(dev)
    out = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
    eng = disflow.DenseInverseSearch(p, W, H, max_batch=B)
    if fma:
        eng.set_precision(disflow.PRECISION_FMA)
    s = torch.cuda.current_stream(dev)
    for _ in range(warmup):
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    wl = disflow.workload(p, W, H)
    # finest-level search launch, one stream, HIP dispatch events (as bench.py)
    eng.set_concurrency(1)
    eng.set_kernel_timing(True)
    for _ in range(3):
        eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    n_f, ms_f = eng.kernel_time(disflow.KERNEL_SEARCH_FINEST)
    refine = None
    if p.var_refine_iters > 0:
        # the finest level's refinement launches (HIP events, eager under timing),
        # against an algorithmic-bytes model per pixel and fixed-point iteration
        # (DESIGN.md 3b): linearisation reads the flow (8 B), I1 (4, the warp's
        # taps once), I0 (4), I0x / I0y (8) and writes B1, B2, A12, D1, D2, the
        # smoothness weight (24): 48 B; the SOR reads those 6 planes (24) and
        # reads + writes the flow (16): 40 B
        px = wl["padded_width"] * wl["padded_height"] // (4 ** p.finest_scale) * B
        refine = {"level_pixels": px, "fixed_point_iterations": p.var_refine_iters}
        for kname, kind, bpp in (("k_vr_lin", disflow.KERNEL_VR_LIN, 48), ("k_vr_sor", disflow.KERNEL_VR_SOR, 40)):
            n_k, ms_k = eng.kernel_time(kind)
            avg = ms_k / max(n_k, 1)
            refine[kname] = {"launches": n_k, "avg_launch_ms": avg, "algorithmic_bytes_per_px": bpp,
                            "achieved_GBps": bpp * px / (avg * 1e-3) / 1e9,
                            "hbm_frac": bpp * px / (avg * 1e-3) / 8e12}
    eng.set_kernel_timing(False)
    launch_ms = ms_f / max(n_f, 1)
    flops = wl["search_flops_finest"] * B
    achieved = flops / (launch_ms * 1e-3) / 1e12
    peak = FMA_PEAK if fma else EXACT_PEAK
    eng.close()
    return {"config": name, "preset": preset, "precision": "fma" if fma else "exact",
            "finest_search": {"avg_launch_ms": launch_ms, "algorithmic_tflops": achieved, "peak": peak,
                              "frac": achieved / peak,
                              "note": "algorithmic ops of the reference (each add/mul 1) / launch time; peak "
                                      + ("157.3 (FMA = 2 ops)" if fma else "78.6 (non-FMA issue)")},
            "knobs": {"C": p.coarsest_scale, "F": p.finest_scale,
                                                        "it": p.iterations, "overlap": p.patch_overlap,
                                                        "var_refine_iters": p.var_refine_iters,
                                                        "paper_mode": p.paper_mode},
            "batch": B, "steps": steps, "ms_per_step": el / steps * 1e3, "pairs_per_s": B * steps / el,
            "refinement_finest_level": refine,
            "patches_per_pair": wl["patches"], "updates_per_pair": wl["updates"],
            "updates_per_s": wl["updates"] * B * steps / el}


def run_colour(steps, warmup):
    W, H, B = 1920, 1080, 32
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    f = torch.from_numpy((rng.standard_normal((B, H, W, 2)) * 4).astype(np.float32)).to(dev)
    out = torch.empty((B, H, W, 3), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    L = disflow.lib()

    def call():
        disflow._check(L.dis_flow_color(f.data_ptr(), B, W, H, -1.0, out.data_ptr(), disflow.MEM_DEVICE,
                                        s.cuda_stream, 0))
    for _ in range(warmup):
        call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        call()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    # algorithmic bytes per field: the flow read once (8 B/px) and the BGR image
    # written (3 B/px); the max-radius pass's second read of each field is
    # served from the L2 / MALL in k_color (dis_color.hip), so it is not counted
    per_field = W * H * (8 + 3)
    moved = B * per_field
    return {"config": "colour 1920x1080 x32", "ms_per_call": el * 1e3, "fields_per_s": B / el,
            "algorithmic_bytes_per_field": per_field, "hbm_gbs": moved / el / 1e9, "hbm_frac": moved / el / 8e12,
            "hbm_frac_two_reads": B * W * H * (8 * 2 + 3) / el / 8e12}


def run_compat(steps, warmup):
    W, H = 1920, 1080
    p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
    C, F, ps = p.coarsest_scale, p.finest_scale, p.patch_size
    I0, I1 = disflow.synth_pair(0, W, H)
    eng = disflow.DenseInverseSearch(p, W, H, max_batch=1)
    eng.set_debug(True)
    eng.calc(I0, I1)
    # the caller's padded planes (construct_pyramide layout), from this engine's own level images
    wl = disflow.workload(p, W, H)
    Wp, Hp = wl["padded_width"], wl["padded_height"]
    P1, PX, PY = [], [], []
    for l in range(C + 1):
        w, h = Wp >> l, Hp >> l
        if l < F:
            z = np.zeros((h + 2 * ps, w + 2 * ps), np.float32)
            P1.append(z), PX.append(z), PY.append(z)
            continue
        P1.append(np.pad(eng.debug_dump(disflow.STAGE_IMG1, l).reshape(h, w), ps, mode="edge"))
        PX.append(np.pad(eng.debug_dump(disflow.STAGE_DX0, l).reshape(h, w), ps))
        PY.append(np.pad(eng.debug_dump(disflow.STAGE_DY0, l).reshape(h, w), ps))
    eng.set_debug(False)

    def compat():
        return disflow.optical_flow_from_pyramids(P1, PX, PY, P1, ps, Wp, Hp, C, F, p.iterations, ps,
                                                  p.patch_overlap, True)

    def calc():
        return eng.calc(I0, I1)
    res = {}
    for name, fn in (("compat", compat), ("calc", calc)):
        for _ in range(warmup):
            fn()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        res[name] = steps / (time.perf_counter() - t0)
    eng.close()
    return {"config": "compat 1920x1080 MEDIUM, one pair per call, host memory",
            "compat_pairs_per_s": res["compat"], "calc_u8_pairs_per_s": res["calc"],
            "compat_over_calc": res["compat"] / res["calc"],
            "note": "compat = dis_flow_from_pyramids (H2D of the padded dx/dy/I1 planes, fast search, "
                    "finest-level flow D2H); calc = dis_calc_u8 host mode (H2D of the u8 frames, full path, "
                    "full-resolution flow D2H)"}


def run_host(steps, warmup):
    W, H, Bmax = 1920, 1080, 32
    dev = torch.device("cuda", 0)
    p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
    pairs = [disflow.synth_pair(k, W, H) for k in range(Bmax)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    fb = W * H * 8
    # the box's D2H rate: page-locked destination, 4 pairs' flow per copy
    d = torch.empty(4 * fb, dtype=torch.uint8, device=dev)
    h = torch.empty(4 * fb, dtype=torch.uint8, pin_memory=True)
    h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    d2h = 10 * 4 * fb / (time.perf_counter() - t0) / 1e9
    del d, h
    eng = disflow.DenseInverseSearch(p, W, H, max_batch=Bmax)
    flow = np.empty((Bmax, H, W, 2), np.float32)
    pf = torch.empty((Bmax, H, W, 2), dtype=torch.float32, pin_memory=True)
    pi0 = torch.from_numpy(I0).pin_memory()
    pi1 = torch.from_numpy(I1).pin_memory()
    res = {}
    for kind, a0, a1, fo in (("pageable", I0.ctypes.data, I1.ctypes.data, flow.ctypes.data),
                             ("page_locked", pi0.data_ptr(), pi1.data_ptr(), pf.data_ptr())):
        for B in (1, 4, 32):
            for _ in range(max(1, warmup)):
                eng.calc_batch_host(B, a0, a1, fo)
            reps = max(2, steps * 4 // B)
            t0 = time.perf_counter()
            for _ in range(reps):
                eng.calc_batch_host(B, a0, a1, fo)
            res[f"{kind}_B{B}"] = B * reps / (time.perf_counter() - t0)
    info = eng.host_pipeline_info()
    eng.close()
    bound = d2h * 1e9 / fb
    return {"config": "host-frame path 1920x1080 MEDIUM (dis_calc_batch_u8, DIS_MEM_HOST)",
            "pairs_per_s": res, "d2h_GBps": d2h, "d2h_bound_pairs_per_s": bound,
            "frac_of_d2h_bound": {k: v / bound for k, v in res.items()}, "pipeline": info,
            "note": "d2h = page-locked 66 MB copies on this box; the bound = that rate / 16.6 MB of flow per pair "
                    "(the uploads, 4.1 MB per pair, run the other PCIe direction)"}


def run_cpu1(budget_s):
    """BASELINE config 1 on the host: 640x480 ULTRAFAST through the C
    restatement, single-core latency and 16-process throughput (bench.py's
    cpu_baseline on this workload)."""
    sys.path.insert(0, ROOT)
    import bench
    W, H = 640, 480
    p = disflow.preset_params(disflow.Preset.ULTRAFAST, W, H)
    workers = min(bench.CPU_WORKER_CAP, len(os.sched_getaffinity(0)))
    r = bench.cpu_baseline(p, W, H, budget_s, workers)
    return {"config": "config 1 CPU: 640x480 ULTRAFAST, C restatement (" +
            os.path.basename(bench.oracle_lib_for_baseline()) + ")",
            "kind": "port", "pairs_per_s": r["value"], "cores": r["cores"], "pairs": r["pairs"],
            "single_core_pairs_per_s": r["single_core"]["value"], "single_core_pairs": r["single_core"]["pairs"],
            "cpu_model": bench.cpu_model(), "budget_s": budget_s,
            "knobs": {"C": p.coarsest_scale, "F": p.finest_scale, "it": p.iterations, "overlap": p.patch_overlap}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1cpu,1,2,3,5,2p,2f,3f,colour,compat,host")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=9.0)
    a = ap.parse_args()
    cfgs = a.configs.split(",")
    if "1cpu" in cfgs:  # forks its workers: before anything initialises the GPU
        cfgs.remove("1cpu")
        print(json.dumps(run_cpu1(a.cpu_seconds)), flush=True)
    for c in cfgs:
        if c == "colour":
            r = run_colour(a.steps, a.warmup)
        elif c == "compat":
            r = run_compat(a.steps, a.warmup)
        elif c == "host":
            r = run_host(a.steps, a.warmup)
        else:
            name, W, H, preset, B = CONFIGS[c][:5]
            steps = max(2, a.steps // (4 if c == "5" else 1))
            r = run(f"config {c}: {name}", W, H, preset, B, steps, a.warmup, *CONFIGS[c][5:])
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
