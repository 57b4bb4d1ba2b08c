#!/usr/bin/env python3
"""Tolerance calibration: how far can the reference's OWN
results move under rounding choices its unverifiable build could have made?

The reference cannot be built here (OpenCV 2.4 / Eigen 3 absent), so the
oracle restates Eigen's reduction order and MSVC's separately rounded float
arithmetic from recollection. This tool runs the same restatement built three
other ways (oracle/Makefile `variants`):
  seqsum  every Eigen .sum() as a plain left-to-right loop
  avxsum  Eigen's sum with 8-wide AVX packets instead of 4-wide SSE
  fma     gcc -ffp-contract=fast -mfma (FMA contraction wherever it applies)
  cvsimd  the pyramid's 2x2 area sums in OpenCV 3.x's SIMD order, (tl+bl)+(tr+br)
          except the W % 4 column tail (the reference's OpenCV version is unknown)
and measures, against the reference-order oracle on the same synthetic pairs:
the final-flow end-point error (mean, p99.9, max, share of pixels > 0.01 px),
and, on the finest searched level with identical pyramids, the share of patches
whose displacement moved at all and by more than 0.5 px (outlier-reset flips);
and the largest EPE over the pixels no flipped finest-level patch reaches
(tests/flipmask.py; each variant's own pyramid and patches).
The stated tolerance is 2x the largest spread observed.

TEST INFRASTRUCTURE: loads only oracle/ builds. Writes one JSON document.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd")]
import oracle_binding as ob  # noqa: E402
from flipmask import flip_mask, outside_max_epe  # noqa: E402

VARIANTS = ("seqsum", "avxsum", "fma", "cvsimd")
WORKLOADS = [
    # name, W, H, preset, paper, seeds
    ("640x480 ULTRAFAST", 640, 480, "ULTRAFAST", 0, range(0, 8)),
    ("1920x1080 MEDIUM", 1920, 1080, "MEDIUM", 0, range(0, 4)),
    ("1920x1080 MEDIUM paper mode", 1920, 1080, "MEDIUM", 1, range(0, 2)),
    ("3840x2160 MEDIUM", 3840, 2160, "MEDIUM", 0, range(900, 902)),
]


def load_variant(name):
    path = os.path.join(ROOT, "oracle", f"libdis_oracle_{name}.so")
    if not os.path.exists(path):
        raise SystemExit(f"{path} missing: make -C oracle variants")
    L = ctypes.CDLL(path)
    base = ob.lib
    for fn, f in list(vars(base).items()):  # every prototype the binding declared
        if fn.startswith("dis_oracle_"):
            getattr(L, fn).argtypes = f.argtypes
            getattr(L, fn).restype = f.restype
    return L


def with_lib(L, fn, *args, **kw):
    saved = ob.lib
    ob.lib = L
    try:
        return fn(*args, **kw)
    finally:
        ob.lib = saved


def stated(wl):
    """Per-workload stated tolerance: 2x the largest spread over the variants."""
    keys = ("mean_epe", "p999_epe", "patch_flip_rate", "max_epe_outside_flips")
    return {k: 2 * max(r[k] for r in wl["variants"].values()) for k in keys}


def epe(a, b):
    return np.sqrt(((a.astype(np.float64) - b.astype(np.float64)) ** 2).sum(-1)).ravel()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "tolerance_r03.json"))
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1), help="oracle patch-loop threads")
    ap.add_argument("--quick", action="store_true", help="one seed per workload")
    ap.add_argument("--only", default="", help="run only workloads whose name contains this")
    a = ap.parse_args()
    import disflow

    libs = {v: load_variant(v) for v in VARIANTS}
    for L in list(libs.values()) + [ob.lib]:  # identical results, shorter wall time
        L.dis_oracle_set_threads.argtypes = [ctypes.c_int]
        L.dis_oracle_set_threads(a.threads)
    report = {"method": __doc__.split("\n\n")[1].replace("\n", " "), "workloads": []}
    worst = {"mean_epe": 0.0, "p999_epe": 0.0, "max_epe": 0.0, "patch_flip_rate": 0.0, "max_epe_outside_flips": 0.0}
    for name, W, H, preset, paper, seeds in WORKLOADS:
        if a.only not in name:
            continue
        seeds = list(seeds)[:1] if a.quick else list(seeds)
        p = disflow.preset_params(disflow.Preset[preset], W, H)
        p.paper_mode = paper
        C, F, ps, it, ov = p.coarsest_scale, p.finest_scale, p.patch_size, p.iterations, p.patch_overlap
        rows = {v: {"epe": [], "moved": [], "flip": [], "outside": [], "reach": []} for v in VARIANTS}
        for seed in seeds:
            I0, I1 = disflow.synth_pair(seed, W, H)
            base = ob.calc_from_params(I0, I1, p)
            Wp, Hp, P0, PX, PY, P1, _, _ = ob.build_pyramids(I0, I1, C, ps)
            _, us0, _ = ob.flow_from_pyramids(P0, PX, PY, P1, ps, Wp, Hp, C, F, it, ps, ov, 1,
                                              capture=True, paper=paper)
            for v, L in libs.items():
                f = with_lib(L, ob.calc_from_params, I0, I1, p)
                rows[v]["epe"].append(epe(f, base))
                _, us, _ = with_lib(L, ob.flow_from_pyramids, P0, PX, PY, P1, ps, Wp, Hp, C, F, it, ps, ov, 1,
                                    capture=True, paper=paper)
                d = np.sqrt(((us[F].astype(np.float64) - us0[F]) ** 2).sum(-1))
                rows[v]["moved"].append(d > 0)
                rows[v]["flip"].append(d > 0.5)
                # the variant's own pyramid and patches (consistent with its flow)
                _, _, V0, VX, VY, V1, _, _ = with_lib(L, ob.build_pyramids, I0, I1, C, ps)
                _, usv, _ = with_lib(L, ob.flow_from_pyramids, V0, VX, VY, V1, ps, Wp, Hp, C, F, it, ps, ov, 1,
                                     capture=True, paper=paper)
                mask, _ = flip_mask(usv[F], us0[F], W, H, C, F, ps, ob.steps(ps, ov))
                mx, reach = outside_max_epe(f, base, mask)
                rows[v]["outside"].append(mx)
                rows[v]["reach"].append(reach)
        wl = {"workload": name, "pairs": len(seeds), "variants": {}}
        for v in VARIANTS:
            e = np.concatenate(rows[v]["epe"])
            moved = np.concatenate(rows[v]["moved"])
            flip = np.concatenate(rows[v]["flip"])
            r = {"mean_epe": float(e.mean()), "p999_epe": float(np.percentile(e, 99.9)),
                 "max_epe": float(e.max()), "pixels_over_0.01px": float((e > 0.01).mean()),
                 "patches_moved": float(moved.mean()), "patch_flip_rate": float(flip.mean()),
                 "max_epe_outside_flips": float(max(rows[v]["outside"])),
                 "flip_reach_fraction": float(np.mean(rows[v]["reach"]))}
            wl["variants"][v] = r
            for k in worst:
                worst[k] = max(worst[k], r[k])
            print(f"{name:28s} {v:7s} mean {r['mean_epe']:.2e}  p99.9 {r['p999_epe']:.2e}  max {r['max_epe']:.3f}  "
                  f">0.01px {r['pixels_over_0.01px']:.2%}  patches moved {r['patches_moved']:.2%}  "
                  f"flips {r['patch_flip_rate']:.3%}  max outside flips {r['max_epe_outside_flips']:.4f} "
                  f"(reach {r['flip_reach_fraction']:.3%})", flush=True)
        wl["stated_tolerance"] = stated(wl)
        report["workloads"].append(wl)
    report["largest_spread"] = worst
    report["stated_tolerance"] = {k: 2 * v for k, v in worst.items() if k != "max_epe"}
    report["stated_tolerance"]["max_epe"] = "reported, not bounded (outlier-reset flips move a patch by up to the outlier threshold)"
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(report, open(a.out, "w"), indent=1)
    print(json.dumps(report["stated_tolerance"]))


if __name__ == "__main__":
    main()
