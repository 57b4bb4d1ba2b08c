"""Structured synthetic scenes for parity tests (no dataset is available: the
reference's own material, MPI Sintel, is absent). Unlike the value-noise
generator (disflow.synth_pair), these frames have the statistics that make
real footage hard for DIS: large flat regions (zero gradients, singular
Hessians), sharp object edges, objects moving independently by up to ~20 px
(occlusions and disocclusions, outlier resets, spread blocks for the tile
fallback), an image-border crossing object and a saturated (0 / 255) region.

scene_pair(seed, W, H) -> (I0, I1) u8; deterministic for a seed."""
import numpy as np


def _layers(rng, W, H):
    """Background + objects: (kind, params, intensity field parameters, motion)."""
    objs = []
    n = int(rng.integers(10, 18))
    for k in range(n):
        kind = "rect" if k % 2 == 0 else "disc"
        cx, cy = rng.uniform(-0.05, 1.05) * W, rng.uniform(-0.05, 1.05) * H  # some cross the border
        sx, sy = rng.uniform(0.04, 0.22) * W, rng.uniform(0.04, 0.22) * H
        flat = k % 3 != 0                                   # two thirds flat, one third textured
        base = float(rng.choice([0.0, 255.0])) if k == 1 else float(rng.uniform(20, 235))  # one saturated
        mv = rng.uniform(-20, 20, 2) if k % 4 != 3 else rng.uniform(-1.5, 1.5, 2)
        objs.append((kind, cx, cy, sx, sy, flat, base, mv, int(rng.integers(1 << 30))))
    return objs


def _render(W, H, objs, bg_shift, t, seed):
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    rng = np.random.default_rng(seed)
    # background: a shallow ramp (near-flat) plus one low-amplitude texture band
    bx, by = xx - t * bg_shift[0], yy - t * bg_shift[1]
    img = 90.0 + 0.01 * bx + 0.006 * by
    band = (by > 0.62 * H) & (by < 0.78 * H)
    img = np.where(band, img + 12.0 * np.sin(bx / 7.0) * np.cos(by / 5.0), img)
    for kind, cx, cy, sx, sy, flat, base, mv, oseed in objs:
        ox, oy = xx - (cx + t * mv[0]), yy - (cy + t * mv[1])
        if kind == "rect":
            m = (np.abs(ox) <= sx / 2) & (np.abs(oy) <= sy / 2)
        else:
            m = (ox / (sx / 2)) ** 2 + (oy / (sy / 2)) ** 2 <= 1.0
        if flat:
            val = np.full_like(img, base)
        else:  # texture attached to the object (moves with it)
            val = base + 25.0 * np.sin(ox / 3.1 + oseed % 7) * np.sin(oy / 4.3) + 10.0 * np.cos((ox + oy) / 2.3)
        img = np.where(m, val, img)
    noise = rng.normal(0.0, 0.6, img.shape)  # sensor noise, independent per frame
    return np.clip(np.round(img + noise), 0, 255).astype(np.uint8)


def scene_pair(seed, W, H):
    rng = np.random.default_rng(seed)
    objs = _layers(rng, W, H)
    bg = rng.uniform(-3, 3, 2)
    return _render(W, H, objs, bg, 0.0, seed * 2 + 1), _render(W, H, objs, bg, 1.0, seed * 2 + 2)
