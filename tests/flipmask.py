"""Flip sites of a non-bit-exact run (test infrastructure).

An outlier reset (src/patch.cpp:185-194) is a discrete event: a one-ulp
difference can decide it the other way and move a patch by up to the outlier
threshold. The tolerance mode's contract therefore bounds the per-pixel error
(end-point error, EPE) only outside the pixels such a "flip" can reach:

  * flipped patch: a finest-level patch whose displacement differs from the
    reference-order oracle's by more than 0.5 px;
  * its reach: the patch footprint (src/patch_grid.cpp:139-140, ps x ps around
    the centre) on level F, widened by one level-F pixel each way for the
    bilinear upsample (src/main.cpp:191-198), at full resolution (x 2^F),
    minus the padding crop.

`flip_mask` returns that full-resolution (H, W) boolean mask; `outside_max_epe`
the largest EPE over the pixels outside it.
"""
import numpy as np


def grid(Wl, Hl, steps):
    """src/patch_grid.cpp:20-23 (npw, nph, offw, offh)."""
    npw = -(-Wl // steps)
    nph = -(-Hl // steps)
    return npw, nph, (Wl - (npw - 1) * steps) // 2, (Hl - (nph - 1) * steps) // 2


def padded(W, H, C):
    sf = 1 << C
    padw = (sf - W % sf) % sf
    padh = (sf - H % sf) % sf
    return W + padw, H + padh, padw // 2, padh // 2


def flip_mask(u_got, u_ref, W, H, C, F, ps, steps, thresh=0.5):
    """u_got, u_ref: finest-level patch displacements (n, 2), patch-id order
    (x-major, src/patch_grid.cpp:39-50)."""
    Wp, Hp, pl, pt = padded(W, H, C)
    Wl, Hl = Wp >> F, Hp >> F
    npw, nph, offw, offh = grid(Wl, Hl, steps)
    d = np.sqrt(((np.asarray(u_got, np.float64).reshape(-1, 2) -
                  np.asarray(u_ref, np.float64).reshape(-1, 2)) ** 2).sum(-1))
    assert d.size == npw * nph, (d.size, npw, nph)
    mask = np.zeros((H, W), bool)
    s = 1 << F
    hp = ps // 2
    for i in np.flatnonzero(~(d <= thresh)):  # NaN counts as flipped
        gx, gy = divmod(int(i), nph)
        cx, cy = gx * steps + offw, gy * steps + offh
        x0, x1 = (cx - hp - 1) * s - pl, (cx + hp + 1) * s - pl  # [x0, x1) full resolution
        y0, y1 = (cy - hp - 1) * s - pt, (cy + hp + 1) * s - pt
        mask[max(0, y0):max(0, min(H, y1)), max(0, x0):max(0, min(W, x1))] = True
    return mask, d


def outside_max_epe(flow_got, flow_ref, mask):
    e = np.sqrt(((flow_got.astype(np.float64) - flow_ref.astype(np.float64)) ** 2).sum(-1))
    out = e[~mask]
    return float(out.max()) if out.size else 0.0, float(mask.mean())
