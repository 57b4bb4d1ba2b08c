#!/usr/bin/env python3
"""How many patch blocks does the tile search list for the fallback kernel
(DIS_STAGE_FALLBACK) on a few inputs? Diagnostic for the parity tests that
must exercise k_search8_fb: structured scenes, and split-motion pairs (two
halves of a texture moving apart by 2d px) at 2 lanes per patch everywhere."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd"))
import numpy as np  # noqa: E402

import disflow  # noqa: E402
import scenes  # noqa: E402


def split_pair(W, H, d, seed=1):
    """Multi-octave texture (low frequencies for the coarse levels to lock
    onto), its left half moving right by d px and its right half left by d."""
    big, _ = disflow.synth_pair(seed, W + 2 * d, H)
    I0 = big[:, d:d + W]
    left = np.arange(W)[None, :] < W // 2
    I1 = np.where(left, big[:, 0:W], big[:, 2 * d:2 * d + W])
    return np.ascontiguousarray(I0), np.ascontiguousarray(I1.astype(np.uint8))


def main():
    for W, H, preset, d in ((640, 480, "MEDIUM", 50), (640, 480, "MEDIUM", 80), (1920, 1080, "MEDIUM", 60),
                            (1920, 1080, "MEDIUM", 100), (640, 480, "FAST", 60)):
        I0, I1 = split_pair(W, H, d)
        p = disflow.preset_params(disflow.Preset[preset], W, H)
        e = disflow.DenseInverseSearch(p, W, H)
        for v in (0, 3):
            e.set_variant(v)
            e.calc(I0, I1)
            print("split", W, H, preset, d, "variant", v, [e.fallback_blocks(l) for l in range(p.finest_scale, p.coarsest_scale + 1)])
    for seed in (30, 31):
        I0, I1 = scenes.scene_pair(seed, 1920, 1080)
        p = disflow.preset_params(disflow.Preset.MEDIUM, 1920, 1080)
        e = disflow.DenseInverseSearch(p, 1920, 1080)
        e.calc(I0, I1)
        print("scene", seed, [e.fallback_blocks(l) for l in range(p.finest_scale, p.coarsest_scale + 1)])


if __name__ == "__main__":
    main()
