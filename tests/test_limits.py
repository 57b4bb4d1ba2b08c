"""Maximum sizes: the engine's frame limit (2^28 pixels, dis_runtime.hip
check_params) and the extreme shapes within it.

At 2^28 pixels every index the kernels form is near its widest: level-0 pixel
indices reach 2^28, flow element indices 2^29, and a second pair in a batch
starts 2 GiB into the flow buffer; a 256 x 2^20 frame has 2^18 level-2 rows
(launch grids whose y extent follows the rows), a 2^20 x 256 frame 2^20
columns. The `gpu` tests run those frames through the C-ABI and compare them
bit for bit with the oracle (threaded; ULTRAFAST keeps the checker at seconds
per frame). The inputs are tiled from seeded synthetic pairs (the generator
itself takes ~1 minute per 2^28-pixel frame on one core); the tiles are
shifted per copy so no two tiles of a frame are equal.
"""
import numpy as np
import pytest

MAX_PIXELS = 1 << 28


def _frames(disflow, seed, W, H, tile=2048):
    a, b = disflow.synth_pair(seed, tile, tile)
    I0 = np.empty((H, W), np.uint8)
    I1 = np.empty_like(I0)
    nx = -(-W // tile)
    for y0 in range(0, H, tile):
        for x0 in range(0, W, tile):
            k = (y0 // tile) * nx + x0 // tile
            h, w = min(tile, H - y0), min(tile, W - x0)
            # per-tile shift of the pattern (rows and columns rolled), the same
            # for both frames: the flow between them stays the synthetic one
            I0[y0:y0 + h, x0:x0 + w] = np.roll(a, (7 * k, 13 * k), axis=(0, 1))[:h, :w]
            I1[y0:y0 + h, x0:x0 + w] = np.roll(b, (7 * k, 13 * k), axis=(0, 1))[:h, :w]
    return I0, I1


def test_frame_limit_is_enforced():
    import disflow
    p = disflow.preset_params(disflow.Preset.ULTRAFAST, 16384, 16384)
    assert disflow.validate(p, 16384, 16384) == 0
    assert disflow.validate(p, 256, 1 << 20) == 0
    assert disflow.validate(p, 1 << 20, 256) == 0
    assert disflow.validate(p, 16385, 16384) != 0      # one column over 2^28
    assert disflow.validate(p, 1 << 20, 257) != 0
    assert disflow.validate(p, 1 << 29, 1) != 0


def test_tiled_frames_are_deterministic():
    import disflow
    a0, a1 = _frames(disflow, 3, 5000, 300, tile=512)
    b0, b1 = _frames(disflow, 3, 5000, 300, tile=512)
    assert a0.shape == (300, 5000) and np.array_equal(a0, b0) and np.array_equal(a1, b1)
    assert not np.array_equal(a0[:, :512], a0[:, 512:1024])


@pytest.mark.gpu
def test_largest_square_frames_batch_bitexact(disflow_mod, oracle):
    W = H = 16384
    assert W * H == MAX_PIXELS
    p = disflow_mod.preset_params(disflow_mod.Preset.ULTRAFAST, W, H)
    pairs = [_frames(disflow_mod, 40 + k, W, H) for k in range(2)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    del pairs
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=2)
    got = eng.calc_batch(I0, I1)
    del eng
    for k in range(2):
        with oracle.threads():
            exp = oracle.calc_from_params(I0[k], I1[k], p)
        assert np.array_equal(got[k].view(np.uint32), exp.view(np.uint32)), f"16384^2 pair {k}"
        assert np.isfinite(exp).all() and np.abs(exp).max() > 0.5  # a real flow field, not zeros
        del exp


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(256, 1 << 20), (1 << 20, 256)])
def test_tallest_and_widest_frames_bitexact(disflow_mod, oracle, W, H):
    assert W * H == MAX_PIXELS
    p = disflow_mod.preset_params(disflow_mod.Preset.ULTRAFAST, W, H)
    I0, I1 = _frames(disflow_mod, 50, W, H)
    got = disflow_mod.DenseInverseSearch(p, W, H).calc(I0, I1)
    with oracle.threads():
        exp = oracle.calc_from_params(I0, I1, p)
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), f"{W}x{H}"
