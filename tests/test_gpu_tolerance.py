"""DIS_PRECISION_FMA (dis_set_precision) against the stated tolerance.

The tolerance mode contracts the search's warp, steepest-descent and Hessian
dot products into fma and solves with the pivots' reciprocals, so it is not
bit-exact; the north star's contract is a stated per-pixel tolerance against
the reference, which DESIGN.md 2 calibrated from the spread of the reference's
own plausible builds (tools/tolerance.py, profiles/tolerance_r03.json: 2x the
largest spread per workload):

    1920x1080 MEDIUM: mean EPE <= 3.3e-4 px, p99.9 EPE <= 5.1e-2 px, patch flips <= 0.014 %,
                      max EPE outside flip sites <= 0.34 px
    3840x2160 MEDIUM: mean EPE <= 1.16e-3 px, p99.9 EPE <= 6.5e-2 px, patch flips <= 0.024 %,
                      max EPE outside flip sites <= 0.62 px

(a patch flip: finest-level displacement moved by > 0.5 px, an outlier reset
decided the other way; its sites: every full-resolution pixel a flipped patch
reaches through the densification and the upsample, tests/flipmask.py; the
per-pixel bound holds everywhere else -- VERDICT r2 item 6, calibrated the same
way in profiles/tolerance_r03.json). Checked here on BASELINE configs 2 (1920x1080 MEDIUM,
4 pairs) and 3 (3840x2160 MEDIUM, the calibration's 2 pairs) against the C
oracle (reference order), which is itself parity-unpinned against the
reference."""
import numpy as np
import pytest

from flipmask import flip_mask, outside_max_epe

pytestmark = pytest.mark.gpu

TOLERANCE = {  # (mean EPE, p99.9 EPE, flip rate, max EPE outside flip sites)
    (1920, 1080): (3.3e-4, 5.1e-2, 1.4e-4, 0.34),
    (3840, 2160): (1.16e-3, 6.5e-2, 2.4e-4, 0.62),
}


def _epe(a, b):
    return np.sqrt(((a.astype(np.float64) - b.astype(np.float64)) ** 2).sum(-1)).ravel()


@pytest.mark.parametrize("W,H,seeds", [(1920, 1080, range(4)), (3840, 2160, range(2))])
def test_fma_mode_within_stated_tolerance(disflow_mod, oracle, W, H, seeds):
    d = disflow_mod
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    seeds = list(seeds)
    pairs = [d.synth_pair(900 + s, W, H) for s in seeds]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    eng = d.DenseInverseSearch(p, W, H, max_batch=len(seeds))
    eng.set_precision(d.PRECISION_FMA)
    eng.set_debug(True)
    got = eng.calc_batch(I0, I1)
    u_gpu = [eng.debug_dump(d.STAGE_PATCH_U, p.finest_scale, k).reshape(-1, 2) for k in range(len(seeds))]
    exact = d.DenseInverseSearch(p, W, H, max_batch=len(seeds)).calc_batch(I0, I1)
    epes, flips, moved, outside, reach = [], [], [], [], []
    oracle.set_threads(16)  # the checker's patch loop threaded: identical results
    for k, (a, b) in enumerate(pairs):
        exp = oracle.calc_from_params(a, b, p)
        assert np.array_equal(exact[k].view(np.uint32), exp.view(np.uint32)), "exact mode must stay bit-exact"
        assert np.isfinite(got[k]).all()
        epes.append(_epe(got[k], exp))
        C, F, ps = p.coarsest_scale, p.finest_scale, p.patch_size
        Wp, Hp, P0, PX, PY, P1, _, _ = oracle.build_pyramids(a, b, C, ps)
        _, us, _ = oracle.flow_from_pyramids(P0, PX, PY, P1, ps, Wp, Hp, C, F, p.iterations, ps,
                                             p.patch_overlap, 1, capture=True)
        dist = np.sqrt(((u_gpu[k].astype(np.float64) - us[F].reshape(-1, 2)) ** 2).sum(-1))
        flips.append(dist > 0.5)
        moved.append(dist > 0)
        mask, _ = flip_mask(u_gpu[k], us[F], W, H, C, F, ps, oracle.steps(ps, p.patch_overlap))
        mx, frac = outside_max_epe(got[k], exp, mask)
        outside.append(mx)
        reach.append(frac)
    oracle.set_threads(1)
    e = np.concatenate(epes)
    flip = np.concatenate(flips).mean()
    mean, p999 = e.mean(), np.percentile(e, 99.9)
    print(f"{W}x{H} FMA mode vs oracle: mean EPE {mean:.2e}, p99.9 {p999:.2e}, max {e.max():.3f}, "
          f"patches moved {np.concatenate(moved).mean():.2%}, flips {flip:.4%}, "
          f"max EPE outside flip sites {max(outside):.4f} (sites {np.mean(reach):.3%} of pixels)")
    assert np.concatenate(moved).any(), "FMA mode ran the exact kernels"
    mean_tol, p999_tol, flip_tol, outside_tol = TOLERANCE[(W, H)]
    assert mean <= mean_tol
    assert p999 <= p999_tol
    assert flip <= flip_tol
    assert max(outside) <= outside_tol


def test_precision_switch_validates_and_exact_is_default(disflow_mod, oracle):
    d = disflow_mod
    W, H = 320, 240
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    I0, I1 = d.synth_pair(31, W, H)
    eng = d.DenseInverseSearch(p, W, H)
    with pytest.raises(d.DisError):
        eng.set_precision(7)
    exp = oracle.calc_from_params(I0, I1, p)
    assert np.array_equal(eng.calc(I0, I1).view(np.uint32), exp.view(np.uint32))
    eng.set_precision(d.PRECISION_FMA)
    eng.set_precision(d.PRECISION_EXACT)
    assert np.array_equal(eng.calc(I0, I1).view(np.uint32), exp.view(np.uint32))
