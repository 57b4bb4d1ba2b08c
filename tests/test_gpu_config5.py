"""BASELINE.json config 5 at its real size: 3840x2160, preset SLOW (F = 0,
C = 7, steps 2, 128 iterations) with variational refinement (3 fixed-point
iterations per level) -- VERDICT r1 "next" item 1.

(a) bit-exact vs the C oracle with the search iterations cut to 8 (the oracle
    finishes in ~15-20 s on one host core); everything else -- refinement on
    every level, the dense-field initialisation, F = 0 -- at full size;
(b) the full preset (it = 128) checked through size-independent properties:
    determinism, batch == single pair, finite output, lower refinement energy
    than the same search without refinement, and tracking of the synthetic
    ground-truth motion.

Refinement is not in the reference (README.md:11), so its parity is to the C
restatement, unpinned against the reference by construction."""
import numpy as np
import pytest

from test_gpu_parity import _assert_bitexact

pytestmark = pytest.mark.gpu

W, H = 3840, 2160


def _slow(disflow):
    p = disflow.preset_params(disflow.Preset.SLOW, W, H)
    assert (p.coarsest_scale, p.finest_scale, p.iterations, p.var_refine_iters) == (7, 0, 128, 3)
    assert abs(p.patch_overlap - 0.75) < 1e-7
    return p


def test_config5_full_size_reduced_iterations_bitexact(disflow_mod, oracle):
    p = _slow(disflow_mod)
    p.iterations = 8
    I0, I1 = disflow_mod.synth_pair(500, W, H)
    got = disflow_mod.DenseInverseSearch(p, W, H).calc(I0, I1)
    exp = oracle.calc_from_params(I0, I1, p)
    _assert_bitexact(got, exp, "3840x2160 SLOW + refinement (it=8)")


def _level0_cropped(oracle, I, C):
    img = oracle.pad_convert(I, C)
    lv0 = oracle.pyramid(img, 0, want_grad=False)[0][0]
    Wp, Hp, pl, pt = oracle.padded_size(W, H, C)
    return np.ascontiguousarray(lv0[pt:pt + H, pl:pl + W])


def test_config5_full_preset_properties(disflow_mod, oracle):
    p = _slow(disflow_mod)
    pairs = [disflow_mod.synth_pair(510 + k, W, H, with_gt=True) for k in range(2)]
    I0 = np.stack([a for a, _, _ in pairs])
    I1 = np.stack([b for _, b, _ in pairs])
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=2)
    batch = eng.calc_batch(I0, I1)
    assert np.isfinite(batch).all()
    again = eng.calc_batch(I0, I1)  # deterministic: no atomics on the data path
    assert np.array_equal(again.view(np.uint32), batch.view(np.uint32))
    for k in range(2):  # a batch computes each pair exactly as alone
        one = eng.calc(I0[k], I1[k])
        assert np.array_equal(one.view(np.uint32), batch[k].view(np.uint32)), k
    p0 = _slow(disflow_mod)
    p0.var_refine_iters = 0
    plain = disflow_mod.DenseInverseSearch(p0, W, H, max_batch=2).calc_batch(I0, I1)
    for k, (_, _, gt) in enumerate(pairs):
        m0 = _level0_cropped(oracle, I0[k], p.coarsest_scale)
        m1 = _level0_cropped(oracle, I1[k], p.coarsest_scale)
        e_ref = oracle.var_energy(m0, m1, batch[k])
        e_plain = oracle.var_energy(m0, m1, plain[k])
        assert e_ref < e_plain, (k, e_ref, e_plain)
        epe = np.sqrt(((batch[k] - gt) ** 2).sum(-1))
        assert np.median(epe) < 1.0, np.median(epe)


def test_refinement_kernel_timing_eager_path_bitexact(disflow_mod):
    # dis_kernel_time classes 4 / 5 (ABI v7): under kernel timing the
    # refinement launches run eagerly with events around the finest level's
    # k_vr_lin / k_vr_sor instead of replaying the per-level graphs -- the
    # flow must not change, and the counts follow the fixed-point iterations
    w, h = 640, 480
    p = disflow_mod.preset_params(disflow_mod.Preset.SLOW, w, h)
    p.iterations = 8
    I0, I1 = disflow_mod.synth_pair(520, w, h)
    eng = disflow_mod.DenseInverseSearch(p, w, h)
    ref = eng.calc(I0, I1)
    eng.set_kernel_timing(True)
    got = eng.calc(I0, I1)
    got2 = eng.calc(I0, I1)
    n_lin, ms_lin = eng.kernel_time(disflow_mod.KERNEL_VR_LIN)
    n_sor, ms_sor = eng.kernel_time(disflow_mod.KERNEL_VR_SOR)
    eng.set_kernel_timing(False)
    _assert_bitexact(got, ref, "refinement under kernel timing")
    _assert_bitexact(got2, ref, "refinement under kernel timing (2nd call)")
    assert n_lin == n_sor == 2 * p.var_refine_iters
    assert ms_lin > 0 and ms_sor > 0
