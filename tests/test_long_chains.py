"""Long iteration chains: the reference's own default run
(src/main.cpp:63-72 -- ps 8, overlap 0.7 -> steps 2, it 1000, C 3, F 0) at the
MPI-Sintel frame size (README.md:13, 1024x436) on two seeds, the SLOW preset at
its full 128 iterations with refinement, and the FAST preset at 1920x1080.

Every bit-exact check before this one stopped at it <= 25; a long chain is
where the kernels' division (div_pre: per-patch reciprocal + Markstein
correction), the outlier reset (src/patch.cpp:185-194) and the thr_sq form of
the outlier test would first show a one-ulp divergence.

CPU tests pin tests/golden/long_chains.json (make_long_chains.py) against the
oracle; the `gpu` tests run the HIP path through the C-ABI and compare it bit
for bit with the oracle computed live on the same inputs (threaded patch loop,
identical results) and with the committed digests.
"""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "long_chains.json")) as f:
    GOLDEN = json.load(f)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _inputs(disflow, e):
    p = disflow.preset_params(getattr(disflow.Preset, e["preset"]), e["W"], e["H"])
    for k, v in e["params"].items():  # the resolved knob tuple the fixture was made with
        got = getattr(p, k)
        assert (abs(got - v) < 1e-7) if isinstance(v, float) else got == v, (k, got, v)
    I0, I1 = disflow.synth_pair(e["seed"], e["W"], e["H"])
    assert _sha(I0) == e["sha_I0"] and _sha(I1) == e["sha_I1"], "synthetic generator changed"
    return p, I0, I1


def _check_against_fixture(flow, e, what):
    if _sha(flow) == e["sha_flow"]:
        return
    flat = np.ascontiguousarray(flow, np.float32).reshape(-1)
    samp = flat[::e["sample_stride"]][:len(e["sample"])]
    exp = np.array(e["sample"], np.float32)
    nbad = int((samp.view(np.uint32) != exp.view(np.uint32)).sum())
    raise AssertionError(f"{what}: flow digest differs from the golden fixture ({nbad} of {len(exp)} sampled "
                         f"values differ; max|flow| {np.abs(flat).max()} vs {e['max_abs']})")


def test_reference_preset_is_the_cli_default():
    import disflow
    p = disflow.preset_params(disflow.Preset.REFERENCE, 1024, 436)
    # src/main.cpp:63-72: patch 8, overlap 0.7 (steps floor(8*0.3) = 2), 1000 iterations, C 3, F 0
    assert (p.patch_size, p.iterations, p.coarsest_scale, p.finest_scale) == (8, 1000, 3, 0)
    assert abs(p.patch_overlap - 0.7) < 1e-7 and p.var_refine_iters == 0 and p.patch_normalization == 1


@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_oracle_matches_long_chain_fixture(name, disflow_mod, oracle):
    e = GOLDEN[name]
    p, I0, I1 = _inputs(disflow_mod, e)
    with oracle.threads():
        flow = oracle.calc_from_params(I0, I1, p)
    _check_against_fixture(flow, e, name)


def test_oracle_threads_do_not_change_results(disflow_mod, oracle):
    # the threaded patch loop is a speed knob of the checker only
    W, H = 160, 120
    p = disflow_mod.preset_params(disflow_mod.Preset.REFERENCE, W, H)
    p.iterations = 40
    I0, I1 = disflow_mod.synth_pair(11, W, H)
    a = oracle.calc_from_params(I0, I1, p)
    with oracle.threads(4):
        b = oracle.calc_from_params(I0, I1, p)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _bitexact(got, exp, what):
    bad = np.ascontiguousarray(got, np.float32).view(np.uint32) != np.ascontiguousarray(exp, np.float32).view(np.uint32)
    if bad.any():
        i = tuple(np.argwhere(bad)[0])
        raise AssertionError(f"{what}: {int(bad.sum())} of {bad.size} values differ; first at {list(i)} "
                             f"got {got[i]} exp {exp[i]}")


@pytest.mark.gpu
def test_reference_default_run_bitexact_on_gpu(disflow_mod, oracle):
    # both seeds as one batch (2 pairs, one sub-batch stream each) and pair 0
    # alone: the it = 1000 chain through every lane layout the auto choice uses
    # (levels 0-1 at 2 lanes per patch, levels 2-3 at 8)
    names = sorted(n for n in GOLDEN if n.startswith("reference_default"))
    es = [GOLDEN[n] for n in names]
    W, H = es[0]["W"], es[0]["H"]
    ins = [_inputs(disflow_mod, e) for e in es]
    p = ins[0][0]
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=len(es))
    got = eng.calc_batch(np.stack([x[1] for x in ins]), np.stack([x[2] for x in ins]))
    single = disflow_mod.DenseInverseSearch(p, W, H).calc(ins[0][1], ins[0][2])
    for k, (e, (_, I0, I1)) in enumerate(zip(es, ins)):
        with oracle.threads():
            exp = oracle.calc_from_params(I0, I1, p)
        _bitexact(got[k], exp, f"{names[k]} (batch)")
        _check_against_fixture(got[k], e, names[k])
    _bitexact(single, got[0], "single pair vs batch")


@pytest.mark.gpu
def test_slow_preset_full_iterations_with_refinement_bitexact_on_gpu(disflow_mod, oracle):
    # config 5's knobs at full iterations (it 128, F 0, steps 2, refinement on)
    (name,) = [n for n in GOLDEN if n.startswith("slow_full_iters")]
    e = GOLDEN[name]
    p, I0, I1 = _inputs(disflow_mod, e)
    assert p.iterations == 128 and p.var_refine_iters > 0
    got = disflow_mod.DenseInverseSearch(p, e["W"], e["H"]).calc(I0, I1)
    with oracle.threads():
        exp = oracle.calc_from_params(I0, I1, p)
    _bitexact(got, exp, name)
    _check_against_fixture(got, e, name)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
def test_fast_preset_1080p_bitexact_on_gpu(disflow_mod, oracle, variant):
    # the FAST preset (it 16, steps 4, F 2) at full 1920x1080; variant 1 forces
    # the generic one-lane-per-patch kernels
    (name,) = [n for n in GOLDEN if n.startswith("fast_1920")]
    e = GOLDEN[name]
    p, I0, I1 = _inputs(disflow_mod, e)
    eng = disflow_mod.DenseInverseSearch(p, e["W"], e["H"])
    eng.set_variant(variant)
    got = eng.calc(I0, I1)
    with oracle.threads():
        exp = oracle.calc_from_params(I0, I1, p)
    _bitexact(got, exp, name)
    _check_against_fixture(got, e, name)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [3, 4, 6])
def test_reference_default_lane_layouts_bitexact_on_gpu(disflow_mod, oracle, variant):
    # the it = 1000 chain on every level with one lane layout forced: 2 lanes
    # per patch (3), 8 lanes per patch (4), one wave per patch (6)
    e = GOLDEN[sorted(n for n in GOLDEN if n.startswith("reference_default"))[0]]
    p, I0, I1 = _inputs(disflow_mod, e)
    eng = disflow_mod.DenseInverseSearch(p, e["W"], e["H"])
    eng.set_variant(variant)
    _check_against_fixture(eng.calc(I0, I1), e, f"reference default, variant {variant}")
