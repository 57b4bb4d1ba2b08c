"""CPU tests of the oracle (the checker): it is compared with an independent
numpy restatement (tests/pyref.py), with the reference's documented quirks
 and with the committed golden fixtures (tests/golden/).

Parity status: UNPINNED against the reference itself -- the reference has no
tests, fixtures or golden vectors and cannot be built here (OpenCV 2.4 and
Eigen 3 are absent); see DESIGN.md "Oracle".
"""
import math
import os

import numpy as np
import pytest

import pyref

f32 = np.float32
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def smooth_noise(rng, H, W, blur=2):
    a = rng.integers(0, 256, size=(H + 2 * blur, W + 2 * blur)).astype(np.float64)
    k = np.ones(2 * blur + 1) / (2 * blur + 1)
    a = np.apply_along_axis(lambda r: np.convolve(r, k, "valid"), 1, a)
    a = np.apply_along_axis(lambda c: np.convolve(c, k, "valid"), 0, a)
    a = (a - a.mean()) / (a.std() + 1e-9) * 45 + 128
    return np.clip(np.round(a), 0, 255).astype(np.uint8)


def shifted_pair(seed, H, W, dx=1.3, dy=-0.7):
    rng = np.random.default_rng(seed)
    big = smooth_noise(rng, H + 16, W + 16)
    I0 = big[8:8 + H, 8:8 + W]
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    sx, sy = xx + 8 - dx, yy + 8 - dy
    x0, y0 = np.floor(sx).astype(int), np.floor(sy).astype(int)
    fx, fy = sx - x0, sy - y0
    b = big.astype(np.float64)
    v = (b[y0, x0] * (1 - fx) * (1 - fy) + b[y0, x0 + 1] * fx * (1 - fy)
         + b[y0 + 1, x0] * (1 - fx) * fy + b[y0 + 1, x0 + 1] * fx * fy)
    I1 = np.clip(np.round(v), 0, 255).astype(np.uint8)
    return np.ascontiguousarray(I0), np.ascontiguousarray(I1)


# --- reference quirks --------------------------------------

def test_q8_ceil_epsilon_is_noop_from_256():
    # ceil(x + 1e-5f) in float32 (src/patch.cpp:233-234)
    assert np.ceil(f32(300) + f32(1e-5)) == 300
    assert np.ceil(f32(200) + f32(1e-5)) == 201
    first = next(i for i in range(1, 1000) if f32(i) + f32(1e-5) == f32(i))
    assert first == 256


def test_q12_steps_float_floor(oracle):
    assert oracle.steps(12, 1.0 / 3.0) == 7   # float floor, not 8
    assert oracle.steps(8, 0.7) == 2          # reference CLI default
    assert oracle.steps(8, 0.625) == 3        # MEDIUM
    assert oracle.steps(8, 0.5) == 4          # ULTRAFAST / FAST
    assert oracle.steps(8, 0.95) == 1         # max(1, .)


def test_grid_geometry_medium_1080p(oracle):
    # level sizes and patch counts of SURVEY.md 8a row a7
    counts = []
    for l in range(1, 7):
        npw, nph, _, _ = oracle.grid(1920 >> l, 1088 >> l, 3)
        counts.append(npw * nph)
    assert counts == [58240, 14560, 3680, 920, 240, 60]
    assert sum(counts) == 77700


def test_padding_split(oracle):
    assert oracle.padded_size(1920, 1080, 6) == (1920, 1088, 0, 4)
    assert oracle.padded_size(641, 483, 3) == (648, 488, 3, 2)


# --- oracle vs independent numpy restatement --------------------------------

@pytest.mark.parametrize("shape", [(24, 40), (33, 17), (8, 8)])
def test_sobel_matches_numpy(oracle, shape):
    rng = np.random.default_rng(1)
    img = rng.random(shape, dtype=np.float32) * 255
    dx, dy = oracle.sobel(img)
    rx, ry = pyref.sobel(img)
    assert np.array_equal(dx, rx) and np.array_equal(dy, ry)


def test_pyramid_matches_numpy(oracle):
    I0, _ = shifted_pair(3, 48, 64)
    f0 = oracle.pad_convert(I0, 3)
    got = oracle.pyramid(f0, 3)
    ref = pyref.pyramid(f0, 3)
    for (a, b, c), (x, y, z) in zip(got, ref):
        assert np.array_equal(a, x) and np.array_equal(b, y) and np.array_equal(c, z)


def test_level0_is_sobel_magnitude(oracle):
    # Q1: the "image" at level 0 is sqrt(dx^2 + dy^2) of the input
    I0, _ = shifted_pair(4, 32, 32)
    f0 = oracle.pad_convert(I0, 2)
    lv0 = oracle.pyramid(f0, 2)[0][0]
    gx, gy = oracle.sobel(f0)
    assert np.array_equal(lv0, np.sqrt(gx * gx + gy * gy))


@pytest.mark.parametrize("ps,overlap,it,norm", [(8, 0.625, 4, 1), (4, 0.5, 3, 1), (6, 0.5, 2, 0),
                                                (8, 0.7, 2, 1)])
def test_patch_search_matches_numpy(oracle, ps, overlap, it, norm):
    W, H, C, F = 64, 48, 2, 0
    I0, I1 = shifted_pair(5, H, W)
    Wp, Hp, P0, PX, PY, P1, py0, py1 = oracle.build_pyramids(I0, I1, C, ps)
    out, us, ds = oracle.flow_from_pyramids(P0, PX, PY, P1, ps, Wp, Hp, C, F, it, ps, overlap, norm,
                                            capture=True)
    st = oracle.steps(ps, overlap)
    prev = None
    for l in range(C, F - 1, -1):
        w, h = Wp >> l, Hp >> l
        if prev is None:
            init = None
        else:
            def init(pid, rx, ry, prev=prev, w=w):
                x, y = int(np.floor(rx / f32(2))), int(np.floor(ry / f32(2)))
                v = prev[y, x]
                return v[0] * f32(2), v[1] * f32(2)
        u, geom = pyref.search_level(PX[l], PY[l], P1[l], ps, w, h, ps, st, it, norm, init)
        assert np.array_equal(u, us[l]), f"patch u differs at level {l}"
        d = pyref.densify(u, geom, w, h, ps, st)
        assert np.array_equal(d, ds[l]), f"dense differs at level {l}"
        prev = d
    assert np.array_equal(out, ds[F])


def test_upsample_matches_formula(oracle):
    rng = np.random.default_rng(9)
    for F in (1, 2):
        Wp, Hp = 32, 24
        fl = rng.standard_normal((Hp >> F, Wp >> F, 2)).astype(np.float32)
        got = oracle.upsample_crop(fl, Wp, Hp, F, 0, 0, Wp, Hp)
        # independent restatement of cv::resize INTER_LINEAR x2^F
        s = fl * f32(2 ** F)
        n_w, n_h = Wp >> F, Hp >> F

        def coefs(nd, ns):
            idx, fr, two = [], [], []
            xmax = nd
            for d in range(nd):
                fx = f32((d + 0.5) * (1.0 / 2 ** F) - 0.5)
                sx = int(np.floor(fx))
                fx = f32(fx - f32(sx))
                if sx < 0:
                    fx, sx = f32(0), 0
                if sx + 1 >= ns:
                    xmax = min(xmax, d)
                    if sx >= ns - 1:
                        fx, sx = f32(0), ns - 1
                idx.append(sx)
                fr.append(fx)
            return idx, fr, [d < xmax for d in range(nd)]

        xi, xf, xt = coefs(Wp, n_w)
        yi, yf, _ = coefs(Hp, n_h)
        hrow = np.empty((n_h, Wp, 2), np.float32)
        for x in range(Wp):
            if xt[x]:
                hrow[:, x] = s[:, xi[x]] * (f32(1) - xf[x]) + s[:, xi[x] + 1] * xf[x]
            else:
                hrow[:, x] = s[:, xi[x]]
        exp = np.empty((Hp, Wp, 2), np.float32)
        for y in range(Hp):
            r1 = min(yi[y] + 1, n_h - 1)
            exp[y] = hrow[yi[y]] * (f32(1) - yf[y]) + hrow[r1] * yf[y]
        assert np.array_equal(got, exp)


def test_q2_identical_frames_do_not_give_zero_flow(oracle):
    # no template subtraction in the residual (src/patch.cpp:171-172)
    I0, _ = shifted_pair(6, 64, 64)
    flow = oracle.calc_u8(I0, I0, C=2, F=0, ps=8, it=8, overlap=0.5)
    assert np.abs(flow).max() > 0.01


def test_translation_is_recovered_roughly(oracle):
    I0, I1 = shifted_pair(7, 96, 128, dx=1.5, dy=0.75)
    flow = oracle.calc_u8(I0, I1, C=3, F=0, ps=8, it=16, overlap=0.5)
    inner = flow[16:-16, 16:-16]
    med = np.median(inner.reshape(-1, 2), axis=0)
    # biased by Q2 but in the right direction and magnitude
    assert 0.5 < med[0] < 2.5 and 0.2 < med[1] < 1.5


def test_deterministic(oracle):
    I0, I1 = shifted_pair(8, 48, 64)
    a = oracle.calc_u8(I0, I1, C=2, F=1, ps=8, it=5, overlap=0.625)
    b = oracle.calc_u8(I0, I1, C=2, F=1, ps=8, it=5, overlap=0.625)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


# --- golden fixtures (regression lock of the oracle) ------------------------

def _golden_files():
    if not os.path.isdir(GOLDEN):
        return []
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz"))


@pytest.mark.parametrize("name", _golden_files())
def test_golden_fixture(oracle, name):
    z = np.load(os.path.join(GOLDEN, name))  # allow_pickle=False (default)
    C, F, ps, it, norm = (int(v) for v in z["knobs_i"])
    overlap = float(z["knobs_f"][0])
    flow = oracle.calc_u8(z["I0"], z["I1"], C=C, F=F, ps=ps, it=it, overlap=overlap, norm=norm)
    assert np.array_equal(flow.view(np.uint32), z["flow"].view(np.uint32))


def test_pad_convert_matches_numpy(oracle):
    # a1: replicate pad to a multiple of 2^C with floor/ceil split (src/main.cpp:139-160)
    rng = np.random.default_rng(12)
    img = rng.integers(0, 256, size=(151, 203), dtype=np.uint8)
    got = oracle.pad_convert(img, 3)
    exp = np.pad(img, ((0, 1), (2, 3)), mode="edge").astype(np.float32)  # 152 x 208
    assert got.shape == (152, 208) and np.array_equal(got, exp)


def _color_cases():
    rng = np.random.default_rng(5)
    f = (rng.standard_normal((37, 53, 2)) * 4).astype(np.float32)
    f[0, 0] = (np.nan, 1)
    f[0, 1] = (1, np.inf)
    f[0, 2] = (2e9, 0)
    f[0, 3] = (0, 0)
    f[0, 4] = (-0.0, 0.0)
    f[1, :8] = [(1, 0), (0, 1), (-1, 0), (0, -1), (3, 4), (-3, 4), (1e-30, 0), (-7, -7)]
    return f


@pytest.mark.parametrize("maxmotion", [-1.0, 0.0, 2.5, 100.0])
def test_flow_color_oracle_matches_numpy(oracle, maxmotion):
    f = _color_cases()
    assert np.array_equal(oracle.flow_color(f, maxmotion), pyref.flow_color(f, maxmotion))


def test_flow_color_known_answers(oracle):
    # src/color_coding.cpp: zero motion is white, invalid is black, the unit
    # vector +x maps to wheel[0] (red) at full saturation, +y to wheel 13/14
    f = np.zeros((1, 4, 2), np.float32)
    f[0, 1] = (1, 0)
    f[0, 2] = (0, 1)
    f[0, 3] = (np.nan, 0)
    c = oracle.flow_color(f, 1.0)
    assert c[0, 0].tolist() == [255, 255, 255]
    assert c[0, 1].tolist() == [0, 0, 255]
    assert c[0, 2].tolist() == [0, 229, 255]
    assert c[0, 3].tolist() == [0, 0, 0]


# ---- variational refinement (not in the reference) ----------

def _vr_case(seed, W=160, H=120):
    import disflow
    I0, I1, gt = disflow.synth_pair(seed, W, H, with_gt=True)
    lv0 = [oracle_binding_levels(I) for I in (I0, I1)]
    return I0, I1, gt, lv0[0], lv0[1]


def oracle_binding_levels(I):
    import oracle_binding as ob
    return ob.pyramid(ob.pad_convert(I, 0), 0)[0][0]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_var_refine_decreases_energy(oracle, seed):
    # energy of the refined DIS flow below that of the unrefined one (the
    # refinement's purpose), on the level-0 images the path refines on
    I0, I1, gt, m0, m1 = _vr_case(seed)
    flow = oracle.calc_u8(I0, I1, 3, 0, 8, 12, 0.5)
    e0 = oracle.var_energy(m0, m1, flow)
    for fp in (1, 2, 3):
        assert oracle.var_energy(m0, m1, oracle.var_refine(m0, m1, flow, fp)) < e0


def test_var_refine_zero_iterations_is_identity(oracle):
    I0, I1, gt, m0, m1 = _vr_case(4)
    flow = oracle.calc_u8(I0, I1, 3, 0, 8, 12, 0.5)
    assert np.array_equal(oracle.var_refine(m0, m1, flow, 0), flow)
    assert np.array_equal(oracle.calc_u8(I0, I1, 3, 0, 8, 12, 0.5, 1, 0), flow)


def test_var_refine_improves_synthetic_accuracy(oracle):
    # mean end-point error vs the generator's ground truth over seeds, the whole
    # coarse-to-fine path with refinement on every level (3 fixed-point iterations)
    import disflow
    e = {0: [], 3: []}
    for seed in (3, 4, 5, 6):
        I0, I1, gt = disflow.synth_pair(seed, 320, 240, with_gt=True)
        for vr in e:
            f = oracle.calc_u8(I0, I1, 4, 0, 8, 16, 0.75, 1, vr)
            e[vr].append(np.sqrt(((f - gt) ** 2).sum(-1)).mean())
    assert np.mean(e[3]) < 0.85 * np.mean(e[0])


# --- paper mode (DIS-paper residual + weighted densification) --
# Not in the reference (parity unpinned by construction): the C oracle's
# restatement is cross-checked by the independent numpy one, plus known answers.

@pytest.mark.parametrize("ps,overlap,it,norm", [(8, 0.625, 4, 1), (4, 0.5, 3, 0), (8, 0.7, 2, 1)])
def test_paper_mode_matches_numpy(oracle, ps, overlap, it, norm):
    W, H, C, F = 64, 48, 2, 0
    I0, I1 = shifted_pair(15, H, W)
    Wp, Hp, P0, PX, PY, P1, py0, py1 = oracle.build_pyramids(I0, I1, C, ps)
    out, us, ds = oracle.flow_from_pyramids(P0, PX, PY, P1, ps, Wp, Hp, C, F, it, ps, overlap, norm,
                                            capture=True, paper=1)
    st = oracle.steps(ps, overlap)
    prev = None
    for l in range(C, F - 1, -1):
        w, h = Wp >> l, Hp >> l
        if prev is None:
            init = None
        else:
            def init(pid, rx, ry, prev=prev, w=w):
                x, y = int(np.floor(rx / f32(2))), int(np.floor(ry / f32(2)))
                v = prev[y, x]
                return v[0] * f32(2), v[1] * f32(2)
        u, geom = pyref.search_level(PX[l], PY[l], P1[l], ps, w, h, ps, st, it, norm, init, I0p=P0[l])
        assert np.array_equal(u, us[l]), f"paper patch u differs at level {l}"
        i0 = P0[l][ps:ps + h, ps:ps + w]
        i1 = P1[l][ps:ps + h, ps:ps + w]
        d = pyref.densify_paper(u, geom, i0, i1, w, h, ps, st)
        assert np.array_equal(d, ds[l]), f"paper dense differs at level {l}"
        prev = d
    assert np.array_equal(out, ds[F])


def test_paper_mode_identical_frames_give_zero_flow(oracle):
    # with the template subtracted, identical frames give b = 0 exactly at u = 0
    # (below 256 px, where Q8's ceil(x + 1e-5f) still samples the template's own
    # pixels): zero flow everywhere -- unlike the reference (Q2)
    I0, _ = shifted_pair(6, 64, 64)
    flow = oracle.calc_u8(I0, I0, C=2, F=0, ps=8, it=8, overlap=0.5, paper=1)
    assert np.array_equal(flow, np.zeros_like(flow))
    assert np.abs(oracle.calc_u8(I0, I0, C=2, F=0, ps=8, it=8, overlap=0.5)).max() > 0.01


def test_paper_mode_is_more_accurate_on_synthetic_pairs(oracle):
    import disflow
    e = {0: [], 1: []}
    for seed in (0, 1, 2):
        I0, I1, gt = disflow.synth_pair(seed, 320, 240, with_gt=True)
        p = disflow.preset_params(disflow.Preset.MEDIUM, 320, 240)
        for paper in e:
            p.paper_mode = paper
            f = oracle.calc_from_params(I0, I1, p)
            e[paper].append(np.sqrt(((f - gt) ** 2).sum(-1)).mean())
    assert np.mean(e[1]) < 0.85 * np.mean(e[0])


# --- tolerance calibration (tools/tolerance.py, profiles/tolerance_r01.json) --

def test_rounding_order_spread_within_stated_tolerance(oracle):
    # the restatement built with another reduction order / FMA contraction moves
    # the flow by far less than the tolerance DESIGN.md 2 states against the
    # (unbuildable) reference; small case of tools/tolerance.py
    import json
    import subprocess

    import disflow
    subprocess.check_call(["make", "-s", "-C", oracle.ORACLE_DIR, "variants"])
    sys_path = os.path.join(oracle.ROOT, "tools")
    import importlib.util
    spec = importlib.util.spec_from_file_location("tolerance", os.path.join(sys_path, "tolerance.py"))
    tol = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tol)
    stated = json.load(open(os.path.join(oracle.ROOT, "profiles", "tolerance_r01.json")))["stated_tolerance"]
    W, H = 320, 240
    p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
    I0, I1 = disflow.synth_pair(3, W, H)
    base = oracle.calc_from_params(I0, I1, p)
    for v in tol.VARIANTS:
        e = tol.epe(tol.with_lib(tol.load_variant(v), oracle.calc_from_params, I0, I1, p), base)
        assert 0 < e.max(), v  # the variants do change the rounding
        assert e.mean() <= stated["mean_epe"] and np.percentile(e, 99.9) <= stated["p999_epe"], v


def test_flip_mask_reach():
    # tests/flipmask.py: a flipped finest-level patch masks its footprint
    # (+1 level-F pixel for the upsample) at full resolution, nothing else
    from flipmask import flip_mask, grid, outside_max_epe
    W, H, C, F, ps, st = 64, 48, 2, 1, 8, 3
    npw, nph, offw, offh = grid(32, 24, st)
    u = np.zeros((npw * nph, 2), np.float32)
    v = u.copy()
    m, d = flip_mask(u, v, W, H, C, F, ps, st)
    assert not m.any() and (d == 0).all()
    gx, gy = 4, 3
    v[gx * nph + gy] = (0.6, 0.0)
    m, _ = flip_mask(u, v, W, H, C, F, ps, st)
    cx, cy = gx * st + offw, gy * st + offh
    ys, xs = np.nonzero(m)
    assert (xs.min(), xs.max() + 1) == ((cx - 5) * 2, (cx + 5) * 2)
    assert (ys.min(), ys.max() + 1) == ((cy - 5) * 2, (cy + 5) * 2)
    f0 = np.zeros((H, W, 2), np.float32)
    f1 = f0.copy()
    f1[ys[0], xs[0]] = (3.0, 4.0)  # inside the site: not counted
    f1[0, W - 1] = (0.0, 0.25)
    mx, frac = outside_max_epe(f1, f0, m)
    assert mx == 0.25 and 0 < frac < 1
    v[0] = (np.nan, 0.0)  # NaN counts as a flip
    assert flip_mask(u, v, W, H, C, F, ps, st)[0][0, 0]
