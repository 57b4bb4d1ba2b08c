"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle on
the same inputs. The bar is BIT-EXACT float32 equality: the kernels evaluate
the reference's float32 expressions in the reference's order (no FMA
contraction, correctly rounded division and sqrt, Eigen's reduction order),
so any difference is a bug, not rounding. (The oracle's own agreement with the
reference is unpinned; see DESIGN.md.)"""
import numpy as np
import pytest

import test_oracle as helpers

pytestmark = pytest.mark.gpu


def _assert_bitexact(got, exp, what):
    got = np.ascontiguousarray(got, np.float32)
    exp = np.ascontiguousarray(exp, np.float32)
    assert got.shape == exp.shape, (what, got.shape, exp.shape)
    bad = got.view(np.uint32) != exp.view(np.uint32)
    if bad.any():
        idx = np.argwhere(bad)
        d = np.abs(got.astype(np.float64) - exp.astype(np.float64))
        raise AssertionError(f"{what}: {bad.sum()} of {bad.size} values differ; first at {idx[0].tolist()} "
                             f"got {got[tuple(idx[0])]} exp {exp[tuple(idx[0])]}; max |diff| {np.nanmax(d)}")


def _params(disflow, C, F, ps, it, overlap, norm=1):
    return disflow.Params(coarsest_scale=C, finest_scale=F, patch_size=ps, iterations=it,
                          patch_overlap=overlap, patch_normalization=norm)


CASES = [
    # (W, H, C, F, ps, it, overlap, norm)
    (640, 480, 4, 2, 8, 12, 0.5, 1),      # config 1: ULTRAFAST 640x480
    (160, 120, 3, 1, 8, 25, 0.625, 1),    # MEDIUM knobs, small
    (203, 151, 3, 0, 8, 10, 0.7, 1),      # ragged size (padding), reference overlap
    (96, 64, 2, 0, 4, 6, 0.5, 1),         # ps 4
    (96, 64, 2, 1, 6, 5, 0.5, 0),         # ps 6, no normalization
    (128, 96, 2, 0, 10, 4, 0.6, 1),       # ps 10
    (64, 48, 1, 0, 16, 3, 0.75, 1),       # ps 16
    (37, 29, 2, 2, 2, 3, 0.0, 1),         # ps 2, F == C
    (64, 64, 3, 0, 8, 0, 0.5, 1),         # iterations 0 (one update)
    (1000, 200, 4, 1, 8, 6, 0.5, 1),      # pyramid dword row loads (stride, pad_left 4- not 16-byte aligned)
    (432, 320, 4, 1, 8, 6, 0.5, 1),       # pyramid 16-byte row loads, 16 x 16 tiles
    (420, 300, 4, 1, 8, 6, 0.5, 1),       # pad_left 6: byte row loads
    (800, 600, 5, 2, 8, 8, 0.5, 1),       # C = 5: register pyramid tail, partial 16 x 16 super-tiles
    (100, 80, 2, 0, 8, 6, 0.5, 1),        # C = 2, W_2 = 25 odd: k_pyr12 scalar level-1/2 stores
    (104, 72, 3, 1, 8, 5, 0.5, 1),        # C = 3, W_2 = 26 = 2 mod 4: scalar stores, register tail level 3
]


@pytest.mark.parametrize("W,H,C,F,ps,it,overlap,norm", [c for c in CASES if c[4] == 8])
def test_wave_per_patch_bitexact(disflow_mod, oracle, W, H, C, F, ps, it, overlap, norm):
    # the north star's mapping (k_search_wave: one wave64 per patch, lane = pixel,
    # Eigen-order cross-lane sums) on every level, incl. ragged sizes, F == 0,
    # no normalisation and iterations 0; paper mode falls back to 2 lanes/patch
    I0, I1 = disflow_mod.synth_pair(W * 5 + H, W, H)
    p = _params(disflow_mod, C, F, ps, it, overlap, norm)
    eng = disflow_mod.DenseInverseSearch(p, W, H)
    eng.set_variant(6)
    _assert_bitexact(eng.calc(I0, I1), oracle.calc_from_params(I0, I1, p), "wave per patch")
    p.paper_mode = 1
    eng = disflow_mod.DenseInverseSearch(p, W, H)
    eng.set_variant(6)
    _assert_bitexact(eng.calc(I0, I1), oracle.calc_from_params(I0, I1, p), "wave per patch, paper mode")


@pytest.mark.parametrize("W,H,C,F,ps,it,overlap,norm", CASES)
def test_end_to_end_bitexact(disflow_mod, oracle, W, H, C, F, ps, it, overlap, norm):
    I0, I1 = disflow_mod.synth_pair(W * 7 + H, W, H)
    p = _params(disflow_mod, C, F, ps, it, overlap, norm)
    eng = disflow_mod.DenseInverseSearch(p, W, H)
    got = eng.calc(I0, I1)
    exp = oracle.calc_u8(I0, I1, C, F, ps, it, overlap, norm)
    _assert_bitexact(got, exp, f"flow {W}x{H}")


@pytest.mark.parametrize("W,H", [(998, 202), (1000, 202), (998, 200), (1000, 200), (259, 197)])
def test_output_interior_tiles_every_pad_parity(disflow_mod, oracle, W, H):
    # k_output's interior-tile path at F == 1 specialises on the parities of
    # pad_top and pad_left (odd / even padding of Wp x Hp) -- all four, plus
    # the border tiles of the general path around them
    I0, I1 = disflow_mod.synth_pair(W + 3 * H, W, H)
    p = _params(disflow_mod, 4, 1, 8, 8, 0.625)
    eng = disflow_mod.DenseInverseSearch(p, W, H)
    _assert_bitexact(eng.calc(I0, I1), oracle.calc_from_params(I0, I1, p), f"flow {W}x{H}")


def test_large_shift_outliers_bitexact(disflow_mod, oracle):
    # big translation: many patches hit the outlier reset / OOB start (Q4, Q5)
    I0, I1 = helpers.shifted_pair(11, 120, 160, dx=9.5, dy=-7.25)
    p = _params(disflow_mod, 2, 0, 8, 20, 0.5)
    got = disflow_mod.DenseInverseSearch(p, 160, 120).calc(I0, I1)
    _assert_bitexact(got, oracle.calc_u8(I0, I1, 2, 0, 8, 20, 0.5), "flow")


def test_flat_image_singular_hessian(disflow_mod, oracle):
    # constant frames: zero gradients, det == 0 regularisation (Q10)
    I0 = np.full((48, 64), 77, np.uint8)
    I1 = I0.copy()
    I1[20:30, 20:40] = 200
    p = _params(disflow_mod, 2, 0, 8, 5, 0.5)
    got = disflow_mod.DenseInverseSearch(p, 64, 48).calc(I0, I1)
    _assert_bitexact(got, oracle.calc_u8(I0, I1, 2, 0, 8, 5, 0.5), "flow")


def test_stage_dumps_bitexact(disflow_mod, oracle):
    W, H, C, F, ps, it, ov = 200, 136, 3, 1, 8, 8, 0.625
    I0, I1 = disflow_mod.synth_pair(5, W, H)
    eng = disflow_mod.DenseInverseSearch(_params(disflow_mod, C, F, ps, it, ov), W, H)
    eng.set_debug(True)
    eng.calc(I0, I1)
    Wp, Hp, P0, PX, PY, P1, py0, py1 = oracle.build_pyramids(I0, I1, C, ps)
    _, us, ds = oracle.flow_from_pyramids(P0, PX, PY, P1, ps, Wp, Hp, C, F, it, ps, ov, 1, capture=True)
    S = disflow_mod
    for l in range(C + 1):
        _assert_bitexact(eng.debug_dump(S.STAGE_IMG0, l).reshape(py0[l][0].shape), py0[l][0], f"img0 l{l}")
        _assert_bitexact(eng.debug_dump(S.STAGE_IMG1, l).reshape(py1[l][0].shape), py1[l][0], f"img1 l{l}")
    for l in range(F, C + 1):
        _assert_bitexact(eng.debug_dump(S.STAGE_DX0, l).reshape(py0[l][1].shape), py0[l][1], f"dx l{l}")
        _assert_bitexact(eng.debug_dump(S.STAGE_DY0, l).reshape(py0[l][2].shape), py0[l][2], f"dy l{l}")
        _assert_bitexact(eng.debug_dump(S.STAGE_PATCH_U, l).reshape(-1, 2), us[l], f"patch u l{l}")
        _assert_bitexact(eng.debug_dump(S.STAGE_DENSE, l).reshape(ds[l].shape), ds[l], f"dense l{l}")


@pytest.mark.parametrize("W,H,C,F,ps,it,ov,kind", [
    (160, 128, 3, 1, 8, 10, 0.7, "synth"),
    (1920, 1080, 6, 1, 8, 25, 0.625, "synth"),      # config 2 knobs: the fast kernel, 2 and 8 lanes/patch
    (640, 480, 4, 2, 8, 12, 0.5, "unrelated"),      # spread blocks: the tile fallback on physical planes
    (320, 240, 3, 0, 6, 8, 0.5, "synth"),           # patch size 6: the generic kernel
])
def test_compat_constructor_path_bitexact(disflow_mod, oracle, W, H, C, F, ps, it, ov, kind):
    # OpticalFlowClass(...) semantics over caller-built padded pyramids
    # (include/optical_flow.hpp:43-54): repeated calls reuse the cached workspace
    if kind == "unrelated":
        I0, _ = disflow_mod.synth_pair(5, W, H)
        I1, _ = disflow_mod.synth_pair(6, W, H)
    else:
        I0, I1 = disflow_mod.synth_pair(21 + W, W, H)
    Wp, Hp, P0, PX, PY, P1, _, _ = oracle.build_pyramids(I0, I1, C, ps)
    exp = oracle.flow_from_pyramids(P0, PX, PY, P1, ps, Wp, Hp, C, F, it, ps, ov, 1)
    for _ in range(2):
        got = disflow_mod.optical_flow_from_pyramids(P0, PX, PY, P1, ps, Wp, Hp, C, F, it, ps, ov, True)
        _assert_bitexact(got, exp, f"compat flow {W}x{H} ps {ps} {kind}")


def test_batch_equals_single_and_deterministic(disflow_mod):
    W, H = 176, 144
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    pairs = [disflow_mod.synth_pair(s, W, H) for s in range(4)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=4)
    batch = eng.calc_batch(I0, I1)
    again = eng.calc_batch(I0, I1)
    assert np.array_equal(batch.view(np.uint32), again.view(np.uint32))
    for streams in (1, 3, 8):
        eng.set_concurrency(streams)
        other = eng.calc_batch(I0, I1)
        assert np.array_equal(other.view(np.uint32), batch.view(np.uint32)), streams
    single = disflow_mod.DenseInverseSearch(p, W, H)
    for k in range(4):
        one = single.calc(I0[k], I1[k])
        assert np.array_equal(one.view(np.uint32), batch[k].view(np.uint32)), k


def test_device_resident_path(disflow_mod):
    import torch
    W, H = 320, 240
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    I0, I1 = disflow_mod.synth_pair(2, W, H)
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=2)
    host = eng.calc(I0, I1)
    d0 = torch.from_numpy(np.stack([I0, I0])).cuda()
    d1 = torch.from_numpy(np.stack([I1, I1])).cuda()
    out = torch.empty((2, H, W, 2), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    eng.calc_device(2, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
    s.synchronize()
    o = out.cpu().numpy()
    assert np.array_equal(o[0].view(np.uint32), host.view(np.uint32))
    assert np.array_equal(o[1].view(np.uint32), host.view(np.uint32))


def test_calls_on_different_streams_do_not_race(disflow_mod):
    # a one-pair call runs on the caller's stream without the
    # fork/join events; the next call on another stream (host mode runs on the
    # context's own stream) must still wait for it before reusing the workspace
    import torch
    W, H = 1280, 720
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    X0, X1 = disflow_mod.synth_pair(31, W, H)
    Y0, Y1 = disflow_mod.synth_pair(32, W, H)
    ref = disflow_mod.DenseInverseSearch(p, W, H, max_batch=1)
    ex, ey = ref.calc(X0, X1), ref.calc(Y0, Y1)
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=2)
    d0 = torch.from_numpy(X0[None]).cuda()
    d1 = torch.from_numpy(X1[None]).cuda()
    out = torch.empty((1, H, W, 2), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    for _ in range(3):
        out.zero_()
        eng.calc_device(1, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), side.cuda_stream)
        gy = eng.calc(Y0, Y1)  # no synchronisation in between
        side.synchronize()
        assert np.array_equal(out[0].cpu().numpy().view(np.uint32), ex.view(np.uint32))
        assert np.array_equal(gy.view(np.uint32), ey.view(np.uint32))


def test_graph_replay_matches_eager_and_tracks_its_key(disflow_mod):
    # dis_set_graphs (default on): a batch call is captured once per key and
    # replayed; new buffers, batch sizes, concurrency and precision re-capture.
    # Every replay must equal the eager path bit for bit.
    import torch
    W, H, B = 640, 480, 4
    d = disflow_mod
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    pairs = [d.synth_pair(70 + k, W, H) for k in range(B)]
    X0 = np.stack([a for a, _ in pairs])
    X1 = np.stack([b for _, b in pairs])
    eager = d.DenseInverseSearch(p, W, H, max_batch=B)
    eager.set_graphs(False)
    ref = eager.calc_batch(X0, X1)
    eng = d.DenseInverseSearch(p, W, H, max_batch=B)
    s = torch.cuda.current_stream()
    bufs = [(torch.from_numpy(X0).cuda(), torch.from_numpy(X1).cuda(),
             torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")) for _ in range(2)]
    for rep in range(3):
        for k, (d0, d1, out) in enumerate(bufs):  # alternating keys: re-capture every call
            for n in (B, 2):
                out.fill_(float("nan"))
                eng.calc_device(n, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
                torch.cuda.synchronize()
                assert np.array_equal(out[:n].cpu().numpy().view(np.uint32), ref[:n].view(np.uint32)), (rep, k, n)
    d0, d1, out = bufs[0]
    for streams in (1, 3):
        eng.set_concurrency(streams)
        for _ in range(2):  # capture, then replay
            out.fill_(float("nan"))
            eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32)), streams
    eng.set_precision(d.PRECISION_FMA)  # a new key: the FMA kernels must run, not the cached exact graph
    eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    assert not np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(eng.calc_batch(X0, X1).view(np.uint32), out.cpu().numpy().view(np.uint32))


def test_graph_cache_ping_pong_without_synchronisation(disflow_mod):
    # a caller alternating buffer sets on one stream with no
    # synchronisation. The graph cache keeps an exec per key (LRU of 4) and
    # never updates an exec while its previous replay may still run: every
    # output must equal the eager result bit for bit.
    import torch
    W, H, B = 640, 480, 2
    d = disflow_mod
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    sets = []
    for j in range(6):  # 6 keys > the 4 cache slots: evictions under load too
        pairs = [d.synth_pair(300 + 2 * j + k, W, H) for k in range(B)]
        sets.append((np.stack([a for a, _ in pairs]), np.stack([b for _, b in pairs])))
    eager = d.DenseInverseSearch(p, W, H, max_batch=B)
    eager.set_graphs(False)
    refs = [eager.calc_batch(X0, X1) for X0, X1 in sets]
    eng = d.DenseInverseSearch(p, W, H, max_batch=B)
    s = torch.cuda.Stream()
    dev = [(torch.from_numpy(X0).cuda(), torch.from_numpy(X1).cuda()) for X0, X1 in sets]
    torch.cuda.synchronize()
    order = [0, 1, 0, 1, 0, 1, 2, 3, 4, 5, 0, 1, 0, 5, 4, 3]
    outs = []
    for j in order:
        out = torch.full((B, H, W, 2), float("nan"), device="cuda")
        torch.cuda.synchronize()
        outs.append(out)
        eng.calc_device(B, dev[j][0].data_ptr(), dev[j][1].data_ptr(), out.data_ptr(), s.cuda_stream)
    s.synchronize()
    for i, (j, out) in enumerate(zip(order, outs)):
        assert np.array_equal(out.cpu().numpy().view(np.uint32), refs[j].view(np.uint32)), (i, j)


def test_two_contexts_two_batches_in_flight(disflow_mod):
    # bench.py `pipelined` (serving form): two contexts, calls alternating on
    # two caller streams, so two batches are in flight on the shared sub-batch
    # streams; every batch must come out bit for bit (graphs and eager), and
    # destroying one side must leave the other working
    import torch
    W, H, B = 640, 480, 4
    d = disflow_mod
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    sets = []
    for j in range(3):
        pairs = [d.synth_pair(700 + 5 * j + k, W, H) for k in range(B)]
        sets.append((np.stack([a for a, _ in pairs]), np.stack([b for _, b in pairs])))
    ref_eng = d.DenseInverseSearch(p, W, H, max_batch=B)
    refs = [ref_eng.calc_batch(X0, X1) for X0, X1 in sets]
    for graphs in (True, False):
        engs = [d.DenseInverseSearch(p, W, H, max_batch=B) for _ in range(2)]
        for e in engs:
            e.set_concurrency(1)
            e.set_graphs(graphs)
        strs = [torch.cuda.Stream() for _ in range(2)]
        dev = [(torch.from_numpy(X0).cuda(), torch.from_numpy(X1).cuda()) for X0, X1 in sets]
        torch.cuda.synchronize()
        outs = []
        for k in range(12):
            j = k % 3
            o = torch.full((B, H, W, 2), float("nan"), device="cuda")
            torch.cuda.synchronize()
            outs.append((j, o))
            engs[k % 2].calc_device(B, dev[j][0].data_ptr(), dev[j][1].data_ptr(), o.data_ptr(), strs[k % 2].cuda_stream)
        torch.cuda.synchronize()
        for k, (j, o) in enumerate(outs):
            assert np.array_equal(o.cpu().numpy().view(np.uint32), refs[j].view(np.uint32)), (graphs, k)
        engs[1].close()  # engine 0 keeps working alone
        got = engs[0].calc_batch(*sets[0])
        assert np.array_equal(got.view(np.uint32), refs[0].view(np.uint32))
        engs[0].close()


def test_two_threads_two_contexts(disflow_mod):
    # contexts on one device share the pooled sub-batch streams;
    # two host threads, each with its own context (graph capture + replay, and
    # eager calls), must both get their own results bit for bit
    import threading
    import torch
    W, H, B = 640, 480, 4
    d = disflow_mod
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    jobs = []
    for t in range(2):
        pairs = [d.synth_pair(500 + 10 * t + k, W, H) for k in range(B)]
        X0 = np.stack([a for a, _ in pairs])
        X1 = np.stack([b for _, b in pairs])
        ref = d.DenseInverseSearch(p, W, H, max_batch=B)
        ref.set_graphs(False)
        jobs.append((X0, X1, ref.calc_batch(X0, X1)))
    errors = []

    def worker(t):
        try:
            X0, X1, ref = jobs[t]
            eng = d.DenseInverseSearch(p, W, H, max_batch=B)
            # every torch operation of this thread on its own stream: no
            # device-wide synchronisation while the other thread may be
            # capturing (HIP fails an in-progress capture then; the library
            # would fall back to an eager call, the caller's op would fail)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                d0, d1 = torch.from_numpy(X0).cuda(), torch.from_numpy(X1).cuda()
                out = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
                for rep in range(12):
                    eng.set_graphs(rep % 3 != 2)  # replays and eager calls interleaved with the other thread's
                    out.fill_(float("nan"))
                    eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
                    host = out.to("cpu", non_blocking=False)
                    s.synchronize()
                    if not np.array_equal(host.numpy().view(np.uint32), ref.view(np.uint32)):
                        errors.append((t, rep))
            eng.close()
        except Exception as e:  # pragma: no cover - surfaced below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not any(x.is_alive() for x in th), "worker thread hung"
    assert not errors, errors


def test_medium_1080p_full_size_bitexact(disflow_mod, oracle):
    # BASELINE config 2 workload at full size against the oracle (a few seconds on CPU)
    W, H = 1920, 1080
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    I0, I1, gt = disflow_mod.synth_pair(0, W, H, with_gt=True)
    got = disflow_mod.DenseInverseSearch(p, W, H).calc(I0, I1)
    exp = oracle.calc_from_params(I0, I1, p)
    _assert_bitexact(got, exp, "1080p medium flow")
    epe = np.sqrt(((got - gt) ** 2).sum(-1))
    assert np.median(epe) < 1.5  # the engine tracks the synthetic motion


def test_invalid_calls_fail_loudly(disflow_mod):
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, 64, 64)
    eng = disflow_mod.DenseInverseSearch(p, 64, 64, max_batch=1)
    with pytest.raises(disflow_mod.DisError):
        eng.calc_batch(np.zeros((2, 64, 64), np.uint8), np.zeros((2, 64, 64), np.uint8))
    with pytest.raises(disflow_mod.DisError):
        eng.debug_dump(disflow_mod.STAGE_DENSE, 0)  # nothing computed yet


@pytest.mark.parametrize("preset", ["MEDIUM", "ULTRAFAST", "SLOW"])
def test_fast_and_generic_kernels_agree_with_oracle(disflow_mod, oracle, preset):
    # the patch-size-8 kernel (tile + DPP reductions) against the generic one and the oracle
    W, H = 480, 272
    p = disflow_mod.preset_params(disflow_mod.Preset[preset], W, H)
    if preset == "SLOW":
        p.iterations = 16  # keep the CPU oracle quick
    I0, I1 = disflow_mod.synth_pair(31, W, H)
    eng = disflow_mod.DenseInverseSearch(p, W, H)
    fast = eng.calc(I0, I1)
    eng.set_variant(1)
    generic = eng.calc(I0, I1)
    _assert_bitexact(fast, generic, "fast vs generic")
    _assert_bitexact(fast, oracle.calc_from_params(I0, I1, p), "fast vs oracle")


def test_uncorrelated_frames_exercise_tile_fallback(disflow_mod, oracle):
    # unrelated frames -> erratic coarse flow -> start positions spread wider
    # than the LDS tile in many blocks (global-read fallback path)
    W, H = 320, 256
    I0, _ = disflow_mod.synth_pair(40, W, H)
    _, I1 = disflow_mod.synth_pair(41, W, H)
    I1 = np.ascontiguousarray(I1[::-1, ::-1])
    p = disflow_mod.Params(coarsest_scale=5, finest_scale=0, patch_size=8, iterations=10,
                           patch_overlap=0.625, patch_normalization=1)
    exp = oracle.calc_from_params(I0, I1, p)
    eng = disflow_mod.DenseInverseSearch(p, W, H)
    # auto: these levels are small enough for 8 lanes per patch, whose kernel
    # reads spread blocks through L1/L2 inline; 2 lanes per patch everywhere
    # (variant 3): the tile kernel lists blocks too spread for its LDS tile
    # (none here: the densified initialisation is smooth) and k_search8_fb
    # searches them; variant 9 caps the usable tile so that most blocks go
    # through that list and kernel
    levels = range(p.finest_scale, p.coarsest_scale + 1)
    for variant in (0, 3, 9):
        eng.set_variant(variant)
        _assert_bitexact(eng.calc(I0, I1), exp, f"flow variant {variant}")
        listed = [eng.fallback_blocks(l) for l in levels]
        assert (sum(listed) > 0) == (variant == 9), listed  # DIS_STAGE_FALLBACK: the fallback kernel ran
    eng.set_variant(1)  # generic kernels: no tile / fallback split, the counters read 0
    eng.calc(I0, I1)
    assert all(eng.fallback_blocks(l) == 0 for l in levels)


def test_dense_grid_overlap_fallbacks(disflow_mod, oracle):
    # steps = 1 (overlap 0.9): the fused output kernel's patch staging does not
    # fit, so the densify + upsample kernels run instead; F = 1 and F = 0
    W, H = 96, 80
    I0, I1 = disflow_mod.synth_pair(50, W, H)
    for F in (1, 0):
        p = disflow_mod.Params(coarsest_scale=3, finest_scale=F, patch_size=8, iterations=4,
                               patch_overlap=0.9, patch_normalization=1)
        got = disflow_mod.DenseInverseSearch(p, W, H).calc(I0, I1)
        _assert_bitexact(got, oracle.calc_from_params(I0, I1, p), f"flow F={F}")


@pytest.mark.parametrize("name", sorted(f for f in __import__("os").listdir(helpers.GOLDEN) if f.endswith(".npz")))
def test_golden_fixtures_on_gpu(disflow_mod, name):
    import os
    z = np.load(os.path.join(helpers.GOLDEN, name))
    C, F, ps, it, norm = (int(v) for v in z["knobs_i"])
    H, W = z["I0"].shape
    p = _params(disflow_mod, C, F, ps, it, float(z["knobs_f"][0]), norm)
    got = disflow_mod.DenseInverseSearch(p, W, H).calc(z["I0"], z["I1"])
    _assert_bitexact(got, z["flow"], name)


@pytest.mark.parametrize("preset", ["MEDIUM", "ULTRAFAST", "SLOW"])
def test_lanes_per_patch_variants_bitexact(disflow_mod, oracle, preset):
    # k_search8<LPP> for LPP 2 (variant 3), 4 (variant 2), 8 (variant 4), 1 (variant 5),
    # k_search_wave (one wave per patch, variant 6) and the auto per-level choice
    # (variant 0) must all equal the oracle, on the LDS-tile path and on the
    # global-read fallback (unrelated frames)
    W, H = 352, 288
    p = disflow_mod.preset_params(disflow_mod.Preset[preset], W, H)
    if preset == "SLOW":
        p.iterations = 12
    I0, I1 = disflow_mod.synth_pair(77, W, H)
    J0, _ = disflow_mod.synth_pair(78, W, H)
    _, J1 = disflow_mod.synth_pair(79, W, H)
    J1 = np.ascontiguousarray(J1[::-1])
    exp = oracle.calc_from_params(I0, I1, p)
    exp_fb = oracle.calc_from_params(J0, J1, p)
    eng = disflow_mod.DenseInverseSearch(p, W, H)
    for variant, name in ((0, "auto"), (3, "LPP2"), (2, "LPP4"), (4, "LPP8"), (5, "LPP1"), (6, "LPP64")):
        eng.set_variant(variant)
        _assert_bitexact(eng.calc(I0, I1), exp, f"{name} vs oracle")
        _assert_bitexact(eng.calc(J0, J1), exp_fb, f"{name} fallback vs oracle")


SUBBATCH_CASES = [
    # (W, H, preset, batch, streams, fma): batches split into sub-batch streams
    # against single-pair oracle runs. In the exact mode no split changes a bit.
    # In the tolerance mode the 8- and 2-lanes-per-patch kernels sum in
    # different orders, and the runtime picks the layout per level from the
    # patches in a sub-batch (kLpp8MaxPatches), so a split can change rounding
    # where it moves a level across that threshold (the results stay within the
    # stated tolerance, tests/test_gpu_tolerance.py). The fma case below keeps
    # every level of 1080p MEDIUM on the same side of it at B = 4 vs 2 x 2, so
    # there the split must not change a bit either.
    (1920, 1080, "MEDIUM", 3, 1, 0),
    (1920, 1080, "MEDIUM", 4, 2, 1),
    (640, 480, "ULTRAFAST", 5, 2, 0),
    (320, 240, "MEDIUM", 2, 1, 0),     # every level at 8 lanes per patch
    (203, 151, "SLOW", 3, 3, 0),       # ragged, F = 0, three sub-batches of one pair
]


@pytest.mark.parametrize("W,H,preset,B,streams,fma", SUBBATCH_CASES)
def test_subbatch_streams_bitexact(disflow_mod, oracle, W, H, preset, B, streams, fma):
    p = disflow_mod.preset_params(disflow_mod.Preset[preset], W, H)
    if preset == "SLOW":
        p.iterations = 16
    pairs = [disflow_mod.synth_pair(900 + 7 * k + W, W, H) for k in range(B)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=B)
    eng.set_concurrency(streams)
    eng.set_precision(fma)
    got = eng.calc_batch(I0, I1)
    eng.set_concurrency(1)
    _assert_bitexact(got, eng.calc_batch(I0, I1), f"{streams} sub-batch streams vs one")
    if not fma:
        for k in range(B):
            _assert_bitexact(got[k], oracle.calc_from_params(I0[k], I1[k], p), f"pair {k} vs oracle")


def test_fallback_counter_follows_graph_replays(disflow_mod):
    # DIS_STAGE_FALLBACK sums the fallback lists of the sub-batches the last
    # call ran; a replayed graph runs the sub-batches it was captured with
    # (a replay of an n = 2 graph after an n = 1 capture used to
    # report one sub-batch's count)
    W, H = 320, 256
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    p.iterations = 4
    pairs = [disflow_mod.synth_pair(60 + k, W, H) for k in range(2)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    levels = range(p.finest_scale, p.coarsest_scale + 1)
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=2)
    eng.set_concurrency(2)
    eng.set_variant(9)  # most blocks through the fallback lists
    eng.set_graphs(False)
    ref = {}
    for n in (2, 1):
        eng.calc_batch(I0[:n], I1[:n])
        ref[n] = [eng.fallback_blocks(l) for l in levels]
    assert sum(ref[2]) > sum(ref[1]) > 0, ref
    eng.set_graphs(True)
    for n in (2, 1, 2, 1, 2):
        eng.calc_batch(I0[:n], I1[:n])
        assert [eng.fallback_blocks(l) for l in levels] == ref[n], (n, ref)


@pytest.mark.gpu
def test_pyramid_sqrt_is_correctly_rounded_on_every_input():
    # k_pyramid takes the Sobel magnitude as sqrt_cr(N) / 8 (N = 64 * (gx^2 + gy^2),
    # an integer < 2^21 for u8 input); tools/sqrt_check compares it with the
    # correctly rounded sqrtf for every possible N on this GPU
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "sqrt_check")
    assert os.path.exists(exe), "tools/sqrt_check not built (__graft_entry__.build)"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "sqrt_cr: 0 mismatches" in out.stdout, out.stdout + out.stderr


@pytest.mark.gpu
def test_colour_fast_division_and_sqrt_are_ieee():
    # dis_color.hip's fast cores (dis_device.h div_core / sqrt_core) and the
    # paper mode's reciprocal (recip_core) rest on this GPU's v_rcp_f32 /
    # v_sqrt_f32 seeds: tools/color_core_check compares them with IEEE a / b,
    # sqrtf and 1.0f / m on every divisor mantissa, whole binades of the sqrt
    # domain and every float of the reciprocal's domain
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "color_core_check")
    assert os.path.exists(exe), "tools/color_core_check not built (__graft_entry__.build)"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.count("mismatches 0") == 9, out.stdout + out.stderr


def test_medium_4k_batch_bitexact(disflow_mod, oracle):
    # BASELINE config 3 (3840x2160 MEDIUM, the LDS/HBM tiling stress case):
    # a batch of 2 (2-lanes-per-patch kernels on the big levels, 2 streams),
    # both pairs against the oracle
    W, H = 3840, 2160
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    pairs = [disflow_mod.synth_pair(900 + k, W, H) for k in range(2)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    got = disflow_mod.DenseInverseSearch(p, W, H, max_batch=2).calc_batch(I0, I1)
    for k in range(2):
        _assert_bitexact(got[k], oracle.calc_from_params(I0[k], I1[k], p), f"4k pair {k}")


def test_bench_batch_matches_single_pair_calls(disflow_mod):
    # the bench configuration (32 x 1080p MEDIUM per call, 2 sub-batch streams,
    # per-level lane layouts chosen by batch size) gives every pair exactly the
    # flow of a one-pair call (different lane layouts on some levels)
    W, H, B = 1920, 1080, 32
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    pairs = [disflow_mod.synth_pair(k, W, H) for k in range(B)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    batch = disflow_mod.DenseInverseSearch(p, W, H, max_batch=B).calc_batch(I0, I1)
    one = disflow_mod.DenseInverseSearch(p, W, H, max_batch=1)
    for k in (0, 7, 16, 31):
        _assert_bitexact(batch[k], one.calc(I0[k], I1[k]), f"pair {k}")


@pytest.mark.parametrize("maxmotion", [-1.0, 3.0])
def test_flow_color_kernel_bitexact(disflow_mod, oracle, maxmotion):
    # dis_flow_color (k_color_maxrad + k_color_pixels) vs the C oracle, byte
    # for byte: special values, a batch of fields, and an engine flow
    rng = np.random.default_rng(9)
    f = (rng.standard_normal((3, 61, 77, 2)) * 5).astype(np.float32)
    f[0, 0, :6] = [(np.nan, 1), (1, np.inf), (2e9, 0), (0, 0), (-0.0, 0.0), (1e-30, -1e-30)]
    W, H = 320, 240
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    I0, I1 = disflow_mod.synth_pair(3, W, H)
    flow = disflow_mod.DenseInverseSearch(p, W, H).calc(I0, I1)
    got = disflow_mod.flow_color(f, maxmotion)
    for k in range(3):
        assert np.array_equal(got[k], oracle.flow_color(f[k], maxmotion)), f"field {k}"
    assert np.array_equal(disflow_mod.flow_color(flow, maxmotion), oracle.flow_color(flow, maxmotion))


@pytest.mark.parametrize("maxmotion", [-1.0, 2.5, 1e-30, 1e30])
def test_flow_color_batch_persistent_bitexact(disflow_mod, oracle, maxmotion):
    # the one-launch colour kernel (k_color: max-pass and colour work items
    # claimed in order, colour items of field f waiting for f's max): a batch
    # of 5 fields (W*H % 4 == 0: float4 loads, dwordx3 stores), ragged values
    # per field, and maxmotion outside div_pre's domain (IEEE division path)
    rng = np.random.default_rng(11)
    f = (rng.standard_normal((5, 96, 128, 2)) * np.array([0.5, 3, 20, 1e-3, 60])[:, None, None, None]).astype(np.float32)
    f[1, 3, :4] = [(np.nan, 0), (1e9, 1), (-0.0, -0.0), (1e-40, 3e-39)]
    f[4, :, :] = 0.0  # a field with maxrad 0 -> max(1, 0)
    got = disflow_mod.flow_color(f, maxmotion)
    for k in range(5):
        assert np.array_equal(got[k], oracle.flow_color(f[k], maxmotion)), f"field {k}"


def test_flow_color_chunked_fast_paths_bitexact(disflow_mod, oracle):
    # 9 full-HD fields = two 128 MB chunks (8 + 1): the colour pass of chunk 0 shares
    # a launch with the max pass of chunk 1 (k_color_step). Values at the
    # edges of the fast division / sqrt domains (dis_color.hip div_rn,
    # sqrt_rn): axis-aligned flows (min/max quotient 0), quotients around
    # 2^-30, squared radii around 2^-96 and 2^96 (fixed range), denormals --
    # each either on the exact fast path or recomputed the IEEE way
    W, H, n = 1920, 1080, 9
    rng = np.random.default_rng(21)
    scales = np.array([4, 0.3, 40, 1e-3, 7, 1e-20, 2, 5, 1e6], np.float32)
    f = (rng.standard_normal((n, H, W, 2)) * scales[:, None, None, None]).astype(np.float32)
    e = np.array([(1.0, 0.0), (0.0, -2.0), (1.0, 2.0 ** -30), (1.0, 2.0 ** -31), (3.0, 2.0 ** -29.5),
                  (2.0 ** -48, 2.0 ** -49), (2.0 ** -49, 0.0), (2.0 ** -60, 2.0 ** -61), (1e-38, 1e-39),
                  (2.0 ** 47, 2.0 ** 46), (-0.0, 5.0), (5.0, -0.0)], np.float32)
    for k in range(n):
        f[k, 7, 100:100 + len(e)] = e * (k + 1)
    got = disflow_mod.flow_color(f, -1.0)
    for k in range(n):
        assert np.array_equal(got[k], oracle.flow_color(f[k], -1.0)), f"field {k}"
    small = f[:2, :64, :64].copy()
    for mm in (2.0 ** -50, 2.0 ** 50):  # fixed ranges putting fx*fx + fy*fy outside [2^-96, 2^96]
        g = disflow_mod.flow_color(small, mm)
        for k in range(2):
            assert np.array_equal(g[k], oracle.flow_color(small[k], mm)), f"maxmotion {mm} field {k}"


def test_flow_color_unaligned_output_bitexact(disflow_mod, oracle):
    # a BGR pointer that is not 4-byte aligned takes the per-pixel store path
    import torch
    rng = np.random.default_rng(12)
    f = (rng.standard_normal((3, 40, 64, 2)) * 4).astype(np.float32)
    d = torch.from_numpy(f).cuda()
    raw = torch.zeros(3 * 40 * 64 * 3 + 1, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    disflow_mod._check(disflow_mod.lib().dis_flow_color(d.data_ptr(), 3, 64, 40, -1.0, raw.data_ptr() + 1,
                                                        disflow_mod.MEM_DEVICE, s.cuda_stream, 0))
    s.synchronize()
    o = raw.cpu().numpy()[1:].reshape(3, 40, 64, 3)
    for k in range(3):
        assert np.array_equal(o[k], oracle.flow_color(f[k]))


def test_flow_color_device_pointers(disflow_mod, oracle):
    import torch
    rng = np.random.default_rng(10)
    f = (rng.standard_normal((2, 50, 40, 2)) * 3).astype(np.float32)
    d = torch.from_numpy(f).cuda()
    out = torch.empty((2, 50, 40, 3), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    disflow_mod._check(disflow_mod.lib().dis_flow_color(d.data_ptr(), 2, 40, 50, -1.0, out.data_ptr(),
                                                        disflow_mod.MEM_DEVICE, s.cuda_stream, 0))
    s.synchronize()
    o = out.cpu().numpy()
    for k in range(2):
        assert np.array_equal(o[k], oracle.flow_color(f[k]))


@pytest.mark.parametrize("variant", [0, 1, 6])
def test_var_refine_path_bitexact(disflow_mod, oracle, variant):
    # variational refinement on every level (fast search with dense-flow init,
    # k_vr_* kernels) vs the oracle's restatement, a batch of 3 on 2 streams;
    # variant 1 = the generic kernels, 6 = one wave per patch
    W, H = 320, 240
    p = disflow_mod.Params(coarsest_scale=4, finest_scale=1, patch_size=8, iterations=10, patch_overlap=0.625,
                           patch_normalization=1, var_refine_iters=3)
    pairs = [disflow_mod.synth_pair(60 + k, W, H) for k in range(3)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=3)
    eng.set_variant(variant)
    got = eng.calc_batch(I0, I1)
    for k in range(3):
        _assert_bitexact(got[k], oracle.calc_from_params(I0[k], I1[k], p), f"pair {k}")


def test_slow_preset_with_refinement_bitexact(disflow_mod, oracle):
    # BASELINE config 5 semantics (SLOW: F = 0, steps 2, refinement on) at a
    # small size with fewer search iterations
    W, H = 192, 144
    p = disflow_mod.preset_params(disflow_mod.Preset.SLOW, W, H)
    assert p.var_refine_iters > 0 and p.finest_scale == 0
    p.iterations = 8
    I0, I1 = disflow_mod.synth_pair(70, W, H)
    got = disflow_mod.DenseInverseSearch(p, W, H).calc(I0, I1)
    _assert_bitexact(got, oracle.calc_from_params(I0, I1, p), "slow + refinement")


# --- paper mode (template-subtracted residual, residual-weighted
# densification). Not in the reference: HIP vs the oracle's restatement, bit-exact.

PAPER_CASES = [
    # (W, H, preset or knobs, variants)
    (352, 288, "MEDIUM"),
    (640, 480, "ULTRAFAST"),
    (203, 151, (3, 0, 8, 10, 0.7, 1)),    # ragged, F = 0
    (96, 64, (2, 1, 6, 5, 0.5, 0)),       # generic kernel (ps 6), no normalisation
    (128, 96, (3, 0, 4, 6, 0.5, 1)),      # generic kernel (ps 4)
]


@pytest.mark.parametrize("W,H,cfg", PAPER_CASES)
def test_paper_mode_bitexact(disflow_mod, oracle, W, H, cfg):
    if isinstance(cfg, str):
        p = disflow_mod.preset_params(disflow_mod.Preset[cfg], W, H)
    else:
        p = _params(disflow_mod, *cfg)
    p.paper_mode = 1
    I0, I1 = disflow_mod.synth_pair(W + 3 * H, W, H)
    J0, _ = disflow_mod.synth_pair(W + 3 * H + 1, W, H)
    exp = oracle.calc_from_params(I0, I1, p)
    exp_fb = oracle.calc_from_params(J0, I1, p)  # unrelated frames: tile fallback blocks
    eng = disflow_mod.DenseInverseSearch(p, W, H)
    variants = ((0, "auto"), (1, "generic"), (3, "LPP2"), (2, "LPP4"), (4, "LPP8"), (5, "LPP1"),
                (9, "LPP2, most blocks through the fallback list")) if p.patch_size == 8 else ((0, "auto"),)
    for variant, name in variants:
        eng.set_variant(variant)
        _assert_bitexact(eng.calc(I0, I1), exp, f"paper {name}")
        if variant == 9:  # the paper-mode fallback kernel (k_search8_fb<2, kPaper>) ran
            assert sum(eng.fallback_blocks(l) for l in range(p.finest_scale, p.coarsest_scale + 1)) > 0
        _assert_bitexact(eng.calc(J0, I1), exp_fb, f"paper {name} fallback")


def test_paper_mode_batch_streams_and_refinement(disflow_mod, oracle):
    # a batch of 3 on 2 sub-batch streams, with and without refinement on top
    W, H = 320, 240
    pairs = [disflow_mod.synth_pair(90 + k, W, H) for k in range(3)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    for vr in (0, 2):
        p = disflow_mod.Params(coarsest_scale=4, finest_scale=1, patch_size=8, iterations=10,
                               patch_overlap=0.625, patch_normalization=1, var_refine_iters=vr, paper_mode=1)
        eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=3)
        eng.set_concurrency(2)
        got = eng.calc_batch(I0, I1)
        for k in range(3):
            _assert_bitexact(got[k], oracle.calc_from_params(I0[k], I1[k], p), f"paper vr={vr} pair {k}")


def test_paper_mode_identical_frames_zero_flow_on_gpu(disflow_mod):
    W, H = 160, 120
    I0, _ = disflow_mod.synth_pair(5, W, H)
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    p.paper_mode = 1
    got = disflow_mod.DenseInverseSearch(p, W, H).calc(I0, I0)
    assert np.array_equal(got, np.zeros_like(got))


@pytest.mark.parametrize("seed,W,H,preset,paper", [
    (3, 1920, 1080, "MEDIUM", 0),
    (4, 1920, 1080, "FAST", 0),
    (5, 1920, 1080, "ULTRAFAST", 0),
    (6, 1920, 1080, "MEDIUM", 1),
    (7, 3840, 2160, "MEDIUM", 0),
])
def test_structured_scenes_bitexact(disflow_mod, oracle, seed, W, H, preset, paper):
    # tests/scenes.py: flat regions (zero gradients), sharp edges, objects moving
    # independently by up to 20 px (occlusions, outlier resets, spread blocks),
    # a border-crossing and a saturated object, sensor noise -- the statistics
    # of real footage the value-noise pairs lack; a batch of two scenes, full size
    import scenes
    pairs = [scenes.scene_pair(seed * 10 + k, W, H) for k in range(2)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    p = disflow_mod.preset_params(disflow_mod.Preset[preset], W, H)
    p.paper_mode = paper
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=2)
    got = eng.calc_batch(I0, I1)
    if seed == 3:  # the scenes send spread blocks to the fallback kernel (the unrelated-frames test aside, only here)
        assert sum(eng.fallback_blocks(l) for l in range(p.finest_scale, p.coarsest_scale + 1)) > 0
    with oracle.threads(16):
        for k in range(2):
            _assert_bitexact(got[k], oracle.calc_from_params(I0[k], I1[k], p), f"scene {seed}/{k} {preset} paper {paper}")


@pytest.mark.parametrize("fma", [0, 1])
def test_fallback_kernel_full_size(disflow_mod, oracle, fma):
    # variant 9 (usable LDS tile capped at 24 rows / columns): most blocks of
    # every level of a 1080p MEDIUM batch take the fallback list and
    # k_search8_fb's global-read path, in both sub-batch streams -- bit-exact
    # against the oracle and the default kernels (exact), and against the
    # tile kernel at 2 lanes per patch everywhere (variant 3; tolerance mode,
    # whose 8-lane coarse-level kernels sum in another order)
    W, H = 1920, 1080
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, W, H)
    pairs = [disflow_mod.synth_pair(700 + k, W, H) for k in range(2)]
    I0 = np.stack([a for a, _ in pairs])
    I1 = np.stack([b for _, b in pairs])
    eng = disflow_mod.DenseInverseSearch(p, W, H, max_batch=2)
    eng.set_precision(fma)
    eng.set_variant(3 if fma else 0)
    ref = eng.calc_batch(I0, I1)
    eng.set_variant(9)
    got = eng.calc_batch(I0, I1)
    listed = sum(eng.fallback_blocks(l) for l in range(p.finest_scale, p.coarsest_scale + 1))
    nblocks = 2 * sum(((W >> l) // 3 // 8 + 1) * ((H >> l) // 3 // 8 + 1) for l in range(p.finest_scale, 4))
    assert listed > nblocks // 4, (listed, nblocks)
    for k in range(2):
        _assert_bitexact(got[k], ref[k], f"variant 9 vs {3 if fma else 0}, pair {k}, fma {fma}")
        if not fma:
            with oracle.threads(16):
                _assert_bitexact(got[k], oracle.calc_from_params(I0[k], I1[k], p), f"variant 9 pair {k}")
