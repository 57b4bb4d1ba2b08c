"""ctypes binding of the CPU oracle (oracle/libdis_oracle.so) -- tests only.

The oracle is test infrastructure (see oracle/dis_oracle.h): it is the checker
the HIP path is compared against, never a product fallback.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# DIS_ORACLE_LIB selects another build of the same source (bench.py's CPU
# baseline uses the -O3 build libdis_oracle_o3.so)
LIB = os.environ.get("DIS_ORACLE_LIB") or os.path.join(ORACLE_DIR, "libdis_oracle.so")


class Params(ctypes.Structure):
    _fields_ = [
        ("coarsest_scale", ctypes.c_int),
        ("finest_scale", ctypes.c_int),
        ("patch_size", ctypes.c_int),
        ("iterations", ctypes.c_int),
        ("patch_overlap", ctypes.c_float),
        ("patch_normalization", ctypes.c_int),
        ("var_refine_iters", ctypes.c_int),
        ("paper_mode", ctypes.c_int),
    ]


def _load():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(os.path.join(ORACLE_DIR, "dis_oracle.c")):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "all", "o3"])
    L = ctypes.CDLL(LIB)
    I, F, V, Z = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
    P = ctypes.POINTER
    L.dis_oracle_steps.argtypes = [I, F]
    L.dis_oracle_steps.restype = I
    L.dis_oracle_set_threads.argtypes = [I]
    L.dis_oracle_set_threads.restype = I
    L.dis_oracle_grid.argtypes = [I, I, I, P(I), P(I), P(I), P(I)]
    L.dis_oracle_padded_size.argtypes = [I, I, I, P(I), P(I), P(I), P(I)]
    L.dis_oracle_pad_convert.argtypes = [V, Z, I, I, I, V]
    L.dis_oracle_pyramid.argtypes = [V, I, I, I, V, V, V]
    L.dis_oracle_sobel.argtypes = [V, I, I, V, V]
    L.dis_oracle_flow_color.argtypes = [V, I, I, F, V]
    L.dis_oracle_var_refine.argtypes = [V, V, I, I, I, V, I]
    L.dis_oracle_var_energy.argtypes = [V, V, I, I, I, V]
    L.dis_oracle_var_energy.restype = ctypes.c_double
    L.dis_oracle_flow_from_pyramids.argtypes = [P(V)] * 4 + [I, V, I, I, I, I, I, I, F, I, V, V]
    L.dis_oracle_flow_from_pyramids.restype = I
    L.dis_oracle_flow_from_pyramids_ex.argtypes = [P(V)] * 4 + [I, V, I, I, I, I, I, I, F, I, I, I, V, V]
    L.dis_oracle_flow_from_pyramids_ex.restype = I
    L.dis_oracle_upsample_crop.argtypes = [V, I, I, I, I, I, I, I, V]
    L.dis_oracle_calc_u8.argtypes = [P(Params), I, I, V, V, Z, V]
    L.dis_oracle_calc_u8.restype = I
    return L


lib = _load()


def _p(a):
    return a.ctypes.data if a is not None else None


def set_threads(n):
    """Threads for the oracle's per-level patch loop (OpenMP); results are
    identical for every count (the patches are independent). Returns the count."""
    return lib.dis_oracle_set_threads(int(n))


class threads:
    """Context manager: run the oracle with n patch-loop threads, then back to 1."""

    def __init__(self, n=None):
        self.n = n if n is not None else min(16, os.cpu_count() or 1)

    def __enter__(self):
        return set_threads(self.n)

    def __exit__(self, *exc):
        set_threads(1)


def steps(ps, overlap):
    return lib.dis_oracle_steps(ps, overlap)


def grid(W, H, st):
    a = [ctypes.c_int() for _ in range(4)]
    lib.dis_oracle_grid(W, H, st, *[ctypes.byref(x) for x in a])
    return tuple(x.value for x in a)  # npw, nph, offw, offh


def padded_size(W, H, C):
    a = [ctypes.c_int() for _ in range(4)]
    lib.dis_oracle_padded_size(W, H, C, *[ctypes.byref(x) for x in a])
    return tuple(x.value for x in a)  # Wp, Hp, pad_left, pad_top


def pad_convert(img_u8, C):
    H, W = img_u8.shape
    Wp, Hp, _, _ = padded_size(W, H, C)
    out = np.empty((Hp, Wp), np.float32)
    a = np.ascontiguousarray(img_u8)
    lib.dis_oracle_pad_convert(_p(a), W, W, H, C, _p(out))
    return out


def level_sizes(Wp, Hp, C):
    return [(Wp >> l, Hp >> l) for l in range(C + 1)]


def pyramid(img, C, want_grad=True):
    """-> list of (img_l, dx_l, dy_l) unpadded planes, levels 0..C."""
    Hp, Wp = img.shape
    sizes = level_sizes(Wp, Hp, C)
    tot = sum(w * h for w, h in sizes)
    lv = np.empty(tot, np.float32)
    dx = np.empty(tot, np.float32) if want_grad else None
    dy = np.empty(tot, np.float32) if want_grad else None
    lib.dis_oracle_pyramid(_p(np.ascontiguousarray(img, dtype=np.float32)), Wp, Hp, C, _p(lv), _p(dx), _p(dy))
    out, off = [], 0
    for w, h in sizes:
        sl = slice(off, off + w * h)
        out.append((lv[sl].reshape(h, w), dx[sl].reshape(h, w) if want_grad else None,
                    dy[sl].reshape(h, w) if want_grad else None))
        off += w * h
    return out


def sobel(img):
    H, W = img.shape
    dx = np.empty((H, W), np.float32)
    dy = np.empty((H, W), np.float32)
    lib.dis_oracle_sobel(_p(np.ascontiguousarray(img, dtype=np.float32)), W, H, _p(dx), _p(dy))
    return dx, dy


def pad_planes(planes, pad, mode):
    """copyMakeBorder (src/main.cpp:43-47): 'edge' for images, zeros for gradients."""
    return [np.ascontiguousarray(np.pad(p, pad, mode=mode), dtype=np.float32) for p in planes]


def flow_from_pyramids(P0, PX, PY, P1, pad, W, H, C, F, it, ps, overlap, norm, capture=False, vr=0, paper=0):
    nl = C + 1

    def arr(lst):
        return (ctypes.c_void_p * nl)(*[p.ctypes.data for p in lst])

    out = np.empty(((H >> F), (W >> F), 2), np.float32)
    st = steps(ps, overlap)
    dbg_u = dbg_d = None
    if capture:
        nu = sum(grid(W >> l, H >> l, st)[0] * grid(W >> l, H >> l, st)[1] for l in range(nl))
        nd = sum((W >> l) * (H >> l) for l in range(nl))
        dbg_u = np.full(2 * nu, np.nan, np.float32)
        dbg_d = np.full(2 * nd, np.nan, np.float32)
    rc = lib.dis_oracle_flow_from_pyramids_ex(
        ctypes.cast(arr(P0), ctypes.POINTER(ctypes.c_void_p)),
        ctypes.cast(arr(PX), ctypes.POINTER(ctypes.c_void_p)),
        ctypes.cast(arr(PY), ctypes.POINTER(ctypes.c_void_p)),
        ctypes.cast(arr(P1), ctypes.POINTER(ctypes.c_void_p)),
        pad, _p(out), W, H, C, F, it, ps, overlap, int(norm), int(vr), int(paper), _p(dbg_u), _p(dbg_d))
    assert rc == 0
    if not capture:
        return out
    us, ds, ou, od = {}, {}, 0, 0
    for l in range(nl):
        w, h = W >> l, H >> l
        npw, nph, _, _ = grid(w, h, st)
        if l >= F:
            us[l] = dbg_u[ou:ou + 2 * npw * nph].reshape(-1, 2).copy()
            ds[l] = dbg_d[od:od + 2 * w * h].reshape(h, w, 2).copy()
        ou += 2 * npw * nph
        od += 2 * w * h
    return out, us, ds


def upsample_crop(flowF, Wp, Hp, F, pl, pt, W, H):
    out = np.empty((H, W, 2), np.float32)
    lib.dis_oracle_upsample_crop(_p(np.ascontiguousarray(flowF, dtype=np.float32)), Wp, Hp, F, pl, pt, W, H, _p(out))
    return out


def calc_u8(I0, I1, C, F, ps, it, overlap, norm=1, vr=0, paper=0):
    H, W = I0.shape
    p = Params(C, F, ps, it, overlap, norm, vr, paper)
    out = np.empty((H, W, 2), np.float32)
    a0 = np.ascontiguousarray(I0, dtype=np.uint8)
    a1 = np.ascontiguousarray(I1, dtype=np.uint8)
    rc = lib.dis_oracle_calc_u8(ctypes.byref(p), W, H, _p(a0), _p(a1), W, _p(out))
    assert rc == 0
    return out


def calc_from_params(I0, I1, params):
    """params: disflow.Params (or anything with the same attributes)."""
    return calc_u8(I0, I1, params.coarsest_scale, params.finest_scale, params.patch_size,
                   params.iterations, params.patch_overlap, params.patch_normalization,
                   getattr(params, "var_refine_iters", 0), getattr(params, "paper_mode", 0))


def build_pyramids(I0, I1, C, ps):
    """The reference's main.cpp front end on top of the oracle: u8 frames ->
    padded pyramids exactly as passed to OpticalFlowClass (src/main.cpp:139-189)."""
    f0 = pad_convert(I0, C)
    f1 = pad_convert(I1, C)
    py0 = pyramid(f0, C)
    py1 = pyramid(f1, C)
    P0 = pad_planes([p[0] for p in py0], ps, "edge")
    PX = pad_planes([p[1] for p in py0], ps, "constant")
    PY = pad_planes([p[2] for p in py0], ps, "constant")
    P1 = pad_planes([p[0] for p in py1], ps, "edge")
    return f0.shape[1], f0.shape[0], P0, PX, PY, P1, py0, py1


def flow_color(flow, maxmotion=-1.0):
    """Middlebury colour coding of one (H, W, 2) field -> (H, W, 3) u8 BGR."""
    f = np.ascontiguousarray(flow, dtype=np.float32)
    H, W = f.shape[:2]
    out = np.empty((H, W, 3), np.uint8)
    lib.dis_oracle_flow_color(f.ctypes.data, W, H, float(maxmotion), out.ctypes.data)
    return out


def var_refine(I0, I1, flow, fp):
    """Variational refinement of a (H, W, 2) flow between float level images."""
    a0 = np.ascontiguousarray(I0, dtype=np.float32)
    a1 = np.ascontiguousarray(I1, dtype=np.float32)
    f = np.array(flow, dtype=np.float32, copy=True, order="C")
    H, W = a0.shape
    lib.dis_oracle_var_refine(_p(a0), _p(a1), W, W, H, _p(f), int(fp))
    return f


def var_energy(I0, I1, flow):
    a0 = np.ascontiguousarray(I0, dtype=np.float32)
    a1 = np.ascontiguousarray(I1, dtype=np.float32)
    f = np.ascontiguousarray(flow, dtype=np.float32)
    H, W = a0.shape
    return lib.dis_oracle_var_energy(_p(a0), _p(a1), W, W, H, _p(f))
