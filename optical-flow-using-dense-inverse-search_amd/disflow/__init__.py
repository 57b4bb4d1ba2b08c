"""disflow -- Python host mirror of the DIS engine's C-ABI (include/dis_abi.h).

The product is the HIP library ``libdis_hip.so`` next to this file; this module
only binds it with ctypes (plain pointers and sizes) so tests and the bench can
drive it. The interface mirrors the reference's entry points:

* :class:`DenseInverseSearch` ``.calc(I0, I1)`` -- u8 frames to full-resolution
  flow (the reference's per-pair body, src/main.cpp:135-198);
* :func:`optical_flow_from_pyramids` -- the ``OpticalFlow::OpticalFlowClass``
  constructor (include/optical_flow.hpp:43-54) over caller-built padded
  pyramids, returning the finest-level flow;
* :class:`Preset` -- build-defined presets.

There is no CPU fallback: every compute call goes to the HIP library and fails
loudly (:class:`DisError`) when it or a device is missing.
"""
from __future__ import annotations

import ctypes
import enum
import os
from dataclasses import dataclass

import numpy as np

# torch (if present) must own the process's HIP runtime before libdis_hip.so is
# loaded, so both bind the same libamdhip64 (it is plumbing: device buffers and
# streams for bench.py; never on the compute path of this module).
try:  # pragma: no cover - import side effect only
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DISFLOW_LIB") or os.path.join(_HERE, "libdis_hip.so")

DIS_OK = 0
DIS_ERR_INVALID_ARGUMENT = -1
DIS_ERR_UNSUPPORTED = -2
DIS_ERR_DEVICE = -3
DIS_ERR_OUT_OF_MEMORY = -4
DIS_ERR_INTERNAL = -5

MEM_HOST = 0
MEM_DEVICE = 1

STAGE_IMG0, STAGE_IMG1, STAGE_DX0, STAGE_DY0, STAGE_PATCH_U, STAGE_DENSE, STAGE_FALLBACK = range(7)

PRECISION_EXACT, PRECISION_FMA = 0, 1

KERNEL_PYRAMID, KERNEL_SEARCH, KERNEL_SEARCH_FINEST, KERNEL_DENSIFY, KERNEL_VR_LIN, KERNEL_VR_SOR = range(6)

# Every symbol include/dis_abi.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "dis_abi_version", "dis_last_error", "dis_preset_params", "dis_validate_params",
    "dis_workload_info", "dis_create", "dis_destroy", "dis_calc_u8", "dis_calc_batch_u8",
    "dis_flow_from_pyramids", "dis_set_debug", "dis_stage_size", "dis_debug_dump",
    "dis_set_kernel_timing", "dis_kernel_time", "dis_synth_pair", "dis_set_kernel_variant",
    "dis_set_concurrency", "dis_set_precision", "dis_set_graphs", "dis_flow_color", "dis_flo_info",
    "dis_read_flo", "dis_write_flo", "dis_build_kind", "dis_set_host_pipeline", "dis_host_pipeline_info",
    "dis_host_alloc", "dis_host_free", "dis_batch_stream_plan", "dis_check_stream_plan",
)


class Preset(enum.IntEnum):
    ULTRAFAST = 0
    FAST = 1
    MEDIUM = 2
    SLOW = 3
    REFERENCE = 4


class DisError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"dis status {status}: {msg}")
        self.status = status


class _Params(ctypes.Structure):
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


class _HostInfo(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int) for k in ("chunk_pairs", "last_chunks", "last_direct_in", "last_direct_out")]


class _Workload(ctypes.Structure):
    _fields_ = [
        ("padded_width", ctypes.c_int),
        ("padded_height", ctypes.c_int),
        ("steps", ctypes.c_int),
        ("patches", ctypes.c_longlong),
        ("updates", ctypes.c_longlong),
        ("algorithmic_bytes", ctypes.c_double),
        ("search_bytes_finest", ctypes.c_double),
        ("search_bytes_all", ctypes.c_double),
        ("search_launches", ctypes.c_int),
        ("patches_finest", ctypes.c_longlong),
        ("search_flops_finest", ctypes.c_double),
    ]


@dataclass
class Params:
    coarsest_scale: int
    finest_scale: int
    patch_size: int = 8
    iterations: int = 25
    patch_overlap: float = 0.625
    patch_normalization: int = 1
    var_refine_iters: int = 0
    paper_mode: int = 0

    def _c(self) -> _Params:
        return _Params(self.coarsest_scale, self.finest_scale, self.patch_size, self.iterations,
                       self.patch_overlap, int(self.patch_normalization), self.var_refine_iters,
                       int(self.paper_mode))

    @staticmethod
    def _from_c(p: _Params) -> "Params":
        return Params(p.coarsest_scale, p.finest_scale, p.patch_size, p.iterations,
                      float(p.patch_overlap), p.patch_normalization, p.var_refine_iters, p.paper_mode)


_lib = None


def lib() -> ctypes.CDLL:
    """Load libdis_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DisError(DIS_ERR_INTERNAL, f"{LIB_PATH} missing: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        P, I, F, D, Z, V = ctypes.POINTER, ctypes.c_int, ctypes.c_float, ctypes.c_double, ctypes.c_size_t, ctypes.c_void_p
        L.dis_abi_version.restype = I
        L.dis_last_error.restype = ctypes.c_char_p
        L.dis_preset_params.argtypes = [I, I, I, P(_Params)]
        L.dis_validate_params.argtypes = [P(_Params), I, I]
        L.dis_workload_info.argtypes = [P(_Params), I, I, P(_Workload)]
        L.dis_create.argtypes = [P(V), P(_Params), I, I, I, I]
        L.dis_destroy.argtypes = [V]
        L.dis_calc_u8.argtypes = [V, V, V, Z, V, I, V]
        L.dis_calc_batch_u8.argtypes = [V, I, V, V, Z, Z, V, I, V]
        L.dis_flow_from_pyramids.argtypes = [P(V)] * 6 + [I, V, I, I, I, I, I, I, F, I, I]
        L.dis_set_debug.argtypes = [V, I]
        L.dis_set_kernel_variant.argtypes = [V, I]
        L.dis_set_concurrency.argtypes = [V, I]
        if L.dis_abi_version() >= 4:  # (older builds load for A/B timing only)
            L.dis_set_precision.argtypes = [V, I]
            L.dis_set_graphs.argtypes = [V, I]
        if L.dis_abi_version() >= 6:
            L.dis_build_kind.restype = ctypes.c_char_p
        if L.dis_abi_version() >= 8:
            L.dis_set_host_pipeline.argtypes = [V, I]
            L.dis_host_pipeline_info.argtypes = [V, P(_HostInfo)]
            L.dis_host_alloc.argtypes = [Z, P(V)]
            L.dis_host_free.argtypes = [V]
            L.dis_batch_stream_plan.argtypes = [I, I, P(I), I, P(I)]
            L.dis_check_stream_plan.argtypes = [P(I), I, I, I]
        L.dis_stage_size.argtypes = [V, I, I, P(Z)]
        L.dis_debug_dump.argtypes = [V, I, I, I, V, Z]
        L.dis_set_kernel_timing.argtypes = [V, I]
        L.dis_kernel_time.argtypes = [V, I, P(I), P(D)]
        L.dis_synth_pair.argtypes = [ctypes.c_uint64, I, I, V, V, V]
        L.dis_flow_color.argtypes = [V, I, I, I, ctypes.c_float, V, I, V, I]
        L.dis_flo_info.argtypes = [ctypes.c_char_p, P(I), P(I)]
        L.dis_read_flo.argtypes = [ctypes.c_char_p, V, I, I, I]
        L.dis_write_flo.argtypes = [ctypes.c_char_p, V, I, I, I]
        for name in EXPORTED_SYMBOLS:
            if name not in ("dis_abi_version", "dis_last_error", "dis_build_kind") and hasattr(L, name):
                getattr(L, name).restype = I
        _lib = L
    return _lib


def build_kind() -> str:
    """"product" (the sources carry no compile-time variants since ABI v7)."""
    return lib().dis_build_kind().decode()


def _check(st: int) -> None:
    if st != DIS_OK:
        raise DisError(st, lib().dis_last_error().decode())


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def preset_params(preset: Preset, width: int, height: int) -> Params:
    p = _Params()
    _check(lib().dis_preset_params(int(preset), width, height, ctypes.byref(p)))
    return Params._from_c(p)


def validate(params: Params, width: int, height: int) -> int:
    return lib().dis_validate_params(ctypes.byref(params._c()), width, height)


def workload(params: Params, width: int, height: int) -> dict:
    w = _Workload()
    _check(lib().dis_workload_info(ctypes.byref(params._c()), width, height, ctypes.byref(w)))
    return {k: getattr(w, k) for k, _ in _Workload._fields_}


def flow_color(flow: np.ndarray, maxmotion: float = -1.0, device: int = 0) -> np.ndarray:
    """Middlebury colour coding (src/color_coding.cpp draw_optical_flow) of an
    (H, W, 2) or (n, H, W, 2) float field on the GPU -> u8 BGR (..., 3)."""
    f = np.ascontiguousarray(flow, dtype=np.float32)
    single = f.ndim == 3
    if single:
        f = f[None]
    if f.ndim != 4 or f.shape[-1] != 2:
        raise DisError(DIS_ERR_INVALID_ARGUMENT, "flow must be (H, W, 2) or (n, H, W, 2)")
    n, H, W = f.shape[:3]
    out = np.empty((n, H, W, 3), np.uint8)
    _check(lib().dis_flow_color(_ptr(f), n, W, H, float(maxmotion), _ptr(out), MEM_HOST, None, device))
    return out[0] if single else out


def read_flo(path: str, channels: int = 2) -> np.ndarray:
    """Read a Middlebury .flo file (src/IO_flow.cpp:10-53) -> (H, W, channels) float32."""
    w, h = ctypes.c_int(), ctypes.c_int()
    _check(lib().dis_flo_info(os.fsencode(path), ctypes.byref(w), ctypes.byref(h)))
    out = np.empty((h.value, w.value, channels), np.float32)
    _check(lib().dis_read_flo(os.fsencode(path), _ptr(out), w.value, h.value, channels))
    return out


def write_flo(path: str, data: np.ndarray) -> None:
    """Write (H, W, channels) float32 as a .flo file (src/IO_flow.cpp:56-98)."""
    d = np.ascontiguousarray(data, dtype=np.float32)
    if d.ndim == 2:
        d = d[..., None]
    _check(lib().dis_write_flo(os.fsencode(path), _ptr(d), d.shape[1], d.shape[0], d.shape[2]))


def batch_stream_plan(nsub: int, nstages: int) -> list:
    """The fork / stage / join ops a batch call with nsub sub-batches issues
    (dis_batch_stream_plan): list of (kind, stream, event, stage)."""
    n = ctypes.c_int()
    _check(lib().dis_batch_stream_plan(nsub, nstages, None, 0, ctypes.byref(n)))
    buf = (ctypes.c_int * (4 * n.value))()
    _check(lib().dis_batch_stream_plan(nsub, nstages, buf, n.value, ctypes.byref(n)))
    return [tuple(buf[4 * i:4 * i + 4]) for i in range(n.value)]


def check_stream_plan(ops, nstreams: int, nevents: int) -> str | None:
    """None if the plan keeps the capture rules (dis_check_stream_plan), else
    the broken rule."""
    flat = [int(v) for op in ops for v in op]
    buf = (ctypes.c_int * max(1, len(flat)))(*flat)
    st = lib().dis_check_stream_plan(buf, len(ops), nstreams, nevents)
    return None if st == DIS_OK else lib().dis_last_error().decode()


def synth_pair(seed: int, width: int, height: int, with_gt: bool = False):
    """Deterministic synthetic u8 pair (and ground-truth flow) for seed."""
    I0 = np.empty((height, width), np.uint8)
    I1 = np.empty((height, width), np.uint8)
    gt = np.empty((height, width, 2), np.float32) if with_gt else None
    _check(lib().dis_synth_pair(seed, width, height, _ptr(I0), _ptr(I1), _ptr(gt) if with_gt else None))
    return (I0, I1, gt) if with_gt else (I0, I1)


class DenseInverseSearch:
    """One device context for W x H pairs (dis_create / dis_destroy)."""

    def __init__(self, params, width: int, height: int, max_batch: int = 1, device: int = 0):
        if isinstance(params, (Preset, int)) and not isinstance(params, Params):
            params = preset_params(Preset(params), width, height)
        self.params = params
        self.width, self.height, self.max_batch = width, height, max_batch
        self._ctx = ctypes.c_void_p()
        _check(lib().dis_create(ctypes.byref(self._ctx), ctypes.byref(params._c()), width, height,
                                max_batch, device))

    def close(self) -> None:
        if self._ctx:
            lib().dis_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def calc(self, I0: np.ndarray, I1: np.ndarray) -> np.ndarray:
        """u8 H x W frames (host) -> H x W x 2 float32 flow (host)."""
        return self.calc_batch(I0[None], I1[None])[0]

    def calc_batch(self, I0: np.ndarray, I1: np.ndarray) -> np.ndarray:
        I0 = np.ascontiguousarray(I0, dtype=np.uint8)
        I1 = np.ascontiguousarray(I1, dtype=np.uint8)
        if I0.shape != I1.shape or I0.ndim != 3 or I0.shape[1:] != (self.height, self.width):
            raise DisError(DIS_ERR_INVALID_ARGUMENT, f"frames must be (n, {self.height}, {self.width})")
        n = I0.shape[0]
        flow = np.empty((n, self.height, self.width, 2), np.float32)
        _check(lib().dis_calc_batch_u8(self._ctx, n, _ptr(I0), _ptr(I1), self.width,
                                       self.width * self.height, _ptr(flow), MEM_HOST, None))
        return flow

    def calc_device(self, n: int, I0_ptr: int, I1_ptr: int, flow_ptr: int, stream: int = 0,
                    stride: int = 0, pair_stride: int = 0) -> None:
        """Asynchronous calc on device-resident buffers (raw device pointers)."""
        _check(lib().dis_calc_batch_u8(self._ctx, n, I0_ptr, I1_ptr, stride, pair_stride, flow_ptr,
                                       MEM_DEVICE, stream or None))

    def set_host_pipeline(self, chunk_pairs: int = 0) -> None:
        """dis_set_host_pipeline: pairs per chunk of a host-memory batch call
        (0 = auto, about 64 MB of flow); results are identical."""
        _check(lib().dis_set_host_pipeline(self._ctx, chunk_pairs))

    def host_pipeline_info(self) -> dict:
        """What the last host-memory call did (chunks, direct DMA of page-locked buffers)."""
        h = _HostInfo()
        _check(lib().dis_host_pipeline_info(self._ctx, ctypes.byref(h)))
        return {k: getattr(h, k) for k, _ in _HostInfo._fields_}

    def calc_batch_host(self, n: int, I0_ptr: int, I1_ptr: int, flow_ptr: int, stride: int = 0,
                        pair_stride: int = 0) -> None:
        """dis_calc_batch_u8 on raw host pointers (pageable or page-locked), synchronous."""
        _check(lib().dis_calc_batch_u8(self._ctx, n, I0_ptr, I1_ptr, stride, pair_stride, flow_ptr,
                                       MEM_HOST, None))

    def set_variant(self, variant: int) -> None:
        """dis_set_kernel_variant (include/dis_abi.h): 0 = auto (specialised kernels),
        1 = generic only, 2 / 3 / 4 / 5 = 4 / 2 / 8 / 1 lanes per patch, 6 = one wave
        per patch, 9 = 2 lanes per patch with the usable LDS tile capped at 24 pixels
        (test hook: most blocks take the fallback list and k_search8_fb); 7 and 8
        were removed in ABI v7."""
        _check(lib().dis_set_kernel_variant(self._ctx, variant))

    def set_concurrency(self, streams: int) -> None:
        """Sub-batch streams per calc (1..8); results are identical for any value."""
        _check(lib().dis_set_concurrency(self._ctx, streams))

    def set_precision(self, mode: int) -> None:
        """PRECISION_EXACT (default, bit-identical to the reference order) or
        PRECISION_FMA (contracted search arithmetic, within the stated tolerance)."""
        _check(lib().dis_set_precision(self._ctx, mode))

    def set_graphs(self, on: bool = True) -> None:
        """Replay batch calls as captured HIP graphs (default on); results are identical."""
        _check(lib().dis_set_graphs(self._ctx, int(on)))

    def set_debug(self, on: bool = True) -> None:
        _check(lib().dis_set_debug(self._ctx, int(on)))

    def debug_dump(self, stage: int, level: int, pair: int = 0) -> np.ndarray:
        cnt = ctypes.c_size_t()
        _check(lib().dis_stage_size(self._ctx, stage, level, ctypes.byref(cnt)))
        out = np.empty(cnt.value, np.float32)
        _check(lib().dis_debug_dump(self._ctx, stage, level, pair, _ptr(out), cnt.value))
        return out

    def fallback_blocks(self, level: int) -> int:
        """Patch blocks of `level` the last calc searched with the fallback
        kernel (start positions too spread for the LDS tile), all sub-batches."""
        return int(self.debug_dump(STAGE_FALLBACK, level)[0])

    def set_kernel_timing(self, on: bool = True) -> None:
        _check(lib().dis_set_kernel_timing(self._ctx, int(on)))

    def kernel_time(self, kernel: int):
        n = ctypes.c_int()
        ms = ctypes.c_double()
        _check(lib().dis_kernel_time(self._ctx, kernel, ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value


def optical_flow_from_pyramids(img_first, img_first_dx, img_first_dy, img_second, img_padding: int,
                               width: int, height: int, coarsest_scale: int, finest_scale: int,
                               iterations: int, patch_size: int, patch_overlap: float,
                               patch_normalization: bool, img_second_dx=None, img_second_dy=None,
                               device: int = 0) -> np.ndarray:
    """OpticalFlowClass(...) (include/optical_flow.hpp:43-54) over padded host
    pyramids (lists of float32 2-D arrays, level 0..C). Returns the finest-level
    flow ((height>>F) x (width>>F) x 2)."""
    nl = coarsest_scale + 1

    def arr(planes):
        planes = [np.ascontiguousarray(p, dtype=np.float32) if p is not None else None for p in planes]
        ptrs = (ctypes.c_void_p * nl)(*[p.ctypes.data if p is not None else None for p in planes])
        return planes, ptrs

    keep = []
    ptrs = []
    for planes in (img_first, img_first_dx, img_first_dy, img_second,
                   img_second_dx or [None] * nl, img_second_dy or [None] * nl):
        k, p = arr(planes)
        keep.append(k)
        ptrs.append(ctypes.cast(p, ctypes.POINTER(ctypes.c_void_p)))
    out = np.empty(((height >> finest_scale), (width >> finest_scale), 2), np.float32)
    _check(lib().dis_flow_from_pyramids(*ptrs, img_padding, _ptr(out), width, height, coarsest_scale,
                                        finest_scale, iterations, patch_size, patch_overlap,
                                        int(patch_normalization), device))
    return out
