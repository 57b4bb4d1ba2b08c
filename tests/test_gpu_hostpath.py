"""The host-frame path (dis_calc_batch_u8 with DIS_MEM_HOST, ABI v8): batches
in chunks whose upload, computation and download overlap, the copies straight
between the caller's buffers (pageable or page-locked) and the device. The
reference's own call pattern is host frames in, host flow out
(src/main.cpp:102-206). Bar: the flows equal the device-resident path's bit
for bit (which the parity suite holds to the oracle), for every chunking and
buffer kind."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pairs(disflow, seeds, W, H):
    ps = [disflow.synth_pair(s, W, H) for s in seeds]
    return np.stack([a for a, _ in ps]), np.stack([b for _, b in ps])


def _device_flows(disflow, p, I0, I1):
    import torch
    n, H, W = I0.shape
    eng = disflow.DenseInverseSearch(p, W, H, max_batch=n)
    d0 = torch.from_numpy(I0).cuda()
    d1 = torch.from_numpy(I1).cuda()
    out = torch.empty((n, H, W, 2), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    eng.calc_device(n, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), s.cuda_stream)
    s.synchronize()
    eng.close()
    return out.cpu().numpy()


def _eq(got, exp, what):
    assert got.shape == exp.shape, (what, got.shape, exp.shape)
    bad = got.view(np.uint32) != exp.view(np.uint32)
    assert not bad.any(), f"{what}: {int(bad.sum())} values differ"


class _Pinned:
    """A numpy view of dis_host_alloc'd (page-locked) memory."""

    def __init__(self, disflow, shape, dtype):
        self.L = disflow.lib()
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        self.p = ctypes.c_void_p()
        disflow._check(self.L.dis_host_alloc(nbytes, ctypes.byref(self.p)))
        buf = (ctypes.c_char * nbytes).from_address(self.p.value)
        self.a = np.frombuffer(buf, dtype=dtype).reshape(shape)

    def free(self):
        self.a = None
        self.L.dis_host_free(self.p)


@pytest.mark.parametrize("chunk", [0, 2, 1, 9])
def test_host_batch_chunks_bitexact_1080p(disflow_mod, chunk):
    d = disflow_mod
    W, H, n = 1920, 1080, 9
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    I0, I1 = _pairs(d, range(40, 40 + n), W, H)
    exp = _device_flows(d, p, I0, I1)
    eng = d.DenseInverseSearch(p, W, H, max_batch=n)
    eng.set_host_pipeline(chunk)
    for rep in range(2):  # the second call replays the captured graphs of both slots
        got = eng.calc_batch(I0, I1)
        _eq(got, exp, f"chunk {chunk} call {rep}")
    info = eng.host_pipeline_info()
    want_chunk = chunk or 4  # auto: about 64 MB of 1080p flow
    assert info["chunk_pairs"] == want_chunk, info
    assert info["last_chunks"] == -(-n // want_chunk), info
    assert info["last_direct_in"] == 0 and info["last_direct_out"] == 0, info
    eng.close()


def test_host_batch_page_locked_buffers_direct(disflow_mod):
    d = disflow_mod
    W, H, n = 1280, 720, 7
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    I0, I1 = _pairs(d, range(70, 70 + n), W, H)
    exp = _device_flows(d, p, I0, I1)
    b0, b1 = _Pinned(d, I0.shape, np.uint8), _Pinned(d, I1.shape, np.uint8)
    fo = _Pinned(d, (n, H, W, 2), np.float32)
    b0.a[:] = I0
    b1.a[:] = I1
    eng = d.DenseInverseSearch(p, W, H, max_batch=n)
    eng.set_host_pipeline(3)
    eng.calc_batch_host(n, b0.a.ctypes.data, b1.a.ctypes.data, fo.a.ctypes.data)
    _eq(fo.a.copy(), exp, "page-locked in and out")
    info = eng.host_pipeline_info()
    assert info["last_direct_in"] == 1 and info["last_direct_out"] == 1 and info["last_chunks"] == 3, info
    # page-locked frames, pageable flow (and the reverse)
    flow = np.empty((n, H, W, 2), np.float32)
    eng.calc_batch_host(n, b0.a.ctypes.data, b1.a.ctypes.data, flow.ctypes.data)
    _eq(flow, exp, "page-locked in, pageable out")
    info = eng.host_pipeline_info()
    assert info["last_direct_in"] == 1 and info["last_direct_out"] == 0, info
    fo.a[:] = 0
    eng.calc_batch_host(n, I0.ctypes.data, I1.ctypes.data, fo.a.ctypes.data)
    _eq(fo.a.copy(), exp, "pageable in, page-locked out")
    eng.close()
    for b in (b0, b1, fo):
        b.free()


def test_host_batch_strided_frames_vs_oracle(disflow_mod, oracle):
    # row stride > width and a pair stride that is no multiple of it, chunks of
    # two pairs with a ragged last chunk, against the C oracle directly
    d = disflow_mod
    W, H, n = 203, 151, 5
    stride, pair_stride = W + 37, (W + 37) * H + 11
    p = d.preset_params(d.Preset.ULTRAFAST, W, H)
    I0, I1 = _pairs(d, range(90, 90 + n), W, H)
    buf0 = np.zeros(pair_stride * n, np.uint8)
    buf1 = np.zeros(pair_stride * n, np.uint8)
    for k in range(n):
        for y in range(H):
            buf0[k * pair_stride + y * stride:k * pair_stride + y * stride + W] = I0[k, y]
            buf1[k * pair_stride + y * stride:k * pair_stride + y * stride + W] = I1[k, y]
    eng = d.DenseInverseSearch(p, W, H, max_batch=n)
    eng.set_host_pipeline(2)
    flow = np.empty((n, H, W, 2), np.float32)
    eng.calc_batch_host(n, buf0.ctypes.data, buf1.ctypes.data, flow.ctypes.data, stride, pair_stride)
    for k in range(n):
        _eq(flow[k], oracle.calc_from_params(I0[k], I1[k], p), f"pair {k} vs oracle")
    assert eng.host_pipeline_info()["last_chunks"] == 3
    eng.close()


def test_host_batch_debug_mode_keeps_whole_batch(disflow_mod):
    # stage dumps read the last call's pairs: in debug mode the host path runs
    # the batch as one chunk whatever the chunk setting
    d = disflow_mod
    W, H, n = 320, 240, 3
    p = d.preset_params(d.Preset.MEDIUM, W, H)
    I0, I1 = _pairs(d, range(5, 5 + n), W, H)
    eng = d.DenseInverseSearch(p, W, H, max_batch=n)
    eng.set_host_pipeline(1)
    eng.set_debug(True)
    eng.calc_batch(I0, I1)
    assert eng.host_pipeline_info()["last_chunks"] == 1
    lvl = p.finest_scale
    last = eng.debug_dump(d.STAGE_PATCH_U, lvl, n - 1)
    single = d.DenseInverseSearch(p, W, H, max_batch=1)
    single.set_debug(True)
    single.calc(I0[n - 1], I1[n - 1])
    _eq(last, single.debug_dump(d.STAGE_PATCH_U, lvl, 0), "last pair's finest patch u")
    eng.set_debug(False)
    _eq(eng.calc_batch(I0, I1), _device_flows(d, p, I0, I1), "after debug off, chunked again")
    assert eng.host_pipeline_info()["last_chunks"] == 3
    eng.close()
    single.close()
