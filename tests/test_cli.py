"""The frame-sequence CLI (src/main.cpp:59-206 conventions)
and its PNG codec: decoder cases on CPU (tests/cpp/png_tool), argument
handling on CPU, the end-to-end run on the GPU against the oracle."""
import os
import struct
import subprocess

import numpy as np
import pytest

import pngio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd")
CLI = os.path.join(PKG, "disflow", "dis_flow")
PNG_TOOL = os.path.join(ROOT, "tests", "cpp", "png_tool")


def _decode(path, tmp):
    out = os.path.join(tmp, "dec.raw")
    subprocess.run([PNG_TOOL, "gray", path, out], check=True)
    raw = open(out, "rb").read()
    w, h = struct.unpack("<ii", raw[:8])
    return np.frombuffer(raw[8:], np.uint8).reshape(h, w)


@pytest.fixture(scope="module")
def tools():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "png_tool"])
    subprocess.check_call(["make", "-s", "-C", PKG])
    return True


@pytest.mark.parametrize("ctype,depth", [(0, 8), (0, 16), (0, 1), (0, 2), (0, 4), (2, 8), (2, 16), (3, 8),
                                         (3, 4), (4, 8), (4, 16), (6, 8), (6, 16)])
def test_png_decoder_colour_types_and_depths(tools, tmp_path, ctype, depth):
    rng = np.random.default_rng(ctype * 100 + depth)
    H, W = 13, 17
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    s = rng.integers(0, 1 << depth, (H, W, ch))
    pal = None
    if ctype == 3:
        pal = rng.integers(0, 256, (1 << depth, 3))
    p = str(tmp_path / "x.png")
    pngio.write_png(p, s, ctype, depth, palette=pal)
    got = _decode(p, str(tmp_path))
    hi = (s >> 8) if depth == 16 else s
    if ctype == 0:
        exp = (s[..., 0] * 255 // ((1 << depth) - 1)) if depth < 8 else hi[..., 0]
    elif ctype == 4:
        exp = hi[..., 0]
    elif ctype == 3:
        rgb = pal[s[..., 0]]
        exp = pngio.luma(rgb[..., 0], rgb[..., 1], rgb[..., 2])
    else:
        exp = pngio.luma(hi[..., 0], hi[..., 1], hi[..., 2])
    assert np.array_equal(got, np.asarray(exp, np.uint8))


def test_png_encoder_round_trip(tools, tmp_path):
    rng = np.random.default_rng(1)
    bgr = rng.integers(0, 256, (9, 14, 3), dtype=np.uint8)
    raw = tmp_path / "b.raw"
    raw.write_bytes(bgr.tobytes())
    out = str(tmp_path / "b.png")
    subprocess.run([PNG_TOOL, "bgr", "14", "9", str(raw), out], check=True)
    assert np.array_equal(pngio.read_rgb8(out), bgr[..., ::-1])


def test_png_decoder_rejects_bad_files(tools, tmp_path):
    p = tmp_path / "bad.png"
    pngio.write_gray8(str(p), np.zeros((4, 4), np.uint8))
    d = bytearray(p.read_bytes())
    d[20] ^= 0xFF  # corrupt IHDR -> CRC mismatch
    p.write_bytes(bytes(d))
    r = subprocess.run([PNG_TOOL, "gray", str(p), str(tmp_path / "o.raw")], capture_output=True, text=True)
    assert r.returncode == 1 and "CRC" in r.stderr


def test_cli_bad_arguments_print_usage(tools, tmp_path):
    # src/main.cpp:93-101: wrong argument count prints the usage and returns 0
    r = subprocess.run([CLI, "a", "b"], capture_output=True, text=True, cwd=tmp_path)
    assert r.returncode == 0 and "Not good parameters!" in r.stdout
    r = subprocess.run([CLI, "f", "1", "2", "5", "8", "3", "0", "0.5", "1", "1"], capture_output=True, text=True,
                       cwd=tmp_path)
    assert r.returncode == 2  # draw_grid (GUI) unsupported


@pytest.mark.gpu
def test_cli_sequence_matches_oracle(tools, tmp_path, disflow_mod, oracle):
    # 4 frames -> 3 pairs in batches of 2, full 10-argument form, --flo
    W, H = 160, 96
    frames = [disflow_mod.synth_pair(50, W, H)[0]]
    for k in range(3):
        frames.append(disflow_mod.synth_pair(51 + k, W, H)[1])
    d = tmp_path / "seq"
    d.mkdir()
    for i, f in enumerate(frames, start=1):
        pngio.write_gray8(str(d / f"frame_{i:04d}.png"), f)
    args = [CLI, "seq", "1", "4", "10", "8", "3", "1", "0.5", "1", "0", "--flo", "--batch", "2"]
    r = subprocess.run(args, capture_output=True, text=True, cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("finish seq/frame_") == 3
    p = disflow_mod.Params(coarsest_scale=3, finest_scale=1, patch_size=8, iterations=10, patch_overlap=0.5,
                           patch_normalization=1)
    for i in range(1, 4):
        exp = oracle.calc_from_params(frames[i - 1], frames[i], p)
        flo = disflow_mod.read_flo(str(tmp_path / f"OF_seq/frame_{i:04d}.flo"))
        assert np.array_equal(flo.view(np.uint32), exp.view(np.uint32)), f"flow {i}"
        rgb = pngio.read_rgb8(str(tmp_path / f"OF_seq/frame_{i:04d}.png"))
        assert np.array_equal(rgb, oracle.flow_color(exp)[..., ::-1]), f"colour {i}"


@pytest.mark.gpu
def test_cli_paper_and_refine_options(tools, tmp_path, disflow_mod, oracle):
    # --paper and --refine K (8f row 1) reach dis_params
    W, H = 128, 96
    I0, I1 = disflow_mod.synth_pair(57, W, H)
    d = tmp_path / "pp"
    d.mkdir()
    pngio.write_gray8(str(d / "frame_0001.png"), I0)
    pngio.write_gray8(str(d / "frame_0002.png"), I1)
    args = [CLI, "pp", "1", "2", "8", "8", "3", "0", "0.5", "1", "0", "--flo", "--paper", "--refine", "2"]
    r = subprocess.run(args, capture_output=True, text=True, cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    p = disflow_mod.Params(coarsest_scale=3, finest_scale=0, patch_size=8, iterations=8, patch_overlap=0.5,
                           patch_normalization=1, var_refine_iters=2, paper_mode=1)
    exp = oracle.calc_from_params(I0, I1, p)
    flo = disflow_mod.read_flo(str(tmp_path / "OF_pp/frame_0001.flo"))
    assert np.array_equal(flo.view(np.uint32), exp.view(np.uint32))
