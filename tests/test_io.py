"""Middlebury .flo I/O (src/IO_flow.cpp:10-98) through the
C-ABI (host code, no GPU): byte layout, round trips, and the malformed-file
cases the reference only printed about."""
import struct

import numpy as np
import pytest


def test_flo_layout_matches_reference_format(disflow_mod, tmp_path):
    f = np.arange(3 * 5 * 2, dtype=np.float32).reshape(3, 5, 2) * 0.25 - 3
    p = tmp_path / "a.flo"
    disflow_mod.write_flo(str(p), f)
    raw = p.read_bytes()
    # "PIEH", int32 width, int32 height, then row-major interleaved float32 (:67-96)
    assert raw[:4] == b"PIEH"
    assert struct.unpack("<ii", raw[4:12]) == (5, 3)
    assert np.array_equal(np.frombuffer(raw[12:], "<f4"), f.ravel())
    assert struct.unpack("<f", b"PIEH")[0] == 202021.25  # the tag read as a float (:19)


@pytest.mark.parametrize("channels", [1, 2, 4])
def test_flo_round_trip(disflow_mod, tmp_path, channels):
    rng = np.random.default_rng(channels)
    f = rng.standard_normal((7, 11, channels)).astype(np.float32)
    f.flat[3] = np.nan
    p = str(tmp_path / "r.flo")
    disflow_mod.write_flo(p, f)
    g = disflow_mod.read_flo(p, channels)
    assert np.array_equal(g.view(np.uint32), f.view(np.uint32))


def test_flo_malformed_files_fail_loudly(disflow_mod, tmp_path):
    f = np.zeros((4, 6, 2), np.float32)
    good = tmp_path / "g.flo"
    disflow_mod.write_flo(str(good), f)
    raw = good.read_bytes()
    cases = {
        "tag": b"PIEX" + raw[4:],
        "short": raw[:-4],
        "long": raw + b"\0\0\0\0",
        "header": raw[:6],
        "dims": raw[:4] + struct.pack("<ii", 0, 4) + raw[12:],
    }
    for name, data in cases.items():
        p = tmp_path / f"{name}.flo"
        p.write_bytes(data)
        with pytest.raises(disflow_mod.DisError):
            disflow_mod.read_flo(str(p))
    with pytest.raises(disflow_mod.DisError):
        disflow_mod.read_flo(str(tmp_path / "missing.flo"))
    with pytest.raises(disflow_mod.DisError):  # wrong channel count for the file size
        disflow_mod.read_flo(str(good), 4)
