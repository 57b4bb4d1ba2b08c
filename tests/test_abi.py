"""CPU tests of the C-ABI boundary (no GPU compute): the HIP library loads,
exports every symbol include/dis_abi.h declares, validates parameters the way
the ABI contract says, and its host-only utilities behave."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dis_abi.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dis_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree(disflow_mod):
    assert declared_functions() == sorted(disflow_mod.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(disflow_mod):
    L = disflow_mod.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert L.dis_abi_version() == 8
    assert not hasattr(L, "dis_pipeline_link")  # removed in v6


def test_no_oracle_linked_into_product(disflow_mod):
    # the product library must not contain or link the CPU oracle
    data = open(disflow_mod.LIB_PATH, "rb").read()
    assert b"dis_oracle" not in data


def test_no_hard_profiler_dependency(disflow_mod):
    # the roctx markers are resolved with dlopen at first use, so the
    # library loads on a ROCm install without the roctx package
    import subprocess
    out = subprocess.run(["readelf", "-d", disflow_mod.LIB_PATH], capture_output=True, text=True, check=True).stdout
    needed = re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", out)
    assert needed and not [n for n in needed if "roctx" in n or "rocprofiler" in n], needed


def test_presets(disflow_mod):
    P = disflow_mod.Preset
    m = disflow_mod.preset_params(P.MEDIUM, 1920, 1080)
    assert (m.coarsest_scale, m.finest_scale, m.patch_size, m.iterations) == (6, 1, 8, 25)
    assert abs(m.patch_overlap - 0.625) < 1e-7
    u = disflow_mod.preset_params(P.ULTRAFAST, 640, 480)
    assert (u.coarsest_scale, u.finest_scale, u.iterations) == (4, 2, 12)
    k = disflow_mod.preset_params(P.MEDIUM, 3840, 2160)
    assert k.coarsest_scale == 7
    r = disflow_mod.preset_params(P.REFERENCE, 1024, 436)
    assert (r.coarsest_scale, r.finest_scale, r.iterations) == (3, 0, 1000)
    assert abs(r.patch_overlap - 0.7) < 1e-7
    tiny = disflow_mod.preset_params(P.ULTRAFAST, 40, 30)
    assert tiny.finest_scale <= tiny.coarsest_scale


@pytest.mark.parametrize("field,value,status", [
    ("patch_size", 7, -1),        # odd sizes are broken in the reference (Q11)
    ("patch_size", 0, -1),
    ("patch_size", 18, -1),
    ("patch_overlap", 1.0, -1),
    ("patch_overlap", -0.1, -1),
    ("finest_scale", 7, -1),      # F > C
    ("finest_scale", -1, -1),
    ("iterations", -1, -1),
    ("var_refine_iters", 65, -1),  # refinement iterations in [0, 64]
    ("var_refine_iters", -1, -1),
    ("paper_mode", 2, -1),        # 0 = the reference, 1 = DIS-paper residual / densification
    ("paper_mode", -1, -1),
])
def test_validation_errors(disflow_mod, field, value, status):
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, 1920, 1080)
    setattr(p, field, value)
    assert disflow_mod.validate(p, 1920, 1080) == status
    assert disflow_mod.lib().dis_last_error()


def test_validation_ok_and_size_errors(disflow_mod):
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, 1920, 1080)
    assert disflow_mod.validate(p, 1920, 1080) == 0
    assert disflow_mod.validate(p, 0, 1080) == -1
    L = disflow_mod.lib()
    assert L.dis_validate_params(None, 10, 10) == -1
    ctx = ctypes.c_void_p()
    assert L.dis_create(ctypes.byref(ctx), ctypes.byref(p._c()), 1920, 1080, 0, 0) == -1  # max_batch 0
    assert L.dis_create(None, ctypes.byref(p._c()), 1920, 1080, 1, 0) == -1
    assert L.dis_calc_u8(None, None, None, 0, None, 0, None) == -1
    assert L.dis_destroy(None) == 0


def test_workload_medium_1080p(disflow_mod):
    p = disflow_mod.preset_params(disflow_mod.Preset.MEDIUM, 1920, 1080)
    w = disflow_mod.workload(p, 1920, 1080)
    assert (w["padded_width"], w["padded_height"], w["steps"]) == (1920, 1088, 3)
    assert w["patches"] == 77700
    assert w["updates"] == 2020200
    assert w["patches_finest"] == 320 * 182
    assert w["search_flops_finest"] == 58240 * (1027 + 26 * 844)  # per patch / per update
    assert abs(w["algorithmic_bytes"] / 1e6 - 72.11) < 0.01
    u = disflow_mod.workload(disflow_mod.preset_params(disflow_mod.Preset.ULTRAFAST, 640, 480), 640, 480)
    assert u["patches"] == 1580 and u["updates"] == 20540
    assert abs(u["algorithmic_bytes"] / 1e6 - 7.38) < 0.01


def test_synth_pair_deterministic(disflow_mod):
    a0, a1, g = disflow_mod.synth_pair(3, 160, 120, with_gt=True)
    b0, b1 = disflow_mod.synth_pair(3, 160, 120)
    c0, _ = disflow_mod.synth_pair(4, 160, 120)
    assert np.array_equal(a0, b0) and np.array_equal(a1, b1)
    assert not np.array_equal(a0, c0)
    assert 90 < a0.mean() < 166 and a0.std() > 20
    assert np.abs(g).max() <= 6.0 + 1e-5


def test_create_without_gpu_fails_loudly(disflow_mod):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(disflow_mod.DisError) as e:
        disflow_mod.DenseInverseSearch(disflow_mod.Preset.MEDIUM, 64, 64)
    assert e.value.status == disflow_mod.DIS_ERR_DEVICE
