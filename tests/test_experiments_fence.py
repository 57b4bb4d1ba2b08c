"""The DIS_EXP_* knock-out switches (wrong values by design) can
never reach a product build: csrc/dis_experiments.h lists every one of them and
#errors unless DIS_EXPERIMENTS is defined, and the Makefile's default build
never defines it. CPU only: greps and the preprocessor."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd")
CSRC = os.path.join(PKG, "csrc")
FENCE = os.path.join(CSRC, "dis_experiments.h")


def _tokens_in_csrc():
    toks = set()
    for f in os.listdir(CSRC):
        if f == "dis_experiments.h":
            continue
        toks |= set(re.findall(r"\bDIS_EXP_\w+", open(os.path.join(CSRC, f)).read()))
    return toks


def _fenced():
    txt = open(FENCE).read()
    return set(re.findall(r"defined\((DIS_EXP_\w+)\)", txt))


def test_every_knockout_switch_is_fenced():
    toks = _tokens_in_csrc()
    assert toks, "no DIS_EXP_ switches found: the grep is broken"
    missing = toks - _fenced()
    assert not missing, f"DIS_EXP_ switches not listed in dis_experiments.h: {sorted(missing)}"


def test_every_source_includes_the_fence_first():
    # dis_common.h includes it before anything else; every .hip reaches it
    # through dis_kernels.h / dis_common.h before its own DIS_EXP_ uses
    common = open(os.path.join(CSRC, "dis_common.h")).read()
    first = re.search(r'#include\s+[<"]([^>"]+)[>"]', common).group(1)
    assert first == "dis_experiments.h"
    for f in os.listdir(CSRC):
        if not f.endswith(".hip"):
            continue
        src = open(os.path.join(CSRC, f)).read()
        m = re.search(r"\bDIS_EXP_\w+", src)
        if not m:
            continue
        inc = [mm.start() for mm in re.finditer(r'#include\s+"dis_(kernels|common)\.h"', src)]
        assert inc and inc[0] < m.start(), f"{f}: a DIS_EXP_ use comes before the fence is included"


def test_default_build_never_defines_experiments():
    mk = open(os.path.join(PKG, "Makefile")).read()
    assert "DIS_EXPERIMENTS" not in mk and "DIS_EXP_" not in mk
    gd = open(os.path.join(ROOT, "__graft_entry__.py")).read()
    assert "DIS_EXPERIMENTS" not in gd and "DIS_EXP_" not in gd


def _pp(*defs):
    return subprocess.run(["g++", "-E", "-x", "c++", *defs, FENCE], capture_output=True, text=True)


@pytest.mark.parametrize("switch", ["DIS_EXP_SKIP_HEAD=4", "DIS_EXP_NO_FB=1", "DIS_EXP_OUT_NOUPS"])
def test_knockout_without_experiments_fails(switch):
    r = _pp(f"-D{switch}")
    assert r.returncode != 0 and "DIS_EXPERIMENTS" in r.stderr
    r = _pp(f"-D{switch}", "-DDIS_EXPERIMENTS")
    assert r.returncode == 0 and '"experiment"' not in r.stdout  # macro only, expanded where used
    assert _pp().returncode == 0


def test_build_variants_adds_experiments_for_knockouts():
    sh = open(os.path.join(ROOT, "tools", "build_variants.sh")).read()
    assert "*DIS_EXP_*) flags=\"$flags -DDIS_EXPERIMENTS\"" in sh


def test_product_library_reports_product_kind():
    import sys
    sys.path.insert(0, PKG)
    import disflow
    if not os.path.exists(disflow.LIB_PATH):
        pytest.skip("library not built")
    assert disflow.build_kind() == "product"
