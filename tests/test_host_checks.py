"""Host-side proofs behind exactness claims of the HIP search kernel.

div_pre (csrc/dis_search8.hip): the per-update divisions of the 2x2 LU solve
(src/patch.cpp:176, Eigen PartialPivLU::solve) by the patch's fixed pivots are
computed from one correctly rounded reciprocal per patch plus two fma
corrections; tools/div_check.c compares that sequence with IEEE division on
random operands of the kernel's range (the GPU parity tests then compare whole
flows bit for bit)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_div_pre_matches_ieee_division(tmp_path):
    exe = str(tmp_path / "div_check")
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                           os.path.join(ROOT, "tools", "div_check.c"), "-lm"])
    out = subprocess.run([exe, "10000000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    assert "0 mismatches" in out.stdout
