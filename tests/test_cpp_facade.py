"""The C++ facade (include/dis/dis.hpp: DenseInverseSearch::calc and the
OpticalFlow::OpticalFlowClass drop-in) exercised from C++ on the GPU and
checked bit-exactly against the oracle (tests/cpp/test_facade.cpp)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "cpp")])
    return os.path.join(HERE, "cpp", "test_facade")


def test_cpp_facade_builds():
    assert os.access(_build(), os.X_OK)


@pytest.mark.gpu
def test_cpp_facade_bitexact_on_gpu():
    exe = _build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK: 0 failure(s)" in r.stdout
