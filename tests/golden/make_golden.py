"""Generate the golden fixtures in tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).

Inputs are seeded numpy frames; expected flows come from the C oracle
(oracle/dis_oracle.c). The reference itself cannot be built here (OpenCV 2.4 /
Eigen 3 absent) and ships no fixtures, so these vectors are a regression lock
of the oracle -- they pin the restatement, not the reference.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_binding  # noqa: E402
from test_oracle import shifted_pair  # noqa: E402

CASES = {
    # name: (W, H, seed, dx, dy, C, F, ps, it, overlap, norm)
    "small_c2f0_ps8": (64, 48, 1, 1.25, -0.5, 2, 0, 8, 8, 0.5, 1),
    "ultrafast_160x120": (160, 120, 2, 2.5, 1.0, 3, 2, 8, 12, 0.5, 1),
    "medium_knobs_96x80": (96, 80, 3, -1.5, 0.75, 3, 1, 8, 25, 0.625, 1),
    "ragged_ps4_nonorm": (75, 53, 4, 0.5, 0.5, 2, 0, 4, 6, 0.5, 0),
}


def main():
    for name, (W, H, seed, dx, dy, C, F, ps, it, ov, norm) in CASES.items():
        I0, I1 = shifted_pair(seed, H, W, dx=dx, dy=dy)
        flow = oracle_binding.calc_u8(I0, I1, C, F, ps, it, ov, norm)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), I0=I0, I1=I1, flow=flow,
                            knobs_i=np.array([C, F, ps, it, norm], np.int32),
                            knobs_f=np.array([ov], np.float32))
        print(name, flow.shape, float(np.abs(flow).max()))


if __name__ == "__main__":
    main()
