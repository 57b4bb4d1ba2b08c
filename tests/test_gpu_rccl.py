"""The RCCL branch of the multi-GPU path on real hardware, as far as one GPU
allows: a one-rank `nccl` (RCCL) process group runs the bench's collectives --
disflow.multi.gather_flow_tensor (the room check's broadcast, then the gather
of device flows into rank 0's receive buffer) and gather_checksums -- on flows
the engine computed on the card. RCCL refuses two ranks on one device, so the
multi-rank forms run under gloo in tests/test_multi.py and test_bench_launch.py,
and with more GPUs only in the driver's scaling run. In a child
process: the group's RCCL state stays out of the test process."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd")

CHILD = r"""
import sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, sys.argv[1])
import disflow
from disflow import multi

torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[2], rank=0, world_size=1)
W, H, B = 320, 240, 3
pairs = [disflow.synth_pair(k, W, H) for k in range(B)]
d0 = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
d1 = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
out = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
eng = disflow.DenseInverseSearch(disflow.preset_params(disflow.Preset.MEDIUM, W, H), W, H, max_batch=B)
eng.calc_device(B, d0.data_ptr(), d1.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
full = multi.gather_flow_tensor(out, B, 0, 1)
assert full is not None and full.is_cuda and tuple(full.shape) == (B, H, W, 2), "gather shape"
assert torch.equal(full.view(torch.int32), out.view(torch.int32)), "gathered flows differ"
sums = multi.gather_checksums(multi.flow_checksum(out), 0, 1)
assert len(sums) == 1 and torch.equal(sums[0], multi.flow_checksum(full)), "checksums differ"
print("rccl ok", dist.get_backend(), tuple(full.shape), float(out.abs().max()))
dist.destroy_process_group()
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_gather_one_rank_on_device_flows():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-c", CHILD, PKG, str(_free_port())], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "rccl ok nccl" in r.stdout
