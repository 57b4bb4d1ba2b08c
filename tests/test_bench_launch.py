"""bench.py's launch contract: `--gpus N` must either run N
ranks or fail -- it may never measure fewer GPUs and print them as N. Checked on
CPU with DIS_BENCH_PLAN_ONLY=1, which makes every rank print its layout and
exit before any GPU call."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["DIS_BENCH_PLAN_ONLY"] = "1"
    env.update(kw)
    return env


def _lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_gpus2_without_launcher_spawns_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo"], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    got = sorted((d["rank"], d["world"], d["gpus"]) for d in _lines(r.stdout))
    assert got == [(0, 2, 2), (1, 2, 2)]


def test_gpus_mismatch_world_size_fails():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dist-backend", "gloo"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE 1" in r.stderr
    assert not _lines(r.stdout)


def test_nccl_ranks_beyond_visible_gpus_fail():
    # this container has no GPU: 2 local ranks under nccl cannot each own one
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="2"),
                       capture_output=True, text=True, timeout=120)
    import torch
    if torch.cuda.device_count() >= 2:
        return
    assert r.returncode != 0
    assert "visible GPU" in r.stderr


def test_single_gpu_default_is_one_rank():
    r = subprocess.run([sys.executable, BENCH], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert [(d["rank"], d["world"], d["gpus"]) for d in _lines(r.stdout)] == [(0, 1, 1)]
