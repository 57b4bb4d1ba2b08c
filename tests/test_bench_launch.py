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


def _dry(world, **kw):
    env = _env(**kw)
    env.pop("DIS_BENCH_PLAN_ONLY")
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(world), "--dist-backend", "gloo", "--dry-run"],
                       env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    return lines[0]


def test_dry_run_config4_topology_8_ranks():
    # BASELINE config 4 (256 x 1080p pairs over 8 ranks) rehearsed
    # on the CPU: 8 gloo ranks, the 256 -> 32-per-rank shard plan, the bench's
    # own gather + checksum verification (gather_and_verify) and pair order
    line = _dry(8)
    assert line["n_gpus"] == 8 and line["value"] is None and line["dry_run"]
    assert line["config"]["global_batch"] == 256 and line["config"]["width"] == 1920
    assert line["shards"] == [[32 * r, 32 * (r + 1)] for r in range(8)]
    g = line["gather"]
    assert g["pairs"] == 256 and g["verified"] and g["pair_order_ok"] and g["world_size"] == 8
    assert g["bytes_received"] == 7 * 32 * 6 * 8 * 2 * 4


def test_dry_run_rank0_receive_failures_reach_every_rank():
    # rank 0 cannot hold the receive buffer (the check, or an allocation that
    # fails although the check passed): every rank leaves the gather together,
    # the line reports the error, nobody blocks in a collective
    for fail, text in (("check", "receive-buffer check failure"), ("alloc", "allocation failed")):
        g = _dry(8, DIS_BENCH_DRY_FAIL=fail)["gather"]
        assert "error" in g and text in g["error"], g


def test_dry_run_uneven_world():
    line = _dry(3)
    assert line["shards"] == [[0, 32], [32, 64], [64, 96]] and line["gather"]["pair_order_ok"]
