"""Multi-rank sharding of frame pairs (disflow.multi): world_size-2 gloo runs on
CPU with a deterministic stand-in compute (the real kernels need a GPU), and a
GPU run where two processes share the one card of the test box and must
reproduce the single-process flows bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import disflow.multi as multi


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_compute(I0, I1):
    # deterministic per-pair stand-in for the GPU path (no cross-pair state)
    d = I1.astype(np.float32) - I0.astype(np.float32)
    return np.stack([d, d * 0.5], axis=-1)


def _pairs(n, H=12, W=16, seed=3):
    rng = np.random.default_rng(seed)
    return (rng.integers(0, 256, (n, H, W), dtype=np.uint8), rng.integers(0, 256, (n, H, W), dtype=np.uint8))


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 32, 256):
        for world in (1, 2, 3, 8):
            got = [multi.shard_bounds(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(got[i][1] == got[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        multi.shard_bounds(4, 2, 2)


def _worker(rank, world, port, n, out_q, use_gpu):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        I0, I1 = _pairs(n) if not use_gpu else _gpu_pairs(n)
        if use_gpu:
            import disflow
            H, W = I0.shape[1:]
            p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
            res = multi.run_sharded(I0, I1, p, W, H, rank=rank, world=world, device=0, max_batch=4,
                                    gather_flows=True)
        else:
            res = multi.run_sharded(I0, I1, None, 16, 12, rank=rank, world=world, compute=_fake_compute,
                                    gather_flows=True)
        if rank == 0:
            out_q.put((res["digests"], res["flows"]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _gather_worker(rank, world, port, n, out_q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        I0, I1 = _pairs(n)
        a, b = multi.shard_bounds(n, rank, world)
        local = torch.from_numpy(_fake_compute(I0[a:b], I1[a:b]))
        got = multi.gather_flow_tensor(local, n, rank, world)
        if rank == 0:
            out_q.put(got.numpy())
        else:
            assert got is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _gpu_pairs(n):
    import disflow
    pairs = [disflow.synth_pair(100 + k, 192, 144) for k in range(n)]
    return np.stack([a for a, _ in pairs]), np.stack([b for _, b in pairs])


def _run(world, n, use_gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q, use_gpu)) for r in range(world)]
    for p in procs:
        p.start()
    digests, flows = q.get(timeout=600)
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    return digests, flows


def test_gloo_world2_gathers_all_pairs_in_order():
    n = 7
    digests, flows = _run(2, n, use_gpu=False)
    I0, I1 = _pairs(n)
    single = multi.run_sharded(I0, I1, None, 16, 12, compute=_fake_compute, gather_flows=True)
    assert digests == single["digests"]
    assert np.array_equal(flows, single["flows"])


@pytest.mark.gpu
def test_two_ranks_on_one_gpu_match_single_process():
    import disflow
    n = 6
    digests, flows = _run(2, n, use_gpu=True)
    I0, I1 = _gpu_pairs(n)
    H, W = I0.shape[1:]
    p = disflow.preset_params(disflow.Preset.MEDIUM, W, H)
    single = multi.run_sharded(I0, I1, p, W, H, max_batch=6, gather_flows=True)
    assert digests == single["digests"]
    assert np.array_equal(flows.view(np.uint32), single["flows"].view(np.uint32))


@pytest.mark.parametrize("world,n", [(2, 7), (3, 8)])
def test_gloo_tensor_gather_uneven_shards(world, n):
    # the bench's RCCL gather (gather_flow_tensor) with gloo on CPU tensors:
    # shards of unequal size come back whole and in pair order
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=600)
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    I0, I1 = _pairs(n)
    assert np.array_equal(got, _fake_compute(I0, I1))


def _fail_worker(rank, world, port, bad_rank, out_q):
    # one rank's compute raises: every rank must leave run_sharded promptly
    # with ShardFailure (no wait for the process-group timeout)
    import time

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=300))

    def compute(I0, I1):
        if rank == bad_rank:
            raise ValueError("injected failure")
        return _fake_compute(I0, I1)

    t0 = time.time()
    try:
        I0, I1 = _pairs(6)
        multi.run_sharded(I0, I1, None, 16, 12, rank=rank, world=world, compute=compute, gather_flows=True)
        out_q.put((rank, "no error", time.time() - t0))
    except multi.ShardFailure as e:
        out_q.put((rank, str(e), time.time() - t0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bad", [(2, 1), (3, 0)])
def test_gloo_failing_rank_fails_every_rank_promptly(world, bad):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, bad, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, msg, secs in res:
        assert msg != "no error"
        assert secs < 60  # far below the 300 s process-group timeout
        if rank == bad:
            assert "injected failure" in msg
        else:
            assert f"[{bad}]" in msg


def _checksum_worker(rank, world, port, n, out_q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        I0, I1 = _pairs(n)
        a, b = multi.shard_bounds(n, rank, world)
        local = torch.from_numpy(_fake_compute(I0[a:b], I1[a:b]))
        full = multi.gather_flow_tensor(local, n, rank, world)
        sums = multi.gather_checksums(multi.flow_checksum(local), rank, world)
        if rank == 0:
            ok = []
            for r in range(world):
                ra, rb = multi.shard_bounds(n, r, world)
                ok.append(torch.equal(multi.flow_checksum(full[ra:rb]), sums[r]))
            # a corrupted shard is detected
            bad = full[0:multi.shard_bounds(n, 0, world)[1]].clone()
            bad.view(-1)[5] += 1.0
            ok.append(not torch.equal(multi.flow_checksum(bad), sums[0]))
            out_q.put(ok)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 8), (3, 7)])
def test_gloo_gather_checksums_verify_shards(world, n):
    # bench.py's gather verification: per-rank bit-level checksums vs rank 0's
    # checksums of the gathered shards
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_checksum_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok)


def test_gather_buffer_size_config4_fits_one_mi355x():
    # BASELINE config 4: 256 x 1920x1080 pairs over 8 ranks, 32 per rank: rank 0
    # receives 8 x 32 flows of 16.6 MB = 4.25 GB, far inside 288 GB of HBM
    nbytes = multi.gather_buffer_bytes(256, 8, 1080, 1920)
    assert nbytes == 8 * 32 * 1080 * 1920 * 2 * 4
    assert abs(nbytes / 1e9 - 4.247) < 0.01
    multi.check_gather_fits(nbytes, 288 * 2**30)
    with pytest.raises(MemoryError):
        multi.check_gather_fits(nbytes, 4 * 2**30)
    # uneven shards: the buffer is world x the largest shard
    assert multi.gather_buffer_bytes(7, 2, 2, 3) == 2 * 4 * 2 * 3 * 2 * 4


def _gather_oom_worker(rank, world, port, out_q):
    # rank 0 cannot hold the receive buffer: every rank raises MemoryError
    # promptly instead of blocking in the collective
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=300))
    multi.check_gather_fits_orig = multi.check_gather_fits
    multi.check_gather_fits = lambda nbytes, free, margin=0.9: multi.check_gather_fits_orig(nbytes, 1)
    try:
        multi.gather_flow_tensor(torch.zeros((2, 4, 5, 2)), 2 * world, rank, world)
        out_q.put((rank, "no error"))
    except MemoryError as e:
        out_q.put((rank, "MemoryError" + (": " + str(e) if rank == 0 else "")))
    finally:
        dist.destroy_process_group()


def test_gloo_gather_refuses_when_rank0_has_no_room():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_oom_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=300)
    assert [g[0] for g in got] == [0, 1]
    assert all(g[1].startswith("MemoryError") for g in got), got
