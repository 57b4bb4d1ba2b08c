"""Multi-GPU runner: frame pairs shard across ranks (one process per GPU).

The reference processes one pair at a time with no cross-pair state
(src/main.cpp:102-206 rebuilds everything per pair), so the path partitions
embarrassingly: rank r computes a contiguous block of pairs on its own device
with its own dis_ctx. There is no collective on the data path; the only
exchange is an optional gather of results to rank 0 (per-pair checksums by
default, whole flow fields on request) over the process group's backend (RCCL
for `nccl`, gloo on CPU in tests).
"""
from __future__ import annotations

import hashlib
import os
from typing import Callable, Optional, Sequence

import numpy as np


def shard_bounds(n_pairs: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced block [start, stop) of pairs owned by `rank`."""
    if world < 1 or not (0 <= rank < world) or n_pairs < 0:
        raise ValueError("bad shard request")
    start = n_pairs * rank // world
    stop = n_pairs * (rank + 1) // world
    return start, stop


def flow_digest(flow: np.ndarray) -> str:
    """Bit-exact fingerprint of one flow field (sha256 of its float32 bytes)."""
    return hashlib.sha256(np.ascontiguousarray(flow, dtype=np.float32).tobytes()).hexdigest()


def _default_compute(params, width: int, height: int, device: int, max_batch: int):
    from . import DenseInverseSearch

    eng = DenseInverseSearch(params, width, height, max_batch=max_batch, device=device)

    def compute(I0: np.ndarray, I1: np.ndarray) -> np.ndarray:
        out = []
        for k in range(0, I0.shape[0], max_batch):
            out.append(eng.calc_batch(I0[k:k + max_batch], I1[k:k + max_batch]))
        return np.concatenate(out) if out else np.empty((0, height, width, 2), np.float32)

    return compute


class ShardFailure(RuntimeError):
    """Raised on every rank of run_sharded when any rank's compute failed."""


def _agree_or_fail(err, rank: int, world: int, group=None):
    """Collective status check before the gather: each rank contributes 1 if
    its compute raised; when any did, every rank raises ShardFailure at once
    (instead of the healthy ranks blocking in the gather until the process
    group times out). The failing rank re-raises its own exception."""
    import torch
    import torch.distributed as dist

    dev = "cpu"
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    flags = torch.zeros(world, dtype=torch.int32, device=dev)
    flags[rank] = 0 if err is None else 1
    dist.all_reduce(flags, op=dist.ReduceOp.SUM, group=group)
    bad = [r for r in range(world) if int(flags[r]) != 0]
    if err is not None:
        raise ShardFailure(f"rank {rank}: shard compute failed: {err!r}") from err
    if bad:
        raise ShardFailure(f"rank {rank}: rank(s) {bad} failed their shard; aborting")


def run_sharded(I0: np.ndarray, I1: np.ndarray, params, width: int, height: int, *, rank: int = 0,
                world: int = 1, device: int = 0, max_batch: int = 32, gather_flows: bool = False,
                compute: Optional[Callable[[np.ndarray, np.ndarray], np.ndarray]] = None,
                group=None):
    """Compute this rank's shard of the (n, H, W) u8 pair stacks I0/I1.

    Every rank receives the full input stacks (or views of them) and computes
    pairs shard_bounds(n, rank, world). Returns, on rank 0, a dict with
    `digests` (per pair, in pair order) and, if gather_flows, `flows`
    (n, H, W, 2); other ranks return their local result dict.
    """
    n = I0.shape[0]
    a, b = shard_bounds(n, rank, world)
    err = None
    try:
        if compute is None:
            compute = _default_compute(params, width, height, device, max_batch)
        local = compute(I0[a:b], I1[a:b]) if b > a else np.empty((0, height, width, 2), np.float32)
    except Exception as e:  # noqa: BLE001 -- reported to every rank below, then re-raised
        err = e
    if world > 1:
        _agree_or_fail(err, rank, world, group)
    elif err is not None:
        raise err
    digests = [flow_digest(f) for f in local]
    result = {"start": a, "stop": b, "digests": digests}
    if gather_flows:
        result["flows"] = local
    if world == 1:
        return result
    import torch.distributed as dist

    gathered: Optional[Sequence] = [None] * world if rank == 0 else None
    payload = {"start": a, "stop": b, "digests": digests, "flows": local if gather_flows else None}
    dist.gather_object(payload, gathered, dst=0, group=group)
    if rank != 0:
        return result
    parts = sorted(gathered, key=lambda p: p["start"])
    out = {"start": 0, "stop": n, "digests": [d for p in parts for d in p["digests"]]}
    if gather_flows:
        out["flows"] = np.concatenate([p["flows"] for p in parts])
    return out


def gather_buffer_bytes(n_total: int, world: int, height: int, width: int) -> int:
    """Bytes rank 0 allocates to receive the gather: world x (largest shard)
    flows of height x width x 2 float32 (config 4: 8 x 32 x 16.6 MB = 4.25 GB)."""
    m = max(shard_bounds(n_total, r, world)[1] - shard_bounds(n_total, r, world)[0] for r in range(world))
    return world * m * height * width * 2 * 4


def check_gather_fits(nbytes: int, free_bytes: int, margin: float = 0.9) -> None:
    """Raise MemoryError (before any rank blocks in the collective) unless the
    receive buffer fits in `margin` of the free memory where it is allocated."""
    if nbytes > margin * free_bytes:
        raise MemoryError(f"gather needs {nbytes / 1e9:.2f} GB on rank 0, only {free_bytes / 1e9:.2f} GB free "
                          f"(limit {margin:.0%}): gather checksums instead (gather_checksums)")


def gather_flow_tensor(local, n_total: int, rank: int, world: int, group=None):
    """The single collective of the multi-GPU path: gather every
    rank's (n_r, H, W, 2) float32 flows -- device tensors under RCCL (`nccl`),
    host tensors under gloo -- into one (n_total, H, W, 2) tensor on rank 0,
    in pair order (shard_bounds blocks). Shards may differ by one pair: each is
    padded to the largest before the gather and cut after. Returns the tensor on
    rank 0 and None elsewhere."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "gloo" and local.is_cuda:  # gloo gathers host tensors
        local = local.cpu()
    a, b = shard_bounds(n_total, rank, world)
    if local.shape[0] != b - a:
        raise ValueError(f"rank {rank} holds {local.shape[0]} flows, its shard is {b - a}")
    m = max(shard_bounds(n_total, r, world)[1] - shard_bounds(n_total, r, world)[0] for r in range(world))
    send = local
    if local.shape[0] < m:
        send = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        send[:local.shape[0]] = local
    # rank 0 receives straight into one (world, m, ...) buffer: with equal
    # shards (the bench case) that buffer IS the result, no second copy.
    # Every rank checks rank 0's room first (the verdict is shared through the
    # group, so no rank is left blocked in the gather when rank 0 cannot
    # allocate): device memory under RCCL, host memory under gloo.
    # The receive buffer is allocated BEFORE the broadcast, so an allocation
    # that fails although the check passed (fragmentation, a concurrent user;
    # torch raises OutOfMemoryError, a RuntimeError) is shared too.
    nbytes = world * m * int(np.prod(local.shape[1:])) * local.element_size()
    ok = torch.ones(1, dtype=torch.int32, device=local.device)
    err, buf = None, None
    if rank == 0:
        try:
            if local.is_cuda:
                free = torch.cuda.mem_get_info(local.device)[0]
            else:
                free = os.sysconf("SC_AVPHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
            check_gather_fits(nbytes, free)
            buf = torch.empty((world,) + tuple(send.shape), dtype=send.dtype, device=send.device)
        except (MemoryError, RuntimeError) as e:
            ok.zero_()
            err = e if isinstance(e, MemoryError) else MemoryError(f"gather: receive buffer allocation failed: {e}")
            buf = None
    dist.broadcast(ok, src=0, group=group)
    if not int(ok.item()):
        raise err if err is not None else MemoryError("gather: rank 0 has no room for the receive buffer")
    recv = list(buf.unbind(0)) if rank == 0 else None
    dist.gather(send.contiguous(), recv, dst=0, group=group)
    if rank != 0:
        return None
    if all(shard_bounds(n_total, r, world)[1] - shard_bounds(n_total, r, world)[0] == m for r in range(world)):
        return buf.view((world * m,) + tuple(send.shape[1:]))
    parts = []
    for r in range(world):
        ra, rb = shard_bounds(n_total, r, world)
        parts.append(buf[r, :rb - ra])
    return torch.cat(parts)


def flow_checksum(flows):
    """Bit-level fingerprint of a float32 flow tensor, computed where it lives:
    two int64 sums of its 32-bit patterns (plain and position-weighted,
    wrapping), so a reordered, truncated or altered shard changes it."""
    import torch

    v = flows.contiguous().view(torch.int32).reshape(-1).to(torch.int64)
    w = torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 65521 + 1
    return torch.stack([v.sum(), (v * w).sum(), torch.tensor(v.numel(), device=v.device)])


def any_rank_failed(failed: bool, world: int, group=None, device=None) -> bool:
    """Collective OR of a per-rank failure flag (all_reduce MAX): every rank
    gets the same answer, so all take the same branch before the next
    collective (a failure seen by one rank must not leave the others
    blocked in a collective it skips)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return failed
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    f = torch.tensor([1 if failed else 0], dtype=torch.int32, device=device)
    dist.all_reduce(f, op=dist.ReduceOp.MAX, group=group)
    return bool(int(f.item()))


def gather_checksums(local_sum, rank: int, world: int, group=None):
    """Every rank's flow_checksum to rank 0 (a list in rank order there, None
    elsewhere)."""
    import torch.distributed as dist

    if dist.get_backend(group) == "gloo" and local_sum.is_cuda:
        local_sum = local_sum.cpu()
    recv = [local_sum.new_empty(local_sum.shape) for _ in range(world)] if rank == 0 else None
    dist.gather(local_sum.contiguous(), recv, dst=0, group=group)
    return recv
