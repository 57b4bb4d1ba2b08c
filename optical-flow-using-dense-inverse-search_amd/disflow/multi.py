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
    if compute is None:
        compute = _default_compute(params, width, height, device, max_batch)
    local = compute(I0[a:b], I1[a:b]) if b > a else np.empty((0, height, width, 2), np.float32)
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
    recv = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    dist.gather(send.contiguous(), recv, dst=0, group=group)
    if rank != 0:
        return None
    parts = []
    for r in range(world):
        ra, rb = shard_bounds(n_total, r, world)
        parts.append(recv[r][:rb - ra])
    return torch.cat(parts)
