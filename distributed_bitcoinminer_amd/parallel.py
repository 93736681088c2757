"""Multi-GPU sharding of the nonce range: one process per GPU.

The reference parallelises the scan only across miner processes, by equal
contiguous chunks (cmu440/bitcoin/server/server.go:165-205), merging results
with a strict ``<`` (server.go:273-276).  On one MI355X node the same data
parallelism runs as one rank per GPU (torch.distributed, backend "nccl" =
RCCL over xGMI): every rank scans a contiguous shard with no communication,
then ONE all-gather of the 16-byte ``(hash, nonce)`` candidates and a
lexicographic min give the answer -- identical to a single-GPU scan because
the merge is associative, commutative and ties go to the lowest nonce.
"""
from __future__ import annotations

from typing import Callable

import numpy as np

MAXU64 = (1 << 64) - 1


def shard_range(lo: int, hi: int, world: int, rank: int, msg=None):
    """Contiguous shard `rank` of inclusive [lo, hi]; None when empty.

    With ``msg``: the cost-weighted split of hm_partition (the one hm_scan uses
    across the devices of one context): digit segments whose kernel costs more
    per nonce get fewer nonces, so ranks finish together.
    Without: equal counts, count = hi-lo+1 = world*q + (rr+1), shards 0..rr
    get q+1 nonces, the rest q."""
    if msg is not None:
        from . import _lib
        return _lib.partition(msg, lo, hi, world)[rank]
    if lo > hi:
        return None
    span_m1 = hi - lo
    q, rr = divmod(span_m1, world)
    start = lo + rank * q + min(rank, rr + 1)
    size = q + (1 if rank <= rr else 0)
    if size == 0:
        return None
    return start, start + size - 1


def merge(results) -> tuple[int, int]:
    """Lexicographic (hash, nonce) min seeded with (MaxUint64, 0)."""
    best = (MAXU64, 0)
    for r in results:
        r = (int(r[0]), int(r[1]))
        if r < best:
            best = r
    return best


def _pack(res) -> np.ndarray:
    return np.array([res[0], res[1]], dtype=np.uint64).view(np.int64)


def distributed_scan(msg, lo: int, hi: int, scan_fn: Callable, device=None):
    """Scan [lo, hi] across the default torch.distributed group.

    ``scan_fn(msg, a, b)`` scans one shard on this rank's GPU (normally
    ``Context.scan``).  The 16-B candidates are all-gathered (RCCL when the
    backend is nccl; gloo in CPU tests) and merged on every rank."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    shard = shard_range(lo, hi, world, rank, msg=msg)
    local = scan_fn(msg, shard[0], shard[1]) if shard is not None else (MAXU64, 0)
    t = torch.from_numpy(_pack(local))
    if device is not None:
        t = t.to(device)
    out = torch.empty(world * 2, dtype=torch.int64, device=t.device)
    dist.all_gather_into_tensor(out, t)
    arr = out.cpu().numpy().view(np.uint64).reshape(world, 2)
    return merge((int(a), int(b)) for a, b in arr)
