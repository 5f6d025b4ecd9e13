"""Multi-GPU partitioning of a checksum batch.

Blocks are independent, so a batch is split into contiguous ranges of
near-equal bytes -- one per rank (one process per GPU) -- and every rank
checksums its own range with no data-path collective.  The only
collectives are control: a barrier before/after the timed region and the
max-over-ranks of the elapsed time (plus sums of byte counts / mismatch
counts when a caller wants whole-job figures).  Works with any
torch.distributed backend (RCCL on the GPU box, gloo on CPU for tests).

The byte-balanced split itself is the engine's host-side
``mck_partition_spans`` (C ABI), so the ranks and the engine's own
multi-device pipeline (``mck_host_batch_checksum``) agree on it.
"""
from __future__ import annotations

import time
from typing import Optional, Sequence, Tuple

import numpy as np

from ._lib import check, lib


def partition_spans(lengths: Optional[Sequence[int]], count: int, parts: int,
                    length: int = 0) -> np.ndarray:
    """first[p] .. first[p+1] = the span range of part p (uint32[parts+1]).
    ``lengths`` = per-span byte lengths, or None with a uniform ``length``."""
    first = np.zeros(parts + 1, dtype=np.uint32)
    if lengths is not None:
        arr = np.ascontiguousarray(np.asarray(lengths, dtype=np.uint32))
        if arr.size != count:
            raise ValueError("len(lengths) != count")
        ptr = arr.ctypes.data
    else:
        ptr = None
    check(lib.mck_partition_spans(ptr, count, length, parts, first.ctypes.data),
          "mck_partition_spans")
    return first


def rank_range(lengths: Optional[Sequence[int]], count: int, world: int, rank: int,
               length: int = 0) -> Tuple[int, int]:
    """[begin, end) span indices this rank owns."""
    first = partition_spans(lengths, count, world, length)
    return int(first[rank]), int(first[rank + 1])


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def barrier(device=None) -> None:
    dist = _dist()
    if dist is None:
        return
    if device is not None and getattr(device, "type", "cpu") == "cuda":
        dist.barrier(device_ids=[device.index])
    else:
        dist.barrier()


def reduce_max(value: float, device=None) -> float:
    """Max over ranks (identity without a process group)."""
    dist = _dist()
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(value: int, device=None) -> int:
    """Sum over ranks of an integer count (bytes, mismatches)."""
    dist = _dist()
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.int64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def combine_span_crcs(local_crc, local_len: int, device=None) -> int:
    """One span split contiguously across ranks (rank r holds bytes
    [off_r, off_r + len_r)): each rank has the CRC32C of its slice (rank 0's
    may carry an init via Extend); the whole span's CRC is the
    util/crc32c.cc:1274 Crc32cCombine fold of the (crc, length) pairs in rank
    order -- the only data exchanged is 8 bytes per rank.
    ``local_crc``: int or a 1-element int32 tensor on ``device``."""
    import torch
    if not isinstance(local_crc, int):
        t = local_crc.reshape(1).to(torch.int64) & 0xFFFFFFFF
    else:
        t = torch.tensor([local_crc & 0xFFFFFFFF], dtype=torch.int64, device=device or "cpu")
    pair = torch.cat([t, torch.tensor([int(local_len)], dtype=torch.int64, device=t.device)])
    dist = _dist()
    if dist is None:
        parts = [pair]
    else:
        parts = [torch.empty_like(pair) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, pair)
    acc = 0
    for p in parts:
        crc, ln = (int(x) for x in p.cpu().tolist())
        acc = int(lib.mck_crc32c_combine(acc, crc, ln))
    return acc


def timed_steps(step, steps: int, sync=None, device=None) -> float:
    """Barrier + sync, run ``steps`` calls of ``step``, sync + barrier; the
    max over ranks of the wall time (seconds)."""
    if sync:
        sync()
    barrier(device)
    if sync:
        sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if sync:
        sync()
    barrier(device)
    if sync:
        sync()
    return reduce_max(time.perf_counter() - t0, device)


__all__ = ["partition_spans", "rank_range", "barrier", "reduce_max", "reduce_sum", "timed_steps",
           "combine_span_crcs"]
