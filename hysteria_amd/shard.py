"""Packet-index sharding across GPUs.

Every datagram depends only on (PSK, salt, payload), so a batch shards by
datagram index with no exchange step: rank r of W processes a contiguous
range and writes its own output.  No collective is needed on the data path.
"""
from __future__ import annotations

import numpy as np


def check_rank_devices(bus_ids: list[str], device_count: int) -> bool:
    """Device binding of a one-process-per-GPU job (bench.py): ``bus_ids[r]`` is the PCI
    bus id rank r bound.  Returns True when two ranks share a card, which is only
    allowed when the node has fewer cards than ranks (a rehearsal of N ranks on one
    card); with enough cards it raises, since a shared card would silently halve
    both ranks' rate in a scaling run."""
    world = len(bus_ids)
    shared = len(set(bus_ids)) < world
    if shared and device_count >= world:
        dup = sorted({b for b in bus_ids if bus_ids.count(b) > 1})
        raise RuntimeError(f"{world} ranks on {device_count} visible devices, but ranks share {dup}: "
                           "check LOCAL_RANK / HIP_VISIBLE_DEVICES")
    return shared


def even_split(n: int, world: int, rank: int) -> tuple[int, int]:
    """(first, count) of rank's contiguous share of n datagrams; counts differ by <= 1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    q, r = divmod(n, world)
    first = rank * q + min(rank, r)
    return first, q + (1 if rank < r else 0)


def byte_balanced_split(lengths: np.ndarray, world: int, rank: int) -> tuple[int, int]:
    """(first, count) splitting a ragged batch so each rank gets ~equal traffic.

    Datagram k weighs lengths[k] + 8 (its bytes plus the salt), and boundary j
    sits at the first datagram whose exclusive weight prefix reaches j/world of
    the total ("split by cumulative bytes").  Same rule as the C ABI's
    hyobfs_shard_bounds (include/hyobfs.h).
    """
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    lengths = np.asarray(lengths, dtype=np.uint64)
    n = lengths.size
    if n == 0:
        return 0, 0
    excl = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lengths + np.uint64(8), out=excl[1:])
    total = int(excl[-1])

    def cut(k: int) -> int:
        if k <= 0:
            return 0
        if k >= world:
            return n
        return int(np.searchsorted(excl[:-1], total * k // world, side="left"))

    a, b = cut(rank), cut(rank + 1)
    return a, b - a


def shard_bounds(lengths, n: int, world: int) -> list[int]:
    """bounds[0..world] of every rank's range, from the C ABI (hyobfs_shard_bounds).

    lengths=None: a uniform batch (split by count).  Host-only call, no device."""
    import ctypes

    from . import _lib
    out = (ctypes.c_uint64 * (world + 1))()
    if lengths is None:
        ptr = None
    else:
        arr = np.ascontiguousarray(lengths, dtype=np.uint32)
        ptr = arr.ctypes.data
    _lib.check(_lib.load().hyobfs_shard_bounds(ptr, n, world, out), "shard_bounds")
    return list(out)


def weak_shard(per_rank: int, rank: int) -> tuple[int, int]:
    """Weak scaling: rank r owns datagrams [r*per_rank, (r+1)*per_rank) of the global batch."""
    return rank * per_rank, per_rank
