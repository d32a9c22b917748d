"""Byte-balanced sharding of packet batches across GPUs.

Packets are independent, so the multi-GPU path is a partition with no
collective: rank r gets one contiguous range of packets, chosen so that every
rank sums about the same number of bytes (a mixed-MTU batch balanced by count
would leave the rank holding the 9000 B packets last).  Used by bench.py and
covered by tests/test_dist.py with a gloo world.
"""
from __future__ import annotations

import numpy as np


def shard_ranges(lengths, world: int) -> list[tuple[int, int]]:
    """Split packets [0, n) into `world` contiguous ranges of near-equal byte
    totals.  `lengths` is an int array, or an int n for uniform packets."""
    if world < 1:
        raise ValueError("world must be >= 1")
    if isinstance(lengths, (int, np.integer)):
        n = int(lengths)
        cuts = [n * r // world for r in range(world + 1)]
        return [(cuts[r], cuts[r + 1]) for r in range(world)]
    lens = np.asarray(lengths, dtype=np.int64)
    n = lens.size
    if n == 0:
        return [(0, 0)] * world
    csum = np.cumsum(lens)
    total = int(csum[-1])
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        # first packet index whose inclusive prefix reaches the target
        cut = int(np.searchsorted(csum, target, side="left")) + 1
        cuts.append(min(max(cut, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard_bytes(lengths, ranges) -> list[int]:
    if isinstance(lengths, (int, np.integer)):
        raise TypeError("needs per-packet lengths")
    lens = np.asarray(lengths, dtype=np.int64)
    return [int(lens[a:b].sum()) for a, b in ranges]
