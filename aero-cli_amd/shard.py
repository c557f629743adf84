"""Channel sharding across GPUs.

VFO channels are independent streams: every rank owns a disjoint channel
set and runs the whole decode path for it; the only inter-rank traffic is
the benchmark's barrier and its max/sum timing reduction.
"""
import numpy as np


def shard_channels(n_channels, world, rank, costs=None):
    """Balanced contiguous shard of channel ids for `rank`.  `costs` (per
    channel, e.g. 5.6 for 10500 bps vs 1.0 for 600 bps, §8(e)) balances by
    load instead of count."""
    if costs is None:
        base, extra = divmod(n_channels, world)
        lo = rank * base + min(rank, extra)
        return np.arange(lo, lo + base + (1 if rank < extra else 0))
    costs = np.asarray(costs, dtype=np.float64)
    cum = np.concatenate([[0.0], np.cumsum(costs)])
    edges = np.searchsorted(cum, np.linspace(0, cum[-1], world + 1), side='left')
    edges[0], edges[-1] = 0, n_channels
    return np.arange(edges[rank], edges[rank + 1])


def channel_offsets(n_channels, pool, rank=0):
    """Start offset (samples) of each channel group g = c // pool in the
    synthetic stream pool, so no two channels see the same sample window."""
    groups = max(1, n_channels // pool)
    g = np.arange(groups, dtype=np.int64)
    return ((g * 7919 + rank * 104729) % 65536).astype(np.int64)
