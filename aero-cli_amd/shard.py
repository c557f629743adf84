"""Channel sharding across GPUs.

VFO channels are independent streams: every rank owns a disjoint channel
set and runs the whole decode path for it.  For the C5 channeliser the one
exchange step is the broadcast of each wideband read from the rank that
received it (RCCL over xGMI); every rank then channelises and decodes only
its own [vfos] entries (shard_vfos).
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


# decode cost per VFO by bit rate (a 10500 channel costs
# about 5.6x a 600/1200 one on the CPU probe)
VFO_COST = {600: 1.0, 1200: 1.0}


def shard_vfos(vfos, world):
    """Owner rank of every [vfos] entry: longest-processing-time-first over
    the per-VFO decode cost, ties by index, so every rank derives the same map."""
    costs = [VFO_COST.get(int(v.get('data_rate', 0)), 5.6) for v in vfos]
    load = [0.0] * world
    owner = [0] * len(vfos)
    for i in sorted(range(len(vfos)), key=lambda i: (-costs[i], i)):
        r = min(range(world), key=lambda r: (load[r], r))
        owner[i] = r
        load[r] += costs[i]
    return owner


def broadcast_reads(buf, src=0):
    """The C5 exchange step: the wideband reads in `buf` (a CUDA tensor on
    the NCCL/RCCL backend, a CPU tensor on gloo) go from rank `src` to all
    (under a one-rank group too, so that `bench.py --dist` runs the call)."""
    import torch.distributed as dist
    if dist.is_initialized():
        dist.broadcast(buf, src=src)
    return buf
