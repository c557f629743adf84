"""Multi-rank path on CPU (gloo, world_size 2): disjoint channel shards that
cover every channel, and the bench's max-over-ranks / sum-over-ranks timing
reduction."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import aero_testlib  # noqa: F401
import shard


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    mine = shard.shard_channels(n, world, rank)
    lens = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(lens, torch.tensor([len(mine)]))
    m = int(max(l.item() for l in lens))  # gloo all_gather needs equal sizes: pad with -1
    padded = torch.full((m,), -1, dtype=torch.int64)
    padded[:len(mine)] = torch.from_numpy(mine.astype(np.int64))
    chunks = [torch.zeros(m, dtype=torch.int64) for _ in lens]
    dist.all_gather(chunks, padded)
    t = torch.tensor([1.0 + rank, 100.0 * (rank + 1)], dtype=torch.float64)
    tmax = t.clone()
    dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
    dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
    if rank == 0:
        q.put(([v for v in torch.cat(chunks).tolist() if v >= 0], float(tmax[0]), float(t[1])))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_and_reduction():
    n, world = 1001, 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    allc, tmax, tsum = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(allc) == list(range(n))
    assert tmax == 2.0 and tsum == 300.0


def test_cost_balanced_shards():
    costs = np.array([5.6] * 10 + [1.0] * 30)  # 10500 bps vs 600 bps channels
    parts = [shard.shard_channels(40, 4, r, costs) for r in range(4)]
    assert sorted(np.concatenate(parts).tolist()) == list(range(40))
    loads = [costs[p].sum() for p in parts]
    assert max(loads) - min(loads) <= 5.6


def test_channel_offsets_distinct():
    off = shard.channel_offsets(32768, 64)
    assert len(np.unique(off)) == len(off)
