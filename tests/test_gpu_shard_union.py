"""Multi-rank decode on the GPU: two ranks (processes, one
engine each, gloo for the gather) decode disjoint shard_channels() shards of
the same channel set on the card; the union of their per-channel ACARS items
and soft-bit digests equals the oracle's for every channel, i.e. sharding
changes nothing about any channel's output (bench.py --gpus N runs exactly
this split, one rank per GPU)."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import aero_testlib as tl
import shard

pytestmark = pytest.mark.gpu

N_CH, SECONDS, CHUNK = 6, 7.0, 4096


def _stream(c):
    return tl.synth(seconds=SECONDS, seed=0xAE90 + c, carrier=12000.0 + 7.5 * c, ebn0=12.0, phase0=0.2 * c)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import aero_engine as ae
    mine = [int(c) for c in shard.shard_channels(N_CH, world, rank)]
    pcm = np.stack([_stream(c) for c in mine], axis=1)  # time-major [n][len(mine)]
    eng = ae.Engine(max_channels=len(mine), flags=ae.F_TRACE_SOFT)
    chans = [eng.open_channel(10500, 48000) for _ in mine]
    for i in range(0, pcm.shape[0], CHUNK):
        eng.push_batch(pcm[i:i + CHUNK])
        eng.run()
    eng.flush()
    res = {c: (eng.items(ch), hashlib.sha256(eng.softbits(ch).tobytes()).hexdigest()) for c, ch in zip(mine, chans)}
    eng.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, res)
    if rank == 0:
        merged = {}
        for part in gathered:
            merged.update(part)
        q.put(merged)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_union_equals_oracle():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    merged = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(merged) == list(range(N_CH))
    n_items = 0
    for c in range(N_CH):
        o = tl.Oracle()
        o.push_chunked(_stream(c), 12000)
        items, digest = merged[c]
        assert digest == hashlib.sha256(o.softbits().tobytes()).hexdigest(), c
        assert items == o.item_lines('A'), c
        n_items += len(items)
    assert n_items > 0
