"""C5 multi-GPU shape on CPU (gloo, world_size 2): every wideband read is
broadcast from rank 0 (the RCCL broadcast of SURVEY.md §8(e)), all ranks see
identical samples, and the [vfos] entries are split by decode cost so each is
channelised and decoded on exactly one rank."""
import hashlib
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import aero_testlib as tl
import shard


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _vfos():
    rates = [10500, 600, 1200, 600] * 16
    return [dict(frequency=tl.CENTER + 5000 * k, data_rate=r, gain=100.0) for k, r in enumerate(rates)]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    owner = shard.shard_vfos(_vfos(), world)
    buf = torch.zeros(2 * 57600 * 2, dtype=torch.float32)
    if rank == 0:
        x = tl.wideband(288000, 2 * 57600, 11, [(1000.0, 0.2)])
        buf.copy_(torch.from_numpy(x.view(np.float32)))
    shard.broadcast_reads(buf, src=0)
    digest = hashlib.sha256(buf.numpy().tobytes()).hexdigest()
    out = [None] * world
    dist.all_gather_object(out, (rank, digest, owner))
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_and_vfo_shards():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    x = tl.wideband(288000, 2 * 57600, 11, [(1000.0, 0.2)])
    want = hashlib.sha256(x.view(np.float32).tobytes()).hexdigest()
    assert all(d == want for _, d, _ in res)
    owners = [o for _, _, o in res]
    assert owners[0] == owners[1]  # every rank derives the same map


def test_vfo_shards_balanced():
    vfos = _vfos()
    for world in (2, 4, 8):
        owner = shard.shard_vfos(vfos, world)
        assert sorted(set(owner)) == list(range(world))
        cost = [shard.VFO_COST.get(v['data_rate'], 5.6) for v in vfos]
        loads = [sum(c for c, o in zip(cost, owner) if o == r) for r in range(world)]
        assert max(loads) - min(loads) <= 5.6
