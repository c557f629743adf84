"""C5 split across ranks on the GPU (bench.py --mode c5
--gpus N): rank 0 holds the 1.536 Msps wideband and broadcasts every 0.25 s
read (shard.broadcast_reads, the path's one exchange step; gloo here, RCCL
over xGMI on a node); every rank channelises the read with the VFOs it does
not own skipped (aero_chan skip masks) and decodes only the VFOs
shard.shard_vfos gives it.  Two ranks share the card.  The union over all 64
VFOs of audio, soft bits, coarse hops (f64 bitwise) and ACARS items equals
the oracle publisher's audio through one oracle decoder per VFO
(publish/publisher.cpp:285-306, publish/vfo.cpp:154-258,
decode/decode.cpp:168-241)."""
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

SECONDS = 8.0


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import aero_engine as ae
    cfg = tl.c5_config()
    owner = shard.shard_vfos(cfg['vfos'], world)
    mine = [v for v in range(len(cfg['vfos'])) if owner[v] == rank]
    ch = ae.Channeliser(cfg['sample_rate'], cfg['center_frequency'], cfg['mains'], cfg['vfos'], max_blocks=2,
                        host_out=True, skip=[owner[v] != rank for v in range(len(cfg['vfos']))])
    B = ch.block_len
    nblk = int(cfg['sample_rate'] * SECONDS) // B
    x = tl.c5_wideband(cfg, SECONDS) if rank == 0 else None
    eng = ae.Engine(max_channels=max(1, len(mine)), flags=ae.F_TRACE_HOPS | ae.F_TRACE_SOFT)
    chans = [eng.open_channel(ae.vfo_bitrate(cfg['vfos'][v]['data_rate'])) if owner[v] == rank else -1
             for v in range(len(cfg['vfos']))]
    rd = torch.empty(B * 2, dtype=torch.float32)
    for b in range(nblk):
        if rank == 0:
            rd.copy_(torch.from_numpy(x[b * B:(b + 1) * B].astype(np.complex64).view(np.float32)))
        shard.broadcast_reads(rd)
        ch.push(rd.numpy().view(np.complex64))
        ch.run()
        ch.feed(eng, chans)
        eng.run()
    eng.flush()
    ch.sync()
    res = {}
    for v in mine:
        res[v] = (_digest(ch.audio(v)), _digest(eng.softbits(chans[v])), _digest(eng.hops(chans[v]).view(np.int64)),
                  eng.items(chans[v]))
    eng.close()
    ch.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, (rank, res))
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_c5_two_ranks_vfo_split_equals_oracle(cpu_libs):
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    import aero_engine as ae
    cfg = tl.c5_config()
    owner = shard.shard_vfos(cfg['vfos'], world)
    merged = {}
    for rank, res in gathered:
        assert sorted(res) == [v for v in range(len(cfg['vfos'])) if owner[v] == rank]
        merged.update(res)
    assert sorted(merged) == list(range(len(cfg['vfos'])))
    assert len(set(owner)) == world
    x = tl.c5_wideband(cfg, SECONDS)
    ref = tl.OraclePublisher(cfg['sample_rate'], cfg['center_frequency'], cfg['mains'], cfg['vfos'])
    nb = int(cfg['sample_rate'] * SECONDS) // ref.block_len
    ref.process(x[:nb * ref.block_len])
    n_items = 0
    for v, vf in enumerate(cfg['vfos']):
        audio = ref.usb(v)
        o = tl.Oracle(bitrate=ae.vfo_bitrate(vf['data_rate']))
        o.push_chunked(audio, ref.info(v)['samples_per_block'])
        a, s, h, items = merged[v]
        assert a == _digest(audio), 'vfo %d audio' % v
        assert s == _digest(o.softbits()), 'vfo %d soft bits' % v
        assert h == _digest(o.hops().view(np.int64)), 'vfo %d hops' % v
        assert items == o.item_lines('A'), 'vfo %d items' % v
        n_items += len(items)
    assert n_items > 30
