"""Parity at the bench's scale (BENCH config C2: 65,536 continuous 10500-bps
OQPSK channels in one engine, lockstep device batch pushes of one 4096-sample
hop per step, the same synthetic pool and channel offsets as bench.py).

At this size the per-channel rings are indexed past 2^31 elements (the AGC
ring alone is 192000 x 65536 doubles) and every kernel runs with its full
grid, so a sample of channels spread over the whole batch (the first, every
2048th + k, the last) is compared with the oracle decoding the same sample
window: soft bits, coarse-hop records (f64 bitwise), CRC-checked frames and
ACARS items.  Traces are kept for the sampled channels only
(aero_trace_select).  Reference: OqpskDemodulator::writeData
(decode/oqpskdemodulator.cpp:284-560) and the AeroL path after it.

The kernels' libm is glibc 2.35's, restated instruction for instruction
(aero_math.h: __atan2_fma, __log_fma, sincos, hypot, tanh; bitwise in
test_math_host.py), so every output is held bit for bit to the glibc
oracle, the f64 hop records (frequency, MSE averages) included."""
import concurrent.futures as cf
import os
import sys

import numpy as np
import pytest

import aero_testlib as tl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

C, P, HOP, HOPS = 65536, 64, 4096, 64


def _pool(length):
    import bench
    M = bench.MODES['oqpsk10500']
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        return np.stack(list(ex.map(lambda k: bench.synth_one(M, length / 48000.0, 0xAE20 + k, k), range(P))))


def _oracle(pcm):
    o = tl.Oracle()
    o.push_chunked(pcm, HOP)
    return o.softbits(), o.hops(), o.frames(), o.item_lines('A')


@pytest.mark.gpu
def test_fullscale_sample_matches_oracle(engine_lib):
    import torch
    import aero_engine as ae
    import shard
    offsets = shard.channel_offsets(C, P)
    span = HOPS * HOP
    pool_host = _pool(span + int(offsets.max()) + 1)
    sel = [2048 * k + k for k in range(32)] + [C - 1]
    keep = set(sel)
    eng = ae.Engine(max_channels=C, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    for _ in range(C):
        eng.open_channel(10500, 48000)
    eng.trace_select(sel)
    pool = torch.from_numpy(pool_host).to('cuda')
    items = {c: [] for c in sel}
    for s in range(HOPS):
        views = [pool[:, int(o) + s * HOP:int(o) + (s + 1) * HOP] for o in offsets]
        x = torch.stack(views).permute(2, 0, 1).reshape(HOP, C).contiguous()
        torch.cuda.synchronize()
        eng.push_batch_device(x.data_ptr(), HOP, C, C)
        eng.run()
        for c, line in eng.drain_items(lines=True, keep=keep):
            items[c].append(line)
    eng.flush()
    for c, line in eng.drain_items(lines=True, keep=keep):
        items[c].append(line)
    total = eng.stat('frames')
    got = {c: (eng.softbits(c), eng.hops(c), eng.frames(c)) for c in sel}
    eng.close()
    wins = {c: pool_host[c % P, int(offsets[c // P]):int(offsets[c // P]) + span] for c in sel}
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        refs = dict(zip(sel, ex.map(lambda c: _oracle(wins[c]), sel)))
    assert total > C, 'the batch decoded %d frames' % total
    for c in sel:
        sb, hops, frames = got[c]
        rsb, rhops, rframes, ritems = refs[c]
        assert len(rsb) > 1000, 'oracle did not lock on channel %d' % c
        assert np.array_equal(sb, rsb), 'channel %d soft bits differ (%d vs %d)' % (c, len(sb), len(rsb))
        assert hops.shape == rhops.shape and np.array_equal(hops.view(np.int64), rhops.view(np.int64)), \
            'channel %d hop records differ' % c
        assert np.array_equal(frames, rframes), 'channel %d frames differ' % c
        assert ritems and items[c] == ritems, 'channel %d ACARS items differ' % c
