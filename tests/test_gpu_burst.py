"""Burst-mode 10500-bps OQPSK on the GPU (aero-cli_amd/csrc/burst.hip +
burst_engine.hip) against the oracle restatement of BurstOqpskDemodulator +
the AeroL R/T branch (oracle/aero_oracle.cpp), pushed with the same message
chunking (burst output depends on message boundaries through lastmse,
decode/burstoqpskdemodulator.cpp:264, 685): delivered soft bits with their
start-of-packet markers, trident-check records (f64, bit-exact), every R/T
test result, every decoded packet and the ACARS items must be identical."""
import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu


def _engine_vs_oracle(streams, chunks):
    import aero_engine as ae
    eng = ae.Engine(max_channels=len(streams), flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    chans = [eng.open_channel(10500, 48000, burst=True) for _ in streams]
    refs = []
    for pcm, chunk in zip(streams, chunks):
        o = tl.Oracle(burst=True)
        o.push_chunked(pcm, chunk)
        refs.append(o)
    # interleave the channels' messages as a multi-VFO host would
    pos = [0] * len(streams)
    while any(p < len(s) for p, s in zip(pos, streams)):
        for k, (pcm, chunk) in enumerate(zip(streams, chunks)):
            if pos[k] < len(pcm):
                eng.push(chans[k], pcm[pos[k]:pos[k] + chunk])
                pos[k] += chunk
        eng.run()
    eng.flush()
    return eng, chans, refs


@pytest.mark.parametrize('seed,chunk', [(2, 12000), (5, 3000)])
def test_burst_matches_oracle(seed, chunk):
    pcm = tl.synth_burst(seconds=20.0, seed=seed, carrier=12000.0, ebn0=14.0)
    eng, (ch,), (o,) = _engine_vs_oracle([pcm], [chunk])
    h, rh = eng.hops(ch), o.hops()
    assert len(rh) > 0 and np.sum(rh[:, 1] == 1.0) > 0
    assert len(h) == len(rh), (len(h), len(rh))
    assert np.array_equal(h.view(np.int64), rh.view(np.int64))
    s, rs = eng.softbits16(ch), o.softbits16()
    assert len(rs) > 1000
    assert np.array_equal(s, rs)
    assert np.array_equal(eng.rt_tests(ch), o.rt_tests())
    pk, rpk = eng.rt_packets(ch), o.rt_packets()
    assert len(rpk) >= 3 and pk == rpk
    items = eng.items(ch)
    assert items == o.item_lines('A') and items
    eng.close()


def test_burst_many_channels_mixed_chunking():
    """Four burst VFOs with different seeds, carriers and message sizes in one
    engine, interleaved; each equals its own oracle."""
    streams = [tl.synth_burst(seconds=12.0, seed=10 + k, carrier=12000.0 + 300.0 * k, ebn0=14.0) for k in range(4)]
    chunks = [12000, 4800, 9600, 2000]
    eng, chans, refs = _engine_vs_oracle(streams, chunks)
    for ch, o in zip(chans, refs):
        assert np.array_equal(eng.softbits16(ch), o.softbits16())
        assert np.array_equal(eng.hops(ch).view(np.int64), o.hops().view(np.int64))
        assert eng.rt_packets(ch) == o.rt_packets()
        assert eng.items(ch) == o.item_lines('A')
    eng.close()


def test_burst_batch_push_equals_oracle():
    """aero_push_pcm_batch on burst channels: one message per channel per
    batch (host and device pointers), each channel equal to its oracle fed
    the same message boundaries."""
    import aero_engine as ae
    import torch
    n, chunk = 6, 12000
    streams = [tl.synth_burst(seconds=10.0, seed=40 + k, carrier=11800.0 + 150.0 * k, ebn0=14.0) for k in range(n)]
    L = min(len(s) for s in streams) // chunk * chunk
    x = np.stack([s[:L] for s in streams], axis=1)  # time-major [L][n]
    eng = ae.Engine(max_channels=n, flags=ae.F_TRACE_SOFT | ae.F_TRACE_FRAMES)
    chans = [eng.open_channel(10500, 48000, burst=True) for _ in range(n)]
    assert chans == list(range(n))
    xd = torch.from_numpy(x).to('cuda')
    torch.cuda.synchronize()
    for k, t in enumerate(range(0, L, chunk)):
        if k % 2:
            eng.push_batch(x[t:t + chunk])
        else:
            eng.push_batch_device(xd[t:].data_ptr(), chunk, n, n)
        eng.run()
    eng.flush()
    for k in range(n):
        o = tl.Oracle(burst=True)
        o.push_chunked(streams[k][:L], chunk)
        assert np.array_equal(eng.softbits16(chans[k]), o.softbits16()), k
        assert eng.rt_packets(chans[k]) == o.rt_packets(), k
        assert eng.items(chans[k]) == o.item_lines('A'), k
    eng.close()
