"""Burst-mode 600/1200-bps MSK on the GPU (aero-cli_amd/csrc/burst_msk.hip +
burst_engine.hip) against the oracle restatement of BurstMskDemodulator + the
AeroL MSK burst branch with updateMSK (oracle/aero_oracle.cpp): delivered soft
bits with their start-of-burst markers, trident-check records (f64,
bit-exact), every R/T test result, every decoded packet and the ACARS items
must be identical."""
import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu


def _engine_vs_oracle(streams, bitrates, chunks):
    import aero_engine as ae
    eng = ae.Engine(max_channels=len(streams), flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    chans = [eng.open_channel(br, 48000, burst=True) for br in bitrates]
    refs = []
    for pcm, br, chunk in zip(streams, bitrates, chunks):
        o = tl.Oracle(bitrate=br, burst=True)
        o.push_chunked(pcm, chunk)
        refs.append(o)
    pos = [0] * len(streams)
    while any(p < len(s) for p, s in zip(pos, streams)):
        for k, (pcm, chunk) in enumerate(zip(streams, chunks)):
            if pos[k] < len(pcm):
                eng.push(chans[k], pcm[pos[k]:pos[k] + chunk])
                pos[k] += chunk
        eng.run()
    eng.flush()
    return eng, chans, refs


def _check(eng, ch, o):
    h, rh = eng.hops(ch), o.hops()
    assert len(rh) > 0 and np.sum(rh[:, 1] == 1) > 0
    assert len(h) == len(rh), (len(h), len(rh))
    assert np.array_equal(h.view(np.int64), rh.view(np.int64))
    s, rs = eng.softbits16(ch), o.softbits16()
    assert len(rs) > 1000
    assert len(s) == len(rs), (len(s), len(rs))
    assert np.array_equal(s, rs), np.nonzero(s != rs)[0][:10]
    assert np.array_equal(eng.rt_tests(ch), o.rt_tests())
    assert eng.rt_packets(ch) == o.rt_packets()
    items = eng.items(ch)
    assert items == o.item_lines('A')


@pytest.mark.parametrize('bitrate,seed,chunk', [(1200, 31, 12000), (600, 32, 3000)])
def test_burst_msk_matches_oracle(bitrate, seed, chunk):
    pcm = tl.synth_burst_msk(seconds=20.0, bitrate=bitrate, seed=seed, carrier=2500.0, ebn0=13.0)
    eng, (ch,), (o,) = _engine_vs_oracle([pcm], [bitrate], [chunk])
    _check(eng, ch, o)  # pops the engine's items
    assert len(o.rt_packets()) >= 3 and o.item_lines('A')
    eng.close()


def test_burst_msk_mixed_rates_many_channels():
    """six MSK burst VFOs, both bit rates, different carriers, noise and message
    sizes, interleaved in one engine; each equals its own oracle"""
    brs = [600, 1200, 1200, 600, 1200, 600]
    streams = [tl.synth_burst_msk(seconds=12.0, bitrate=br, seed=40 + k, carrier=1500.0 + 700.0 * k,
                                  ebn0=12.0 + k % 3) for k, br in enumerate(brs)]
    chunks = [12000, 4800, 9600, 2000, 16384, 7000]
    eng, chans, refs = _engine_vs_oracle(streams, brs, chunks)
    for ch, o in zip(chans, refs):
        _check(eng, ch, o)
    eng.close()


def test_burst_msk_batch_push_device():
    """aero_push_pcm_batch on MSK burst channels from a device buffer"""
    import aero_engine as ae
    import torch
    n, chunk = 4, 12000
    streams = [tl.synth_burst_msk(seconds=10.0, bitrate=1200, seed=60 + k, carrier=2000.0 + 400.0 * k, ebn0=14.0)
               for k in range(n)]
    L = min(len(s) for s in streams) // chunk * chunk
    x = np.stack([s[:L] for s in streams], axis=1)
    eng = ae.Engine(max_channels=n, flags=ae.F_TRACE_SOFT | ae.F_TRACE_FRAMES)
    chans = [eng.open_channel(1200, 48000, burst=True) for _ in range(n)]
    xd = torch.from_numpy(x).to('cuda')
    torch.cuda.synchronize()
    for t in range(0, L, chunk):
        eng.push_batch_device(xd[t:].data_ptr(), chunk, n, n)
        eng.run()
    eng.flush()
    for k in range(n):
        o = tl.Oracle(bitrate=1200, burst=True)
        o.push_chunked(streams[k][:L], chunk)
        assert np.array_equal(eng.softbits16(chans[k]), o.softbits16()), k
        assert eng.rt_packets(chans[k]) == o.rt_packets(), k
        assert eng.items(chans[k]) == o.item_lines('A'), k
    eng.close()


def test_burst_msk_open_rules():
    """burst MSK accepts the audio at any labelled rate (the demodulator is set
    for 48 kHz, decode/decode.cpp:123-132); other burst bit rates are refused"""
    import aero_engine as ae
    eng = ae.Engine(max_channels=4)
    eng.open_channel(600, 12000, burst=True)
    eng.open_channel(1200, 24000, burst=True)
    with pytest.raises(Exception):
        eng.open_channel(8400, 48000, burst=True)
    eng.close()
