"""GPU channeliser (aero-cli_amd/csrc/chan.hip) against the oracle
restatement of aero-publish (oracle/pub_oracle.cpp): every sub-VFO's int16
audio and every main VFO's 4-bit IQ bit-exact (int16 / int8 work), across
batch boundaries (max_blocks smaller than the pushed reads, so FIR and
half-band histories cross both in-batch and between-batch read boundaries),
with DC removal, late 1/5 and 1/6 decimation, the audio low-pass, int16
wrap-around and device-pointer pushes; then the audio goes straight into the
decoder (aero_chan_feed) and the decoder's coarse-estimator hops equal the
oracle decoder's on the oracle channeliser's audio."""
import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu

C = tl.CENTER


def _run_pair(name, nblk, max_blocks, dcc=False, device_push=False):
    import aero_engine as ae
    cfg = tl.PUB_CONFIGS[name]
    fs = cfg['sample_rate']
    ref = tl.OraclePublisher(fs, C, cfg['mains'], cfg['vfos'], correct_dc_bias=dcc)
    x = tl.wideband(fs, nblk * ref.block_len, 0xC5 + nblk, cfg['tones'])
    ref.process(x)
    ch = ae.Channeliser(fs, C, cfg['mains'], cfg['vfos'], correct_dc_bias=dcc, max_blocks=max_blocks, host_out=True)
    assert ch.block_len == ref.block_len
    if device_push:
        import torch
        t = torch.from_numpy(x.view(np.float32)).to('cuda')
        torch.cuda.synchronize()
        for b in range(nblk):
            ch.push_device(t.data_ptr() + b * ref.block_len * 8, 1)
    else:
        for b in range(nblk):
            ch.push(x[b * ref.block_len:(b + 1) * ref.block_len])
    ch.run()
    ch.sync()
    return cfg, ref, ch


@pytest.mark.parametrize('name,nblk,max_blocks,dcc', [('r1536k', 5, 2, False), ('r288k', 7, 3, True),
                                                      ('r1920k', 4, 4, False), ('r288k', 3, 1, False)])
def test_channeliser_bit_exact(name, nblk, max_blocks, dcc):
    cfg, ref, ch = _run_pair(name, nblk, max_blocks, dcc)
    for v in range(len(cfg['vfos'])):
        want, got = ref.usb(v), ch.audio(v)
        info = ch.vfo_info(v)
        assert info['out_rate'] == ref.info(v)['out_rate'] and info['late'] == ref.info(v)['late']
        assert len(want) == nblk * info['samples_per_block'] and len(got) == len(want)
        assert np.count_nonzero(want) > len(want) // 2
        bad = np.flatnonzero(want != got)
        assert bad.size == 0, 'vfo %d: %d mismatches, first at %d (%d vs %d)' % (
            v, bad.size, bad[0], want[bad[0]], got[bad[0]])
    for m, d in enumerate(cfg['mains']):
        want, got = ref.iq(m), ch.iq(m)
        assert np.array_equal(want, got), 'main %d IQ' % m
        if d.get('publish'):
            assert len(want) > 0
    ch.close()


def test_channeliser_device_push():
    cfg, ref, ch = _run_pair('r1536k', 3, 3, device_push=True)
    for v in range(len(cfg['vfos'])):
        assert np.array_equal(ref.usb(v), ch.audio(v))
    ch.close()


def test_channeliser_feeds_decoder():
    """Wideband -> channeliser -> decoder on the GPU without leaving HBM,
    against oracle channeliser -> oracle decoder (C5 chain)."""
    import aero_engine as ae
    cfg = tl.PUB_CONFIGS['r288k']
    fs = cfg['sample_rate']
    nblk = 10
    ref = tl.OraclePublisher(fs, C, cfg['mains'], cfg['vfos'])
    x = tl.wideband(fs, nblk * ref.block_len, 0xC55, cfg['tones'])
    ch = ae.Channeliser(fs, C, cfg['mains'], cfg['vfos'], max_blocks=2)
    eng = ae.Engine(max_channels=4, flags=ae.F_TRACE_HOPS | ae.F_TRACE_SOFT)
    chans = [eng.open_channel(ae.vfo_bitrate(v['data_rate'])) for v in cfg['vfos']]
    oracles = [tl.Oracle(bitrate=ae.vfo_bitrate(v['data_rate'])) for v in cfg['vfos']]
    for b in range(nblk):
        blk = x[b * ref.block_len:(b + 1) * ref.block_len]
        ref.process(blk)
        ch.push(blk)
        ch.run()
        ch.feed(eng, chans)
        eng.run()
    eng.flush()
    for v, o in enumerate(oracles):
        o.push_chunked(ref.usb(v), ch.vfo_info(v)['samples_per_block'])
        h, rh = eng.hops(chans[v]), o.hops()
        assert len(h) == len(rh) > 0
        assert np.array_equal(h.view(np.int64), rh.view(np.int64))
        assert np.array_equal(eng.softbits(chans[v]), o.softbits())
    eng.close()
    ch.close()
