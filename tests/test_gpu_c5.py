"""C5 at its configured size on one GPU: a generated
1.536 Msps SDRReceiver INI with 3 main VFOs and 64 [vfos] (6 x 10500,
29 x 600 / 1200 alternating), synthetic Aero signals in every VFO, through
the GPU channeliser (aero_chan.h) straight into the GPU decoder
(aero_chan_feed) -- against the oracle publisher's audio decoded by one
oracle decoder per VFO (publish/vfo.cpp:154-258 -> decode/decode.cpp:168-241):
every VFO's int16 audio, soft bits, coarse-estimator hops (f64 bitwise) and
ACARS items identical."""
import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu

SECONDS = 8.0


def test_c5_64_vfos_channeliser_to_decoder(engine_lib, cpu_libs):
    import aero_engine as ae
    cfg = tl.c5_config()
    assert len(cfg['vfos']) == 64 and len(cfg['mains']) == 3
    x = tl.c5_wideband(cfg, SECONDS)
    ref = tl.OraclePublisher(cfg['sample_rate'], cfg['center_frequency'], cfg['mains'], cfg['vfos'])
    B = ref.block_len
    nblk = len(x) // B
    ref.process(x[:nblk * B])
    ch = ae.Channeliser(cfg['sample_rate'], cfg['center_frequency'], cfg['mains'], cfg['vfos'], max_blocks=2,
                        host_out=True)
    assert ch.block_len == B
    eng = ae.Engine(max_channels=64, flags=ae.F_TRACE_HOPS | ae.F_TRACE_SOFT)
    chans = [eng.open_channel(ae.vfo_bitrate(v['data_rate'])) for v in cfg['vfos']]
    for b in range(nblk):
        ch.push(x[b * B:(b + 1) * B])
        ch.run()
        ch.feed(eng, chans)
        eng.run()
    eng.flush()
    ch.sync()
    items_total = 0
    for v, vf in enumerate(cfg['vfos']):
        audio = ref.usb(v)
        got = ch.audio(v)
        assert np.array_equal(audio, got), 'vfo %d audio' % v
        o = tl.Oracle(bitrate=ae.vfo_bitrate(vf['data_rate']))
        o.push_chunked(audio, ch.vfo_info(v)['samples_per_block'])
        h, rh = eng.hops(chans[v]), o.hops()
        assert len(h) == len(rh) > 0, v
        assert np.array_equal(h.view(np.int64), rh.view(np.int64)), 'vfo %d hops' % v
        sb = eng.softbits(chans[v])
        assert len(sb) > 0 and np.array_equal(sb, o.softbits()), 'vfo %d soft bits' % v
        want = o.item_lines('A')
        assert eng.items(chans[v]) == want, 'vfo %d items' % v
        items_total += len(want)
    assert items_total > 30
    eng.close()
    ch.close()
