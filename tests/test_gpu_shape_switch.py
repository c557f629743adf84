"""A live group that changes demodulator shape between launches.

The continuous OQPSK and MSK groups run the few-channel kernels (16 lanes
per channel) while the group holds at most AERO_OQPSK_WIDE / AERO_MSK_WIDE
channels, and the one-lane kernels (OQPSK: chain + FIR helper waves) above
that (engine.hip run_pass).  Opening one more channel therefore switches the
kernels in the middle of the other channels' streams.  Both shapes keep the
same state layout and operation order, so the switch must not change a bit:
with the threshold at 2, two channels stream, a third opens mid-stream, and
every channel's soft bits, hop records, frames and items equal the oracle's
(decode/oqpskdemodulator.cpp:284-620, decode/mskdemodulator.cpp:252-469)."""
import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu


def _run_switch(ae, streams, opens, chunk, bitrate, flags):
    eng = ae.Engine(max_channels=4, flags=flags)
    chans = [None] * len(streams)
    pos = [0] * len(streams)
    k = 0
    while any(c is None or pos[i] < len(streams[i]) for i, c in enumerate(chans)):
        for i, s in enumerate(streams):
            if chans[i] is None and k >= opens[i]:
                chans[i] = eng.open_channel(bitrate)
            if chans[i] is not None and pos[i] < len(s):
                eng.push(chans[i], s[pos[i]:pos[i] + chunk])
                pos[i] += chunk
        eng.run()
        k += 1
    eng.flush()
    return eng, chans


def _check(eng, chans, streams, chunk, oracle_kw):
    for i, (s, ch) in enumerate(zip(streams, chans)):
        o = tl.Oracle(**oracle_kw)
        o.push_chunked(s, chunk)
        sb = eng.softbits(ch)
        assert len(sb) > 1000 and np.array_equal(sb, o.softbits()), 'channel %d soft bits differ' % i
        h, rh = eng.hops(ch), o.hops()
        assert h.shape == rh.shape and np.array_equal(h.view(np.int64), rh.view(np.int64)), \
            'channel %d hop records differ' % i
        assert np.array_equal(eng.frames(ch), o.frames()), 'channel %d frames differ' % i
        items = eng.items(ch)
        assert items and items == o.item_lines('A'), 'channel %d items differ' % i


def test_oqpsk_group_switches_shape_mid_stream(engine_lib, monkeypatch):
    import aero_engine as ae
    monkeypatch.setenv('AERO_OQPSK_WIDE', '2')
    streams = [tl.synth(seconds=12.0, seed=0x5100 + i, carrier=f, ebn0=12.0)
               for i, f in enumerate((12037.5, 9500.0, 13100.0))]
    # the third channel opens after 5 messages (60000 samples) of the first two
    eng, chans = _run_switch(ae, streams, (0, 0, 5), 12000, 10500,
                             ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES | ae.F_DCD_TICK)
    _check(eng, chans, streams, 12000, dict(dcd_tick=True))
    eng.close()


def test_msk_group_switches_shape_mid_stream(engine_lib, monkeypatch):
    import aero_engine as ae
    monkeypatch.setenv('AERO_MSK_WIDE', '2')
    streams = [tl.synth_msk(seconds=30.0, bitrate=600, seed=sd, carrier=f, ebn0=12.0)
               for sd, f in ((0xAE40, 1800.0), (0x5201, 2100.0), (0x5202, 1500.0))]
    eng, chans = _run_switch(ae, streams, (0, 0, 7), 3000, 600,
                             ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    _check(eng, chans, streams, 3000, dict(bitrate=600))
    eng.close()
