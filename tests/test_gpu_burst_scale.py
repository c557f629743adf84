"""Burst OQPSK and burst MSK at a channel count where a pass hands the host
256 or more R/T tests, without parity traces (AERO_F_TRACE_FRAMES only), so
the paths the bench runs are the ones compared with the oracle: the next
pass launched before the host handles this pass's tests, and the tests split
over the engine's host threads by channel (burst_engine.hip process_tests).
Every channel's R/T test results, packets and ACARS items must equal its
own oracle fed the same message boundaries (decode/aerol.h:614-836,
decode/burstoqpskdemodulator.cpp:262-703, decode/burstmskdemodulator.cpp)."""
import concurrent.futures as cf

import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu

N, CHUNK, SECONDS = 320, 12000, 8.0


def _streams(kind):
    # every channel's first burst starts at the same sample (lead_in), so one
    # pass sees all of them mid-burst
    if kind == 'oqpsk':
        return [tl.synth_burst(seconds=SECONDS, seed=300 + k, carrier=11500.0 + 16.0 * k, ebn0=14.0,
                               phase0=0.1 * k) for k in range(N)]
    return [tl.synth_burst_msk(seconds=SECONDS, bitrate=1200, seed=400 + k, carrier=1800.0 + 20.0 * k, ebn0=14.0,
                               phase0=0.1 * k) for k in range(N)]


def _oracle(args):
    pcm, bitrate = args
    o = tl.Oracle(bitrate=bitrate, burst=True)
    o.push_chunked(pcm, CHUNK)
    return o.rt_tests(), o.rt_packets(), o.item_lines('A')


@pytest.mark.parametrize('kind', ['oqpsk', 'msk'])
def test_burst_untraced_split_passes_match_oracle(engine_lib, kind):
    import aero_engine as ae
    bitrate = 10500 if kind == 'oqpsk' else 1200
    streams = _streams(kind)
    eng = ae.Engine(max_channels=N, flags=ae.F_TRACE_FRAMES)
    chans = [eng.open_channel(bitrate, 48000, burst=True) for _ in range(N)]
    L = min(len(s) for s in streams)
    for t in range(0, L, CHUNK):
        for ch, s in zip(chans, streams):
            eng.push(ch, s[t:t + CHUNK])
        eng.run()
    eng.flush()
    assert eng.stat('rt_pass_max') >= 256, 'no pass reached the split path (%d tests)' % eng.stat('rt_pass_max')
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        refs = list(ex.map(_oracle, [(s[:L], bitrate) for s in streams]))
    packets = 0
    for k, (ch, (rtests, rpk, ritems)) in enumerate(zip(chans, refs)):
        assert np.array_equal(eng.rt_tests(ch), rtests), 'channel %d R/T tests differ' % k
        pk = eng.rt_packets(ch)
        assert pk == rpk, 'channel %d R/T packets differ' % k
        assert eng.items(ch) == ritems, 'channel %d items differ' % k
        packets += len(pk)
    assert packets >= N
    eng.close()
