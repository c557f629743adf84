"""GPU parity of the C channel (8400 bps) against the oracle.

OqpskDemodulator at fb = 8400 with its per-message JFastFir prefilter
(decode/oqpskdemodulator.cpp:174-240, 292-324, 376-390, 463-472, 555-557),
the windowed coarse estimator (decode/coarsefreqestimate.cpp:97-104) and
AeroL::DecodeC (decode/aerol.cpp:2145-2432) on the engine (cchan.hip,
coarse.hip) vs the oracle restatement on the same messages: soft bits,
rotated pt (f64 bitwise), hop records, frames (SU bytes + CRC masks), the
Call_progress SUs, the voice frames with their AES tags and the DCD
changes.  The prefilter makes the output depend on the message boundaries,
so engine and oracle get the same messages (sizes 4800, 9600, 12000)."""
import concurrent.futures as cf

import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu

CASES = [  # seed, carrier Hz, Eb/N0 dB, seconds, message size
    (0xC100, 12037.5, 12.0, 24.0, 12000),
    (0xC101, 15500.0, 8.0, 24.0, 4800),
    (0xC102, 9050.0, 6.0, 20.0, 9600),
    (0xC103, 7020.0, 14.0, 20.0, 12000),
]


def _oracle(pcm, chunk):
    o = tl.Oracle(bitrate=8400, trace_pt=True)
    o.push_chunked(pcm, chunk)
    return o.softbits(), o.pt(), o.hops(), o.frames(), o.c_units(), o.voice(), o.events()[0]


@pytest.fixture(scope='module')
def c_refs(cpu_libs):
    streams = [tl.synth_c(seconds=sec, seed=s, carrier=f, ebn0=eb) for s, f, eb, sec, _ in CASES]
    with cf.ThreadPoolExecutor(max_workers=len(CASES)) as ex:
        refs = [f.result() for f in [ex.submit(_oracle, s, c[4]) for s, c in zip(streams, CASES)]]
    return streams, refs


def _run(ae, streams, flags):
    eng = ae.Engine(max_channels=len(streams), flags=flags)
    chans = [eng.open_channel(8400, 48000) for _ in streams]
    pos = [0] * len(streams)
    while any(p < len(s) for p, s in zip(pos, streams)):
        for k, (s, ch) in enumerate(zip(streams, chans)):
            if pos[k] < len(s):
                eng.push(ch, s[pos[k]:pos[k] + CASES[k][4]])
                pos[k] += CASES[k][4]
        eng.run()
    eng.flush()
    return eng, chans


def test_c_channel_matches_oracle(engine_lib, c_refs):
    import aero_engine as ae
    streams, refs = c_refs
    eng, chans = _run(ae, streams, ae.F_TRACE_PT | ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    for k, ch in enumerate(chans):
        rsb, rpt, rh, rfr, rcu, rv, redges = refs[k]
        sb = eng.softbits(ch)
        assert len(rsb) > 10000 and len(sb) == len(rsb) and np.array_equal(sb, rsb), 'case %d soft bits differ' % k
        pt = eng.pt(ch)
        assert pt.shape == rpt.shape and np.array_equal(pt.view(np.int64), rpt.view(np.int64)), \
            'case %d pt differs' % k
        h = eng.hops(ch)
        assert h.shape == rh.shape and np.array_equal(h.view(np.int64), rh.view(np.int64)), \
            'case %d hop records differ' % k
        assert len(rfr) >= 320 * 20 and np.array_equal(eng.frames(ch), rfr), 'case %d frames differ' % k
        assert np.array_equal(eng.c_units(ch), rcu), 'case %d Call_progress SUs differ' % k
        assert eng.voice(ch) == rv, 'case %d voice frames differ' % k
        assert eng.channel_events(ch)[0] == redges, 'case %d DCD changes differ' % k
    assert sum(len(r[4]) for r in refs) >= 40
    eng.close()


def test_c_channel_deferred_viterbi(engine_lib, c_refs):
    """The production order: a pass's Viterbi runs inside the next pass."""
    import aero_engine as ae
    streams, refs = c_refs
    eng, chans = _run(ae, streams, ae.F_TRACE_FRAMES)
    for k, ch in enumerate(chans):
        _, _, _, rfr, rcu, rv, _ = refs[k]
        assert np.array_equal(eng.frames(ch), rfr), 'case %d frames differ' % k
        assert np.array_equal(eng.c_units(ch), rcu), 'case %d Call_progress SUs differ' % k
        assert eng.voice(ch) == rv, 'case %d voice frames differ' % k
    eng.close()


def test_c_channel_ragged_messages(engine_lib, cpu_libs):
    """Message sizes around the prefilter's 2048-sample blocks (shorter than a
    block, ending on and just past a block boundary, the 32768 maximum, one
    sample): everything equal to the oracle fed the same messages."""
    import aero_engine as ae
    pcm = tl.synth_c(seconds=14.0, seed=0xC1A5, carrier=11000.0, ebn0=12.0)
    sizes = [1, 2047, 2048, 2049, 32768, 100, 4096, 12000, 6143, 1, 30000, 2048, 9000]
    msgs, p, k = [], 0, 0
    while p < len(pcm):
        n = sizes[k % len(sizes)]
        msgs.append(pcm[p:p + n])
        p += n
        k += 1
    o = tl.Oracle(bitrate=8400, trace_pt=True)
    for m in msgs:
        o.push(m)
    eng = ae.Engine(max_channels=1, flags=ae.F_TRACE_PT | ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    ch = eng.open_channel(8400, 48000)
    for m in msgs:
        eng.push(ch, m)
        eng.run()
    eng.flush()
    sb = eng.softbits(ch)
    assert len(sb) > 10000 and np.array_equal(sb, o.softbits())
    assert np.array_equal(eng.pt(ch).view(np.int64), o.pt().view(np.int64))
    assert np.array_equal(eng.hops(ch).view(np.int64), o.hops().view(np.int64))
    assert np.array_equal(eng.frames(ch), o.frames()) and len(o.frames()) > 0
    assert np.array_equal(eng.c_units(ch), o.c_units())
    assert eng.voice(ch) == o.voice()
    eng.close()
