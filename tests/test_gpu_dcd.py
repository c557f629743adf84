"""GPU parity of AeroL's 1 s DCD timer on the sample clock (AERO_F_DCD_TICK).

60-s continuous 10500-bps OQPSK channels (C2) that each lose two ZMQ
messages, against the oracle with ORACLE_DCD_TICK: soft bits, CRC-checked
frames, ACARS items and the DataCarrierDetect changes, bitwise.  With the
timer, the framing depends on the CRCs of the frames before each tick
(decode/aerol.cpp:1043-1058, 1096, 1108, 1545-1556); aerol.hip's frame_kernel
stops a channel where they are still being decoded and resumes it after the
Viterbi.  Both paths are checked: the pass-by-pass one of the parity traces,
and the production one where a pass's Viterbi runs inside the next pass.
Both demodulator shapes record the ticks (oqpsk_kernel fixture)."""
import concurrent.futures as cf

import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu

SECONDS = 60.0
CASES = [  # seed, carrier Hz, Eb/N0 dB, message size, lead-in, the two lost messages
    (0x6A00, 12037.5, 12.0, 12000, 1000, (20, 130)),
    (0x6A01, 9050.3, 9.0, 4800, 1000, (75, 400)),
    (0x6A02, 13999.7, 5.0, 12000, 1000, (60, 170)),   # CRC failures: datacd falls and rises on its own
    (0x6A03, 7020.0, 11.0, 9600, 48000, (100, 200)),  # hunter steps first
]


def _messages(case):
    seed, f, eb, msg, li, lost = case
    pcm = tl.synth(seconds=SECONDS, seed=seed, carrier=f, ebn0=eb, lead_in=li)
    return [pcm[i:i + msg] for k, i in enumerate(range(0, len(pcm), msg)) if k not in lost]


def _oracle(msgs, tick):
    o = tl.Oracle(dcd_tick=tick)
    for m in msgs:
        o.push(m)
    return o.softbits(), o.frames(), o.item_lines('A'), o.events()[0]


@pytest.fixture(scope='module')
def dcd_refs(cpu_libs):
    msgs = [_messages(c) for c in CASES]
    with cf.ThreadPoolExecutor(max_workers=len(CASES) + 1) as ex:
        ticked = [ex.submit(_oracle, m, True) for m in msgs]
        untimed = ex.submit(_oracle, msgs[0], False)
        return msgs, [f.result() for f in ticked], untimed.result()


def _engine_run(msgs, flags):
    import aero_engine as ae
    eng = ae.Engine(max_channels=len(msgs), flags=flags | ae.F_DCD_TICK)
    chans = [eng.open_channel(10500, 48000) for _ in msgs]
    k = 0
    while any(k < len(m) for m in msgs):
        for m, ch in zip(msgs, chans):
            if k < len(m):
                eng.push(ch, m[k])
        eng.run()
        k += 1
    eng.flush()
    return eng, chans


def test_dcd_tick_lost_messages(engine_lib, oqpsk_kernel, dcd_refs):
    import aero_engine as ae
    msgs, refs, untimed = dcd_refs
    # the timer matters here: the untimed reference loses the channel after the first lost message
    assert len(refs[0][2]) > len(untimed[2]) + 20
    assert sum(r[3] > 1 for r in refs) >= 3  # datacd fell (and rose again) on most channels
    # pass by pass (parity traces: each pass's Viterbi right after its framing)
    eng, chans = _engine_run(msgs, ae.F_TRACE_SOFT | ae.F_TRACE_FRAMES)
    for k, ch in enumerate(chans):
        rsb, rfr, rit, redges = refs[k]
        sb = eng.softbits(ch)
        assert len(sb) == len(rsb) and np.array_equal(sb, rsb), 'case %d soft bits differ' % k
        assert np.array_equal(eng.frames(ch), rfr), 'case %d frames differ' % k
        assert eng.items(ch) == rit, 'case %d items differ' % k
        assert eng.channel_events(ch)[0] == redges, 'case %d DCD changes differ' % k
    eng.close()
    # production: a pass's Viterbi runs in the next pass, so the framing that
    # stopped at a tick resumes a pass later
    eng, chans = _engine_run(msgs, ae.F_TRACE_FRAMES)
    for k, ch in enumerate(chans):
        _, rfr, rit, redges = refs[k]
        assert np.array_equal(eng.frames(ch), rfr), 'case %d frames differ (deferred Viterbi)' % k
        assert eng.items(ch) == rit, 'case %d items differ (deferred Viterbi)' % k
        assert eng.channel_events(ch)[0] == redges, 'case %d DCD changes differ (deferred Viterbi)' % k
    eng.close()
