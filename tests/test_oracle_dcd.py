"""AeroL's 1 s DCD timer on the sample clock, in the oracle (CPU).

The shipped aero-decode runs Qt's event loop (decode/main.cpp:106), so
AeroL's QTimer fires AeroL::updateDCD every second (decode/aerol.cpp:900-902,
1043-1058).  Once CRC failures have drained datacdcountdown (:1545-1556), a
tick clears datacd and the UW search runs at every bit again (:1096, :1108).
Without the timer a continuous channel that has synced once searches for the
UW only in the window at the expected frame boundary, so one lost message
(or a sound card dropping a buffer, :1998-2001) leaves it unsynced for good.
ORACLE_DCD_TICK fires the timer after every 48000 input samples."""
import numpy as np
import pytest

import aero_testlib as tl


@pytest.fixture(scope='module')
def c2_30s(cpu_libs):
    return tl.synth(seconds=30.0, seed=0xAE20)


def _items(pcm, tick, chunk=12000):
    o = tl.Oracle(dcd_tick=tick)
    o.push_chunked(pcm, chunk)
    return o.item_lines('A'), o.events()[0]


def test_tick_neutral_on_an_intact_stream(c2_30s):
    a, ea = _items(c2_30s, False)
    b, eb = _items(c2_30s, True)
    assert len(a) >= 90 and a == b
    assert ea == eb == 1  # one "no signal => signal" edge, never lost


def test_tick_resyncs_after_a_lost_buffer(c2_30s):
    # one 0.3-s buffer (14400 samples) lost at t = 10 s
    pcm = np.concatenate([c2_30s[:480000], c2_30s[480000 + 14400:]])
    untimed, e0 = _items(pcm, False)
    ticked, e1 = _items(pcm, True)
    intact, _ = _items(c2_30s, True)
    # untimed: nothing after the loss; ticked: datacd drops within ~1 s of
    # the garbage frame's CRC failures and the UW search finds the frames again
    assert len(untimed) <= 30, len(untimed)
    assert len(ticked) >= 80, len(ticked)
    assert e0 == 1 and e1 == 3  # signal, lost, signal again
    # every item the untimed run decoded (all before the loss) is in the ticked run
    assert ticked[:len(untimed)] == untimed
    assert set(ticked) <= set(intact)


def test_tick_chunk_invariant(c2_30s):
    """The tick is on the sample clock, so a continuous channel stays
    chunk-invariant."""
    pcm = np.concatenate([c2_30s[:600000], c2_30s[600000 + 12000:]])
    ref, e = _items(pcm, True, 12000)
    for chunk in (4800, 48000):
        got, e2 = _items(pcm, True, chunk)
        assert got == ref and e2 == e
