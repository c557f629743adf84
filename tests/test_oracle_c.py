"""The C channel (8400 bps) in the oracle: the synthetic
C-channel transmitter (tools/aero_synth.cpp aero_synth_c8400) through the
restated receive chain -- OqpskDemodulator at fb = 8400 with its JFastFir
prefilter (decode/oqpskdemodulator.cpp:174-240, 292-324, 376-390, 463-472,
555-557), the windowed coarse estimator (decode/coarsefreqestimate.cpp:
97-104) and AeroL::DecodeC (decode/aerol.cpp:2145-2432: dual 52-bit
preambles, 4 x 64 deinterleave, rate-3/4 depuncture, Viterbi, delay line,
descrambler, three SUs and 25 voice frames per 0.5-s frame) -- recovers
every transmitted SU and voice frame once locked.  A round trip, the pin
this path has (no reference fixtures exist; parity unpinned otherwise)."""
import numpy as np
import pytest

import aero_testlib as tl


@pytest.mark.parametrize('seed,carrier,ebn0', [(0xAEC1, 12037.5, 12.0), (0xAEC3, 15500.0, 8.0)])
def test_c_channel_round_trip(cpu_libs, seed, carrier, ebn0):
    pcm, fr = tl.synth_c(seconds=30.0, seed=seed, carrier=carrier, ebn0=ebn0, return_frames=True)
    o = tl.Oracle(bitrate=8400)
    o.push_chunked(pcm, 12000)
    frames = tl.frame_records(o.frames())
    assert len(frames) >= 48
    # the first two frames decode before the delay line and the Viterbi
    # overlap hold the previous frame; every later one is intact
    assert all(m == 7 and len(f) == 36 for f, m in frames[2:])
    tx_su = [bytes(r[:36]) for r in fr]
    tx_v = [bytes(r[36:]) for r in fr]
    got = [f for f, _ in frames[2:]]
    k = tx_su.index(got[0])  # the frame a decoded frame carries (one behind the air frame)
    assert got == tx_su[k:k + len(got)]
    voice = o.voice()[2:]
    assert [v for _, v in voice] == tx_v[k:k + len(got)]
    # Call_progress SUs (message 0x30) and the AES each voice frame is tagged with
    cps = [bytes(r) for r in o.c_units()]
    want = [su[12 * j:12 * j + 12] for su in got for j in range(3) if su[12 * j] == 0x30]
    assert cps[-len(want):] == want
    for (aes, _), su in zip(voice, got):
        last = [su[12 * j + 1:12 * j + 4] for j in range(3) if su[12 * j] == 0x30]
        assert aes == (int.from_bytes(last[-1], 'big') if last else 0)


def test_c_channel_chunking_changes_only_rounding(cpu_libs):
    """The prefilter re-mixes each message from its saved phase and retunes
    to the message's mean carrier (oqpskdemodulator.cpp:300-316, 555-557), so
    unlike the P channel the C channel is not chunk-invariant bit for bit;
    the decoded SUs are the same."""
    pcm = tl.synth_c(seconds=16.0, seed=0xAEC5, carrier=11000.0, ebn0=14.0)
    outs = []
    for chunk in (4800, 12000):
        o = tl.Oracle(bitrate=8400)
        o.push_chunked(pcm, chunk)
        outs.append((o.softbits(), tl.frame_records(o.frames())))
    good = [set(f for f, m in fr if m == 7) for _, fr in outs]
    assert len(good[0]) >= 25 and len(good[0] & good[1]) >= len(good[0]) - 2
