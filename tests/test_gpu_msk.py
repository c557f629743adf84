"""GPU parity of the continuous MSK path (`aero-decode -b 600|1200`): the HIP
engine vs the CPU oracle on the same synthetic VFO streams.  Soft bits,
coarse-hop records, Viterbi blocks, frames and ACARS items bit-exact; the
rotated pt_msk soft-metric floats within 1e-5 (BASELINE.json north_star)."""
import numpy as np
import pytest

import aero_testlib as tl

PT_TOL = 1e-5

CASES = [
    # bitrate, baud, seed, carrier Hz, Eb/N0 dB, seconds, message size (samples)
    (600, 600, 0xAE40, 1800.0, 12.0, 24.0, 3000),
    (600, 600, 0xAE41, 300.0, 9.0, 16.0, 1000),
    (600, 600, 0xAE42, 2411.0, 14.0, 20.0, 12000),
    (1200, 600, 0xAE43, 1800.0, 12.0, 20.0, 6000),
    (1200, 1200, 0xAE44, 3000.0, 12.0, 12.0, 24000),
]


def _streams(cases):
    return [tl.synth_msk(seconds=sec, bitrate=br, baud=bd, seed=seed, carrier=f, ebn0=eb)
            for br, bd, seed, f, eb, sec, _ in cases]


def _run(eng, chans, streams, chunks):
    pos = [0] * len(streams)
    while any(p < len(s) for p, s in zip(pos, streams)):
        for k, (s, ch) in enumerate(zip(streams, chans)):
            if pos[k] < len(s):
                eng.push(ch, s[pos[k]:pos[k] + chunks[k]])
                pos[k] += chunks[k]
        eng.run()
    eng.flush()


@pytest.mark.gpu
def test_msk_engine_matches_oracle(engine_lib, msk_kernel):
    import aero_engine as ae
    streams = _streams(CASES)
    chunks = [c[6] for c in CASES]
    eng = ae.Engine(max_channels=8, flags=ae.F_TRACE_ALL)
    chans = [eng.open_channel(c[0]) for c in CASES]
    _run(eng, chans, streams, chunks)
    for k, (s, ch) in enumerate(zip(streams, chans)):
        o = tl.Oracle(trace_pt=True, bitrate=CASES[k][0])
        o.push_chunked(s, chunks[k])
        sb_o, sb_e = o.softbits(), eng.softbits(ch)
        assert len(sb_o) > 1000
        assert len(sb_e) == len(sb_o), 'case %d soft-bit count %d vs %d' % (k, len(sb_e), len(sb_o))
        assert np.array_equal(sb_e, sb_o), 'case %d soft bits differ at %s' % (k, np.nonzero(sb_e != sb_o)[0][:10])
        assert np.array_equal(eng.hops(ch), o.hops()), 'case %d hop records differ' % k
        p_o, p_e = o.pt(), eng.pt(ch)
        assert p_o.shape == p_e.shape
        assert np.max(np.abs(p_o - p_e)) <= PT_TOL
        assert np.array_equal(eng.blocks(ch), o.blocks()), 'case %d Viterbi blocks differ' % k
        assert np.array_equal(eng.frames(ch), o.frames()), 'case %d frames differ' % k
        assert eng.items(ch) == o.item_lines('A'), 'case %d ACARS items differ' % k
    eng.close()


@pytest.mark.gpu
def test_mixed_kinds_one_engine(engine_lib):
    """10500 OQPSK and 600/1200 MSK channels interleaved in one engine: every
    channel equals its own oracle (channel ids route to per-kind groups)."""
    import aero_engine as ae
    oq = [tl.synth(seconds=8.0, seed=0xAE70 + k, carrier=12037.5 + k, ebn0=12.0) for k in range(2)]
    mk = _streams([(600, 600, 0xAE72, 600.0, 12.0, 16.0, 3000), (1200, 600, 0xAE73, 600.0, 12.0, 16.0, 6000)])
    eng = ae.Engine(max_channels=4, flags=ae.F_TRACE_SOFT)
    order = [('o', 0), ('m', 0), ('o', 1), ('m', 1)]
    chans, streams, chunks, rates = [], [], [], []
    for kind, k in order:
        if kind == 'o':
            chans.append(eng.open_channel(10500))
            streams.append(oq[k]), chunks.append(12000), rates.append(10500)
        else:
            br = (600, 1200)[k]
            chans.append(eng.open_channel(br))
            streams.append(mk[k]), chunks.append(3000 * (k + 1)), rates.append(br)
    assert chans == [0, 1, 2, 3]
    drained = []
    pos = [0] * 4
    while any(p < len(s) for p, s in zip(pos, streams)):
        for k in range(4):
            if pos[k] < len(streams[k]):
                eng.push(chans[k], streams[k][pos[k]:pos[k] + chunks[k]])
                pos[k] += chunks[k]
        eng.run()
        drained += eng.drain_items(lines=True)
    eng.flush()
    drained += eng.drain_items(lines=True)
    for k in range(4):
        o = tl.Oracle(bitrate=rates[k])
        o.push_chunked(streams[k], chunks[k])
        assert np.array_equal(eng.softbits(chans[k]), o.softbits()), 'channel %d soft bits differ' % k
        assert [line for c, line in drained if c == chans[k]] == o.item_lines('A'), 'channel %d items' % k
    eng.close()


@pytest.mark.gpu
def test_msk_many_channels(engine_lib, msk_kernel):
    """300 MSK-600 channels (two 256-lane workgroups, out of step: carriers,
    phases, noise, push sizes) against the oracle, channel by channel."""
    import aero_engine as ae
    nch = 300
    rng = np.random.default_rng(5)
    streams = [tl.synth_msk(seconds=8.0, bitrate=600, seed=0xAE80 + k, carrier=float(rng.uniform(200, 700)),
                            ebn0=float(rng.uniform(9, 14)), phase0=float(rng.uniform(0, 6.28)))
               for k in range(nch)]
    chunks = [int(rng.choice([500, 2048, 3000, 9000])) for _ in range(nch)]
    eng = ae.Engine(max_channels=nch, flags=ae.F_TRACE_SOFT)
    chans = [eng.open_channel(600) for _ in range(nch)]
    _run(eng, chans, streams, chunks)
    for k in range(nch):
        o = tl.Oracle(bitrate=600)
        o.push_chunked(streams[k], 3000)
        assert np.array_equal(eng.softbits(chans[k]), o.softbits()), 'channel %d soft bits differ' % k
        assert eng.items(chans[k]) == o.item_lines('A'), 'channel %d items differ' % k
    eng.close()
