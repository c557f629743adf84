"""GPU parity at SURVEY.md §8(d)'s stream length: 60 s per channel.

Eight continuous 10500-bps OQPSK VFOs (C2) at different carriers (signal
hunting from the default centre, AFC offsets) and Eb/N0 from 6 to 14 dB (the
discrete decisions fed by the libm values: mse < 0.65 gating, (int)WTptr
truncation, IfHavePassedPoint, DCD), one 60-s MSK 600 and one MSK 1200
channel (C3) and one 60-s burst OQPSK channel (C4), against the glibc
oracle: soft bits, rotated pt_qpsk (f64 bitwise), coarse-hop records (f64
bitwise), CRC-checked frames and ACARS items; for the burst channel the
trident records, R/T tests and packets.  Since the device libm is glibc's
own (aero_math.h), nothing is compared within a tolerance.
Reference: decode/oqpskdemodulator.cpp:284-620, decode/mskdemodulator.cpp:
252-428, decode/burstoqpskdemodulator.cpp:262-703, decode/aerol.cpp."""
import concurrent.futures as cf

import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu

SECONDS = 60.0
C2 = [  # seed, carrier Hz, Eb/N0 dB, message size, lead-in samples
    (0x6000, 12037.5, 14.0, 12000, 1000),
    (0x6001, 7020.0, 12.0, 12000, 48000),     # hunter steps to a far carrier
    (0x6002, 15500.0, 10.0, 4800, 24000),
    (0x6003, 9050.3, 9.0, 12000, 1000),
    (0x6004, 12811.1, 8.0, 9600, 96000),      # long acquisition
    (0x6005, 11000.0, 5.0, 12000, 1000),
    (0x6006, 13999.7, 4.0, 3000, 1000),       # low Eb/N0: CRC failures, marginal lock, DCD edges
    (0x6007, 12000.0, 11.0, 48000, 5000),
]


def _oracle_c2(pcm, chunk):
    o = tl.Oracle(trace_pt=True)
    o.push_chunked(pcm, chunk)
    return o.softbits(), o.pt(), o.hops(), o.frames(), o.item_lines('A')


def test_c2_sixty_seconds_eight_channels(engine_lib):
    import aero_engine as ae
    streams = [tl.synth(seconds=SECONDS, seed=s, carrier=f, ebn0=eb, lead_in=li) for s, f, eb, _, li in C2]
    chunks = [c[3] for c in C2]
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        futs = [ex.submit(_oracle_c2, s, c) for s, c in zip(streams, chunks)]  # beside the GPU run
        eng = ae.Engine(max_channels=len(streams), flags=ae.F_TRACE_PT | ae.F_TRACE_SOFT | ae.F_TRACE_HOPS |
                        ae.F_TRACE_FRAMES)
        chans = [eng.open_channel(10500, 48000) for _ in streams]
        pos = [0] * len(streams)
        while any(p < len(s) for p, s in zip(pos, streams)):
            for k, (s, ch) in enumerate(zip(streams, chans)):
                if pos[k] < len(s):
                    eng.push(ch, s[pos[k]:pos[k] + chunks[k]])
                    pos[k] += chunks[k]
            eng.run()
        eng.flush()
        refs = [f.result() for f in futs]
    locked = 0
    for k, ch in enumerate(chans):
        rsb, rpt, rh, rfr, rit = refs[k]
        sb = eng.softbits(ch)
        assert len(sb) == len(rsb) and np.array_equal(sb, rsb), 'C2 case %d soft bits differ' % k
        pt = eng.pt(ch)
        assert pt.shape == rpt.shape and np.array_equal(pt.view(np.int64), rpt.view(np.int64)), \
            'C2 case %d pt_qpsk differs' % k
        h = eng.hops(ch)
        assert h.shape == rh.shape and np.array_equal(h.view(np.int64), rh.view(np.int64)), \
            'C2 case %d hop records differ' % k
        assert np.array_equal(eng.frames(ch), rfr), 'C2 case %d frames differ' % k
        assert eng.items(ch) == rit, 'C2 case %d items differ' % k
        locked += len(rit) > 0
    assert locked >= 6, 'only %d of 8 channels decoded ACARS' % locked
    eng.close()


@pytest.mark.parametrize('bitrate,seed,carrier,ebn0', [(600, 0x6100, 1800.0, 12.0), (1200, 0x6110, 2100.0, 12.0)])
def test_c3_sixty_seconds(engine_lib, bitrate, seed, carrier, ebn0):
    import aero_engine as ae
    pcm = tl.synth_msk(seconds=SECONDS, bitrate=bitrate, baud=600, seed=seed, carrier=carrier, ebn0=ebn0)
    chunk = 3000 if bitrate == 600 else 6000
    o = tl.Oracle(bitrate=bitrate)
    o.push_chunked(pcm, chunk)
    eng = ae.Engine(max_channels=1, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    ch = eng.open_channel(bitrate)
    for i in range(0, len(pcm), chunk):
        eng.push(ch, pcm[i:i + chunk])
        eng.run()
    eng.flush()
    sb, rsb = eng.softbits(ch), o.softbits()
    assert len(rsb) > 10000 and np.array_equal(sb, rsb)
    h, rh = eng.hops(ch), o.hops()
    assert h.shape == rh.shape and np.array_equal(h.view(np.int64), rh.view(np.int64))
    assert np.array_equal(eng.frames(ch), o.frames())
    items = eng.items(ch)
    assert items and items == o.item_lines('A')
    eng.close()


def test_c4_sixty_seconds(engine_lib):
    import aero_engine as ae
    pcm = tl.synth_burst(seconds=SECONDS, seed=0x6200, carrier=12100.0, ebn0=12.0)
    chunk = 12000
    o = tl.Oracle(burst=True)
    o.push_chunked(pcm, chunk)
    eng = ae.Engine(max_channels=1, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    ch = eng.open_channel(10500, 48000, burst=True)
    for i in range(0, len(pcm), chunk):
        eng.push(ch, pcm[i:i + chunk])
        eng.run()
    eng.flush()
    h, rh = eng.hops(ch), o.hops()
    assert len(rh) > 0 and h.shape == rh.shape and np.array_equal(h.view(np.int64), rh.view(np.int64))
    s, rs = eng.softbits16(ch), o.softbits16()
    assert len(rs) > 10000 and np.array_equal(s, rs)
    assert np.array_equal(eng.rt_tests(ch), o.rt_tests())
    pk = eng.rt_packets(ch)
    assert len(pk) >= 5 and pk == o.rt_packets()
    items = eng.items(ch)
    assert items and items == o.item_lines('A')
    eng.close()
