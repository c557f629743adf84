"""Oracle properties of the burst MSK path (`aero-decode -b 600|1200 --burst`,
decode/burstmskdemodulator.cpp + the MSK branch of AeroL::Decode with
RTChannelDeleaveFECScram::updateMSK, decode/aerol.cpp:1155-1178,
decode/aerol.h:614-753): bursts from the synthetic 1200-baud transmitter
(carrier start tone, 0-1 preamble, UW, R/T packet) are detected by the trident
check at their carrier, every decoded packet is one that was transmitted, T
packets decode at their target block (blocks 5, 11 and 3 S + 5 are the only
tests), and both bit rates give downlink ACARS items."""
import numpy as np
import pytest

import aero_testlib as tl

OK_R, OK_T, BAD, NOTHING = 3, 5, 0, 8


@pytest.fixture(scope='module', params=[600, 1200])
def bursts(request, cpu_libs):
    br = request.param
    pcm, pk = tl.synth_burst_msk(seconds=30.0, bitrate=br, seed=21, carrier=2500.0, ebn0=13.0,
                                 return_packets=True)
    o = tl.Oracle(bitrate=br, burst=True)
    o.push_chunked(pcm, 12000)
    return br, pk, o


def test_trident_detects_carrier(bursts):
    _, pk, o = bursts
    h = o.hops()  # per trident check: sample, detected, mixer Hz, gain, minval, bins
    det = h[h[:, 1] == 1.0]
    assert len(det) >= len(pk) - 1
    # mixer2 lands on the mid-point of the two 0-1 preamble lines (integer bins)
    assert np.all(np.abs(det[:, 2] - 2500.0) < 3 * 48000.0 / 32768)


def test_decoded_packets_were_transmitted(bursts):
    _, pk, o = bursts
    got = o.rt_packets()
    assert len(got) >= len(pk) - 2 and any(k == 'T' for k, _ in got) and any(k == 'R' for k, _ in got)
    for kind, info in got:
        assert any(k == kind and info[:len(b)] == b for k, b in pk)


def test_tests_only_at_msk_blocks(bursts):
    """updateMSK tests at block 5 (R, then reset of the T target), 11 (SU
    count peek), 50 and the target block 3 S + 5; R failures are Nothing,
    T header failures Bad"""
    _, pk, o = bursts
    t = o.rt_tests()
    assert len(t)
    for bp, r in t:
        assert bp % 64 == 0 and (bp // 64 in (5, 11, 50) or (bp // 64 - 5) % 3 == 0)
        assert r in (OK_R, OK_T, BAD, NOTHING)
    tpk = [(k, b) for k, b in o.rt_packets() if k == 'T']
    ts = [bp for bp, r in t if r == OK_T]
    assert len(ts) == len(tpk)
    for bp, (_, info) in zip(ts, tpk):
        nsu = (bp // 64 - 5) // 3  # (S + 1) * 3 + 2 blocks
        assert len(info) == bp // 16 - 1 and len(info) >= 6 + 12 * nsu


def test_items_are_downlink(bursts):
    _, _, o = bursts
    items = o.item_lines('A')
    assert items
    for line in items:
        f = dict(kv.split('=', 1) for kv in line.split()[1:])
        assert f['downlink'] == '1' and f['valid'] == '1'


def test_start_of_burst_markers(bursts):
    """one -1 marker per detected burst; groups are emitted at >= 12 entries,
    the marker counting (burstmskdemodulator.cpp:503-505, 689-692)"""
    _, _, o = bursts
    s16 = o.softbits16()
    assert np.sum(s16 < 0) == np.sum(o.hops()[:, 1] == 1.0)


def test_noise_only_no_packets(cpu_libs):
    pcm = np.random.default_rng(19).normal(0, 2000, 48000 * 6).astype(np.int16)
    o = tl.Oracle(bitrate=1200, burst=True)
    o.push_chunked(pcm, 12000)
    assert o.rt_packets() == []
    assert o.item_lines('A') == []


def test_chunk_invariant(cpu_libs):
    """unlike burst OQPSK (lastmse), the MSK burst demodulator does not depend
    on message boundaries"""
    pcm = tl.synth_burst_msk(seconds=8.0, bitrate=1200, seed=23, carrier=3100.0, ebn0=14.0)
    a, b = tl.Oracle(bitrate=1200, burst=True), tl.Oracle(bitrate=1200, burst=True)
    a.push_chunked(pcm, 12000)
    b.push_chunked(pcm, 1777)
    assert np.array_equal(a.softbits16(), b.softbits16())
    assert a.rt_packets() == b.rt_packets() and a.rt_packets()
