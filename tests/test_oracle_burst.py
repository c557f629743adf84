"""Oracle properties of the burst OQPSK path (`aero-decode -b 10500 --burst`,
decode/burstoqpskdemodulator.cpp + the R/T branch of AeroL::Decode): bursts
from the synthetic R/T transmitter are detected at their carrier by the
trident check, every decoded R/T packet is one that was transmitted, and the
R user-data / T SUs come out as downlink ACARS items."""
import numpy as np
import pytest

import aero_testlib as tl


@pytest.fixture(scope='module')
def bursts(cpu_libs):
    pcm, pk = tl.synth_burst(seconds=30.0, seed=2, carrier=12000.0, ebn0=14.0, return_packets=True)
    o = tl.Oracle(burst=True)
    o.push_chunked(pcm, 12000)
    return pcm, pk, o


def test_trident_detects_carrier(bursts):
    _, pk, o = bursts
    h = o.hops()  # per trident check: sample, detected, mixer Hz, gain, maxval, bin
    det = h[h[:, 1] == 1.0]
    assert len(det) >= len(pk) // 2
    assert np.all(np.abs(det[:, 2] - 12000.0) < 2 * 48000.0 / 32768)


def test_decoded_packets_were_transmitted(bursts):
    _, pk, o = bursts
    got = o.rt_packets()
    assert len(got) >= 4
    for kind, info in got:
        if kind == 'R':  # 20 bytes: the 19 sent + the tail byte
            assert any(k == 'R' and info[:19] == b for k, b in pk)
        else:  # T: the infofield is the packet minus nothing (chop(1) drops the tail byte)
            assert any(k == 'T' and info[:len(b)] == b for k, b in pk)


def test_items_are_downlink(bursts):
    _, _, o = bursts
    items = o.item_lines('A')
    assert items
    for line in items:
        f = dict(kv.split('=', 1) for kv in line.split()[1:])
        assert f['downlink'] == '1' and f['valid'] == '1'


def test_start_of_packet_markers(bursts):
    """one -1 marker per detected burst, delivered with the soft bits of its
    group (groups close at >= 32 entries, burstoqpskdemodulator.cpp:455-458, 683-690)"""
    _, _, o = bursts
    s16 = o.softbits16()
    assert np.sum(s16 >= 0) % 2 == 0
    assert np.sum(s16 < 0) == np.sum(o.hops()[:, 1] == 1.0)


def test_noise_only_no_packets(cpu_libs):
    pcm = np.random.default_rng(9).normal(0, 2000, 48000 * 6).astype(np.int16)
    o = tl.Oracle(burst=True)
    o.push_chunked(pcm, 12000)
    assert o.rt_packets() == []
    assert o.item_lines('A') == []
