"""Oracle properties of the continuous MSK path (`aero-decode -b 600|1200`,
decode/mskdemodulator.cpp + the 600/1200 branch of AeroL::Decode):
the synthetic MSK transmitter's frames decode to exactly what was
transmitted, items carry the transmitted messages, and output does not
depend on how the stream is split into ZMQ messages (SURVEY.md §8(b):
probe-confirmed chunk invariance for MSK)."""
import numpy as np
import pytest

import aero_testlib as tl


@pytest.fixture(scope='module')
def msk600(cpu_libs):
    return tl.synth_msk(seconds=30.0, bitrate=600, seed=0xAE40, carrier=1800.0, ebn0=12.0, return_frames=True)


def test_msk600_frames_decode_to_transmitted(msk600):
    pcm, tx = msk600
    o = tl.Oracle(bitrate=600)
    o.push_chunked(pcm, 3000)
    recs = tl.frame_records(o.frames())
    good = [info for info, m in recs if m == (1 << 6) - 1]
    assert len(good) >= 6  # the hunter reaches the 1800 Hz carrier after ~8 s
    assert all(len(info) == 72 for info in good)
    tx_list = [bytes(t) for t in tx]
    idx = [tx_list.index(info) for info in good]
    assert idx == list(range(idx[0], idx[0] + len(idx))), 'frames out of order'


def test_msk600_items(msk600):
    pcm, _ = msk600
    o = tl.Oracle(bitrate=600)
    o.push_chunked(pcm, 3000)
    items = o.item_lines('A')
    assert len(items) >= 3
    for line in items:
        f = dict(kv.split('=', 1) for kv in line.split()[1:])
        assert f['valid'] == '1'


def test_msk600_soft_bit_rate(msk600):
    """600 soft bits per second, delivered in groups of 12
    (decode/mskdemodulator.cpp:404-407)."""
    pcm, _ = msk600
    o = tl.Oracle(bitrate=600)
    o.push_chunked(pcm, 3000)
    n = len(o.softbits())
    assert n % 12 == 0
    assert abs(n - 600 * len(pcm) / 12000) < 24


@pytest.mark.parametrize('chunk', [1, 500, 2048, 12000])
def test_msk600_chunk_invariance(msk600, chunk):
    pcm, _ = msk600
    pcm = pcm[:12000 * 10]
    ref = tl.Oracle(bitrate=600)
    ref.push_chunked(pcm, 3000)
    o = tl.Oracle(bitrate=600)
    o.push_chunked(pcm, chunk)
    assert np.array_equal(o.softbits(), ref.softbits())
    assert np.array_equal(o.hops(), ref.hops())
    assert o.item_lines('A') == ref.item_lines('A')


def test_msk600_hunter_steps_450hz(cpu_libs):
    """No signal: centre steps of 450 Hz every 15 hops of 2048 samples,
    clamped to [450, 5550] (decode/decode.cpp:193, mskdemodulator.cpp:220-240)."""
    pcm = np.random.default_rng(11).normal(0, 3000, 12000 * 12).astype(np.int16)
    o = tl.Oracle(bitrate=600)
    o.push_chunked(pcm, 3000)
    h = o.hops()
    assert np.all(np.diff(h[:, 0]) == 2048)
    centers = h[:, 3]
    moved = [k for k in range(1, len(h)) if centers[k] != centers[k - 1]]
    assert moved and moved[0] >= 14  # 15 no-signal hops in a row at the earliest
    for k in moved:
        assert centers[k] % 450.0 == 0.0 and 450.0 <= centers[k] <= 5550.0


def test_msk1200_framing_at_600_baud(cpu_libs):
    """aero-decode -b 1200 demodulates at fb = 600 with 24 kHz input and
    N = 9 framing (decode/decode.cpp:142-150, aerol.cpp:984-993): a 600-baud
    stream in the 1200 frame layout decodes some transmitted frames."""
    pcm, tx = tl.synth_msk(seconds=30.0, bitrate=1200, baud=600, seed=0xAE41, carrier=1800.0,
                           return_frames=True)
    o = tl.Oracle(bitrate=1200)
    o.push_chunked(pcm, 6000)
    assert len(o.softbits()) == pytest.approx(600 * 30, abs=30)
    tx_set = {bytes(t) for t in tx}
    good = [info for info, m in tl.frame_records(o.frames()) if m == 0x3F]
    assert good and all(info in tx_set for info in good)
