"""End-to-end property of the oracle: the synthetic transmitter's frames
decode to exactly what was transmitted, and continuous-mode output is
independent of how the stream is split into ZMQ messages."""
import numpy as np
import pytest

import aero_testlib as tl


@pytest.fixture(scope='module')
def stream(cpu_libs):
    return tl.synth(seconds=16.0, seed=0xAE20, carrier=12037.5, ebn0=12.0, return_frames=True)


def test_frames_decode_to_transmitted(stream):
    pcm, tx = stream
    o = tl.Oracle()
    o.push_chunked(pcm, 12000)
    recs = tl.frame_records(o.frames())
    good = [(info, m) for info, m in recs if m == (1 << 26) - 1]
    assert len(good) >= 20
    tx_set = {bytes(t) for t in tx}
    for info, _ in good:
        assert info in tx_set
    # consecutive, in transmit order
    idx = [next(i for i, t in enumerate(tx) if bytes(t) == info) for info, _ in good]
    assert idx == list(range(idx[0], idx[0] + len(idx)))


def test_acars_items_are_transmitted_messages(stream):
    pcm, tx = stream
    o = tl.Oracle()
    o.push_chunked(pcm, 12000)
    items = o.item_lines('A')
    assert len(items) >= 20
    for line in items:
        f = dict(kv.split('=', 1) for kv in line.split()[1:])
        assert f['valid'] == '1'
        if f['nonacars'] == '0':
            msg = bytes.fromhex(f['msg'])
            assert all(32 <= c < 127 or c in (10, 13) for c in msg)
            assert bytes.fromhex(f['reg']).startswith(b'N')


@pytest.mark.parametrize('chunk', [1, 777, 4096, 96000])
def test_chunk_invariance(stream, chunk):
    pcm, _ = stream
    pcm = pcm[:48000 * 8]
    ref = tl.Oracle()
    ref.push_chunked(pcm, 12000)
    o = tl.Oracle()
    o.push_chunked(pcm, chunk)
    assert np.array_equal(o.softbits(), ref.softbits())
    assert o.item_lines('A') == ref.item_lines('A')


def test_noise_only_hunts(cpu_libs):
    """No carrier: the hunter steps the centre 5250 Hz every 15 hops
    (decode/hunter.cpp:21-42) whenever 15 hops in a row report no signal.
    (The MSE gate lets noise through at times, as in the reference.)"""
    pcm = np.random.default_rng(7).normal(0, 3000, 48000 * 6).astype(np.int16)
    o = tl.Oracle()
    o.push_chunked(pcm, 12000)
    h = o.hops()
    centers = h[:, 3]
    assert centers[0] == 0.0
    # hunter steps: after 15 consecutive no-signal hops the centre moves to a
    # multiple of 5250 Hz (AFC may also move it while the MSE gate is open)
    hunted = [k for k in range(15, len(h)) if np.all(h[k - 14:k + 1, 5] == 0.0) and centers[k] != centers[k - 1]]
    assert hunted, 'hunter never stepped'
    for k in hunted:
        assert centers[k] % 5250.0 == 0.0
