"""Committed fixtures in tests/golden/ (written by tests/golden/make_golden.py):
the oracle against SURVEY.md Appendix B's known answers (measured on the
reference's own classes), the oracle against its regression digests, and
(-m gpu) the HIP engine against the same digests through the C ABI."""
import hashlib
import json
import os

import numpy as np
import pytest

import aero_testlib as tl

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_appendix_b_fixture(cpu_libs):
    k = _load('appendix_b_kat.json')
    L = tl.Oracle.lib()
    b = np.frombuffer(k['crc16_x25']['input'].encode(), dtype=np.uint8).copy()
    assert L.oracle_crc16_bytes(b.ctypes.data, len(b)) == k['crc16_x25']['calcusingbytes']
    bits = np.zeros(5000, dtype=np.int32)
    L.oracle_scrambler_bits(bits.ctypes.data, 5000)
    assert ''.join(map(str, bits[:64])) == k['scrambler']['first64']
    assert int(bits[64:].sum()) == k['scrambler']['ones_64_5000']
    idx = np.zeros(64 * 78, dtype=np.int32)
    L.oracle_deinterleave_perm(78, idx.ctypes.data)
    assert list(idx[:8] % 256) == k['deinterleaver_78']['first8_mod256']
    p = np.zeros(64)
    L.oracle_rrc_design(*k['rrc_design']['args'], p.ctypes.data)
    assert p[0] == k['rrc_design']['p0'] and p[27] == k['rrc_design']['p27']
    assert abs(p[:55].sum() - k['rrc_design']['sum']) < 1e-15
    t = np.zeros(2 * k['ciswt1']['wtsize'])
    L.oracle_cis_table(t.ctypes.data)
    assert t[2] == k['ciswt1']['re'] and t[3] == k['ciswt1']['im']


def _stream(s):
    if s['kind'] == 'oqpsk10500':
        return tl.synth(seconds=s['seconds'], seed=s['seed'], carrier=s['carrier'], ebn0=s['ebn0']), 10500, 48000
    return (tl.synth_msk(seconds=s['seconds'], bitrate=600, seed=s['seed'], carrier=s['carrier'], ebn0=s['ebn0']),
            600, 12000)


def _digests(soft, items):
    return hashlib.sha256(np.asarray(soft, dtype=np.uint8).tobytes()).hexdigest(), \
        hashlib.sha256('\n'.join(items).encode()).hexdigest()


@pytest.mark.parametrize('k', range(3))
def test_oracle_regression_fixture(cpu_libs, k):
    s = _load('oracle_regression.json')[k]
    pcm, rate, _ = _stream(s)
    o = tl.Oracle(bitrate=rate)
    o.push_chunked(pcm, s['chunk'])
    soft, items = o.softbits(), o.item_lines('A')
    assert len(soft) == s['n_soft'] and len(items) == s['n_items'] > 0
    assert _digests(soft, items) == (s['soft_sha256'], s['items_sha256'])


@pytest.mark.gpu
def test_engine_matches_golden_digests(engine_lib, cpu_libs):
    import aero_engine as ae
    fx = _load('oracle_regression.json')
    eng = ae.Engine(max_channels=len(fx), flags=ae.F_TRACE_SOFT)
    chans, streams = [], []
    for s in fx:
        pcm, rate, fs = _stream(s)
        chans.append(eng.open_channel(rate, fs))
        streams.append(pcm)
    pos = [0] * len(fx)
    while any(p < len(x) for p, x in zip(pos, streams)):
        for k, s in enumerate(fx):
            if pos[k] < len(streams[k]):
                eng.push(chans[k], streams[k][pos[k]:pos[k] + s['chunk']])
                pos[k] += s['chunk']
        eng.run()
    eng.flush()
    for ch, s in zip(chans, fx):
        soft, items = eng.softbits(ch), eng.items(ch)
        assert len(soft) == s['n_soft'] and len(items) == s['n_items']
        assert _digests(soft, items) == (s['soft_sha256'], s['items_sha256'])
    eng.close()
