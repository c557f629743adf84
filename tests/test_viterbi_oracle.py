"""libcorrect-convention Viterbi restatement: behavioural pins (the library
itself is absent, SURVEY.md Appendix D -> parity unpinned)."""
import numpy as np

import aero_testlib as tl


def _encode(msg):
    L = tl.Oracle.lib()
    enc = np.zeros(2 * (len(msg) + 1) + 8, dtype=np.uint8)
    nbits = L.oracle_conv_encode(msg.ctypes.data, len(msg), enc.ctypes.data)
    bits = np.unpackbits(enc)[:nbits]
    return bits


def _decode(soft):
    L = tl.Oracle.lib()
    out = np.zeros(len(soft) // 16 + 8, dtype=np.uint8)
    L.oracle_viterbi_decode_soft(np.ascontiguousarray(soft, dtype=np.uint8).ctypes.data, len(soft),
                                 out.ctypes.data)
    return out


def test_roundtrip_clean(cpu_libs):
    r = np.random.default_rng(1)
    msg = r.integers(0, 256, 400, dtype=np.uint8)
    bits = _encode(msg)
    soft = (bits * 255).astype(np.uint8)
    assert np.array_equal(_decode(soft)[:400], msg)


def test_roundtrip_noisy(cpu_libs):
    r = np.random.default_rng(2)
    msg = r.integers(0, 256, 400, dtype=np.uint8)
    bits = _encode(msg)
    x = (2.0 * bits - 1.0) + r.normal(0, 0.5, bits.size)
    soft = np.clip(np.round(x * 0.75 * 127 + 128), 0, 255).astype(np.uint8)
    assert np.array_equal(_decode(soft)[:400], msg)


def test_erasures_are_tolerated(cpu_libs):
    r = np.random.default_rng(3)
    msg = r.integers(0, 256, 300, dtype=np.uint8)
    soft = (_encode(msg) * 255).astype(np.uint8)
    soft[::7] = 128
    assert np.array_equal(_decode(soft)[:300], msg)
