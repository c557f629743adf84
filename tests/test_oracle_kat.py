"""The oracle against the known-answer values measured by compiling the
reference's own classes."""
import ctypes

import numpy as np

import aero_testlib as tl


def test_crc16_x25(cpu_libs):
    L = tl.Oracle.lib()
    b = np.frombuffer(b'123456789', dtype=np.uint8).copy()
    assert L.oracle_crc16_bytes(b.ctypes.data, 9) == 0x906E   # AeroLcrc16::calcusingbytes


def test_scrambler_prefix(cpu_libs):
    L = tl.Oracle.lib()
    bits = np.zeros(5000, dtype=np.int32)
    L.oracle_scrambler_bits(bits.ctypes.data, 5000)
    assert ''.join(map(str, bits[:64])) == \
        '0001001100011011110001000010010100001111100011000001010111101111'
    assert int(bits[64:5000].sum()) == 2485


def test_deinterleaver_kat(cpu_libs):
    L = tl.Oracle.lib()
    idx = np.zeros(64 * 78, dtype=np.int32)
    L.oracle_deinterleave_perm(78, idx.ctypes.data)
    assert list(idx[:8] % 256) == [0, 58, 116, 46, 104, 34, 92, 150]
    assert sorted(idx) == list(range(64 * 78))


def test_rrc_design_kat(cpu_libs):
    L = tl.Oracle.lib()
    p = np.zeros(64)
    L.oracle_rrc_design(1.0, 55, 48000.0, 5250.0, p.ctypes.data)
    taps = p[:55]
    assert taps[0] == -0.0029086670661150099
    assert taps[27] == 0.4210843993477924
    assert abs(taps.sum() - 3.0241558898789509) < 1e-15


def test_cis_table_kat(cpu_libs):
    L = tl.Oracle.lib()
    t = np.zeros(2 * 19999)
    L.oracle_cis_table(t.ctypes.data)
    assert t[2] == 0.99999995064704328 and t[3] == 0.00031417496893919669


def test_fft_is_jfft_dft(cpu_libs):
    """JFFT restatement computes the DFT (forward) and scaled inverse."""
    L = tl.Oracle.lib()
    r = np.random.default_rng(3)
    x = r.normal(size=1024) + 1j * r.normal(size=1024)
    buf = np.ascontiguousarray(x.astype(np.complex128))
    L.oracle_fft(buf.ctypes.data, 1024, 0)
    assert np.allclose(buf, np.fft.fft(x), atol=1e-9)
    L.oracle_fft(buf.ctypes.data, 1024, 1)
    assert np.allclose(buf, x, atol=1e-12)
