"""The C ABI library loads on a CPU-only host, exports every symbol that
include/aero_engine.h and include/aero_chan.h declare, and fails cleanly
without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import aero_testlib as tl

HEADERS = [os.path.join(tl.ROOT, 'include', h) for h in ('aero_engine.h', 'aero_chan.h')]


def _declared():
    src = ''.join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r'\b(aero_[a-z_]+)\s*\(', src)))


def test_library_exports_header_symbols(engine_lib):
    import aero_engine
    names = _declared()
    assert 'aero_push_pcm' in names and 'aero_pop_items' in names and 'aero_chan_feed' in names
    for n in names:
        assert hasattr(engine_lib, n), n
        assert n in aero_engine._SIGS, 'python mirror lacks ' + n


def test_create_without_gpu_is_an_error_not_a_crash(engine_lib):
    import aero_engine
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip('GPU present')
    except ImportError:
        pass
    with pytest.raises(aero_engine.AeroError) as ei:
        aero_engine.Engine(4)
    assert ei.value.rc == aero_engine.AERO_E_NOGPU


def test_item_struct_layout():
    import aero_engine
    assert ctypes.sizeof(aero_engine.AcarsItem) == 4 + 16 + 4 + 16 + 4 + 3584


def test_engine_tables_match_oracle(engine_lib, cpu_libs):
    """Host tables the engine uploads == the oracle's (same glibc calls)."""
    L = engine_lib
    cis = np.zeros(2 * 19999)
    tw = np.zeros(2 * 16384)
    twi = np.zeros(2 * 16384)
    taps = np.zeros(64)
    n = ctypes.c_int()
    L.aero_host_tables(cis.ctypes.data_as(ctypes.c_void_p), tw.ctypes.data_as(ctypes.c_void_p),
                       twi.ctypes.data_as(ctypes.c_void_p), taps.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n))
    O = tl.Oracle.lib()
    ocis = np.zeros_like(cis)
    O.oracle_cis_table(ocis.ctypes.data)
    otw = np.zeros_like(tw)
    otwi = np.zeros_like(twi)
    O.oracle_twiddles(16384, 0, otw.ctypes.data)
    O.oracle_twiddles(16384, 1, otwi.ctypes.data)
    otaps = np.zeros(64)
    O.oracle_rrc_design(1.0, 55, 48000.0, 5250.0, otaps.ctypes.data)
    assert n.value == 55
    for a, b in ((cis, ocis), (tw, otw), (twi, otwi), (taps, otaps)):
        assert np.array_equal(a.view(np.int64), b.view(np.int64))


@pytest.mark.parametrize('sps', [20, 40])
def test_engine_msk_tables_match_oracle(engine_lib, cpu_libs, sps):
    """MSK group tables (8192-point twiddles, 2*sps-tap half-sine matched
    filter, decode/mskdemodulator.cpp:126-133) == the oracle's."""
    L = engine_lib
    tw, twi, taps = np.zeros(2 * 8192), np.zeros(2 * 8192), np.zeros(2 * sps)
    L.aero_host_msk_tables(ctypes.c_int(sps), tw.ctypes.data_as(ctypes.c_void_p), twi.ctypes.data_as(ctypes.c_void_p),
                           taps.ctypes.data_as(ctypes.c_void_p))
    O = tl.Oracle.lib()
    otw, otwi, otaps = np.zeros_like(tw), np.zeros_like(twi), np.zeros_like(taps)
    O.oracle_twiddles(8192, 0, otw.ctypes.data)
    O.oracle_twiddles(8192, 1, otwi.ctypes.data)
    O.oracle_msk_taps(sps, otaps.ctypes.data)
    for a, b in ((tw, otw), (twi, otwi), (taps, otaps)):
        assert np.array_equal(a.view(np.int64), b.view(np.int64))


def test_twiddle_inverse_is_conjugate(cpu_libs):
    """JFFT's inverse twiddles are the forward ones conjugated, bit for bit
    (mirrored std::exp arguments, decode/jfft.cpp:41-53)."""
    O = tl.Oracle.lib()
    for n in (8192, 16384):
        tw, twi = np.zeros(2 * n), np.zeros(2 * n)
        O.oracle_twiddles(n, 0, tw.ctypes.data)
        O.oracle_twiddles(n, 1, twi.ctypes.data)
        used = 2 * (n - 1)  # JFFT::init fills n - 1 entries (stages 2 .. n)
        assert np.array_equal(tw[0:used:2].view(np.int64), twi[0:used:2].view(np.int64))
        assert np.array_equal((-tw[1:used:2]).view(np.int64), twi[1:used:2].view(np.int64))


@pytest.mark.parametrize('fs,f', [(1536000, 300000.0), (192000, -20000.0), (288000, 0.0)])
def test_chan_oscillator_matches_oracle(engine_lib, cpu_libs, fs, f):
    """Channeliser NCO queue (publish/oscillator.cpp:4-28) == the oracle's."""
    a, b = np.zeros(2 * fs, dtype=np.float32), np.zeros(2 * fs, dtype=np.float32)
    engine_lib.aero_host_pub_osc(ctypes.c_double(fs), ctypes.c_double(f), a.ctypes.data_as(ctypes.c_void_p))
    tl.OraclePublisher.lib().oracle_pub_osc(fs, f, b.ctypes.data)
    assert np.array_equal(a.view(np.int32), b.view(np.int32))


@pytest.mark.parametrize('args', [(2, 240000, 24000, 12000.0), (2, 12000, 3000, 750.0), (2, 288000, 24000, 9600.0)])
def test_chan_filter_designs_match_oracle(engine_lib, cpu_libs, args):
    """firfilter::low_pass (publish/firfilter.cpp:47-99) and FIRHilbert
    (publish/dsp.cpp:181-215) designs == the oracle's."""
    a, b = np.zeros(4096, dtype=np.float32), np.zeros(4096, dtype=np.float32)
    f = engine_lib.aero_host_pub_low_pass
    f.restype = ctypes.c_int
    na = f(*[ctypes.c_double(v) for v in args], a.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(4096))
    nb = tl.OraclePublisher.lib().oracle_pub_low_pass(*args, b.ctypes.data, 4096)
    assert na == nb > 0 and np.array_equal(a[:na].view(np.int32), b[:nb].view(np.int32))
    h1, h2 = np.zeros(125, dtype=np.float32), np.zeros(125, dtype=np.float32)
    engine_lib.aero_host_pub_hilbert(ctypes.c_int(125), ctypes.c_int(12000), h1.ctypes.data_as(ctypes.c_void_p))
    tl.OraclePublisher.lib().oracle_pub_hilbert(125, 12000, h2.ctypes.data)
    assert np.array_equal(h1.view(np.int32), h2.view(np.int32))
