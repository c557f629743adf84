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


@pytest.mark.parametrize('sps', [20, 25, 26, 31, 40, 66, 80, 160])
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


def _msk_consts(L, fs):
    iv = (ctypes.c_int * 9)()
    dv = (ctypes.c_double * 8)()
    rc = L.aero_x_msk_rate_consts(ctypes.c_int(fs), iv, dv)
    return rc, list(iv), list(dv)


# coarse.hip MskCoarseBins<Fs> (the fixed-rate kernels' compile-time bins):
# START, STOP, ILO, IHI, EPB
FIXED_BINS = {12000: (614, 7578, 3482, 4710, 205), 24000: (307, 7885, 3789, 4403, 102),
              48000: (154, 8038, 3942, 4250, 51)}


@pytest.mark.parametrize('fs', sorted(FIXED_BINS))
def test_generic_msk_constants_equal_fixed_rate_ones(engine_lib, fs):
    """The host computation the generic-rate MSK groups run with
    (engine.hip msk_gen_consts: CoarseFreqEstimate::setSettings(13, 900, 600,
    Fs), decode/coarsefreqestimate.cpp:39-76, and MskDemodulator::setSettings,
    decode/mskdemodulator.cpp:94-218) gives, at the three compiled rates, the
    constants the compiled kernels were built with."""
    rc, iv, dv = _msk_consts(engine_lib, fs)
    assert rc == 0
    sps, d8_old, d8_new, start, stop, ilo, ihi, epb, d8_len = iv
    assert (start, stop, ilo, ihi, epb) == FIXED_BINS[fs]
    assert sps == fs // 600 and (d8_old, d8_new) == (sps // 2, sps // 2 - 1) and d8_len == sps // 2 + 1
    f48 = fs == 48000
    assert dv[1:6] == ([1.308825621597620e-04, -1.308825621597620e-04, -1.998196509168551, 0.999738234875681, 0.025]
                       if f48 else
                       [5.233248111921052e-04, -5.233248111921052e-04, -1.974342917561558, 0.998953350377616, 0.0125])


def test_generic_msk_constants_at_other_rates(engine_lib):
    """Rates without a compiled kernel: an odd SPS gives delayt8 a half-sample
    delay (ages ceil / floor of SPS/2, weights 0.5 / 0.5, DSP.h:358-384); the
    fold search stays inside the y bins every MSK group keeps; rates outside
    [12000, 96000] are refused."""
    for fs in (15000, 16000, 18750, 22050, 40000, 96000):
        rc, iv, dv = _msk_consts(engine_lib, fs)
        assert rc == 0, fs
        sps, d8_old, d8_new, start, stop, ilo, ihi, epb, d8_len = iv
        assert sps == fs // 600
        if sps % 2:
            assert (d8_old, d8_new, d8_len) == (sps // 2 + 1, sps // 2, sps // 2 + 2) and dv[6:8] == [0.5, 0.5]
        else:
            assert (d8_old, d8_new, d8_len) == (sps // 2, sps // 2 - 1, sps // 2 + 1)
        hz = fs / 8192.0
        assert start == max(round(900 / hz), 1) and stop == 8192 - start and epb == round(600 / (2 * hz))
        assert 3276 <= ilo - epb - 1 and ihi + epb <= 4915  # MSK_YLO / MSK_YHI
    for fs in (11025, 8000, 96001, 192000):
        assert _msk_consts(engine_lib, fs)[0] == -6  # AERO_E_RATE
