"""The engine's host-side C++ on the CPU (tools/hostcheck.cpp over
aero-cli_amd/csrc/acars_host.cpp and tables_host.cpp, no GPU):

* PChannelHost fed the oracle's CRC-checked P-channel frames (AeroL::Decode's
  SU dispatch, ISUData, ParserISU, ACARSDefragmenter, decode/aerol.cpp:
  158-524, 1571-1965) and burst R/T packets (aerol.cpp:1253-1460) produces
  the oracle's ACARS items (reassembled, and fragments with
  --disable-reassembly);
* the tables the kernels read, built on the host (CIS, JFFT twiddles, RRC,
  MSK matched filter, scrambler, the aero-publish low-pass / Hilbert /
  oscillator designs), equal the oracle's bit for bit.

scripts/asan_check.sh runs this file (with the oracle and host tests) against
AddressSanitizer + UBSan builds of the same sources."""
import ctypes
import os

import numpy as np
import pytest

import aero_testlib as tl
import aero_engine as ae

SO = os.environ.get('AERO_HOSTCHECK_SO') or os.path.join(tl.ROOT, 'tools', 'libaero_hostcheck.so')


@pytest.fixture(scope='module')
def hc():
    if not os.environ.get('AERO_HOSTCHECK_SO'):
        import build
        build.build_hostcheck()
    L = ctypes.CDLL(SO)
    L.hc_create.restype = ctypes.c_void_p
    L.hc_destroy.argtypes = [ctypes.c_void_p]
    L.hc_frame.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_int]
    L.hc_rt_packet.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    L.hc_items.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.hc_items.restype = ctypes.c_size_t
    L.hc_rrc.restype = ctypes.c_int
    L.hc_pub_low_pass.restype = ctypes.c_int
    L.hc_pub_osc_len.restype = ctypes.c_int
    L.hc_pub_low_pass.argtypes = [ctypes.c_double] * 4 + [ctypes.c_void_p, ctypes.c_int]
    L.hc_rrc.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
    L.hc_pub_osc_len.argtypes = [ctypes.c_double]
    L.hc_pub_osc.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
    L.hc_pub_hilbert.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return L


def _items(L, h):
    arr = (ae.AcarsItem * 256)()
    out = []
    while True:
        n = L.hc_items(h, arr, 256)
        out += [ae.item_line(arr[i]) for i in range(n)]
        if n < 256:
            return out


@pytest.mark.parametrize('bitrate,seed', [(10500, 0xAE20), (10500, 0xAE23), (600, 0xAE40)])
def test_pchannel_items_from_oracle_frames(hc, bitrate, seed):
    if bitrate == 10500:
        pcm = tl.synth(seconds=20.0, seed=seed)
    else:
        pcm = tl.synth_msk(seconds=40.0, bitrate=600, baud=600, seed=seed, ebn0=14.0)
    o = tl.Oracle(bitrate=bitrate)
    o.push_chunked(pcm, 6000)
    frames = tl.frame_records(o.frames())
    assert len(frames) > 5
    for disable in (0, 1):  # reassembled messages; fragments as they arrive (--disable-reassembly)
        h = hc.hc_create(disable)
        for info, mask in frames:
            hc.hc_frame(h, info, len(info), mask, 1)
        got = _items(hc, h)
        hc.hc_destroy(h)
        ref = o.item_lines('F' if disable else 'A')
        assert ref and got == ref, disable


def test_burst_rt_items_from_oracle_packets(hc):
    pcm = tl.synth_burst(seconds=30.0, seed=3, carrier=12000.0, ebn0=14.0)
    o = tl.Oracle(burst=True)
    o.push_chunked(pcm, 12000)
    pk = o.rt_packets()
    assert len(pk) >= 3
    for disable in (0, 1):
        h = hc.hc_create(disable)
        for kind, info in pk:
            nsus = max(0, (len(info) + 1 - 6) // 12) if kind == 'T' else 0
            hc.hc_rt_packet(h, int(kind == 'R'), info, len(info), nsus)
        got = _items(hc, h)
        hc.hc_destroy(h)
        ref = o.item_lines('F' if disable else 'A')
        assert ref and got == ref, disable


def _u(a):
    return np.ascontiguousarray(a).view(np.uint64 if a.dtype == np.float64 else np.uint32)


def test_tables_equal_oracle(hc):
    O = tl.Oracle.lib()
    a, b = np.zeros(19999 * 2), np.zeros(19999 * 2)
    hc.hc_cis(a.ctypes.data_as(ctypes.c_void_p))
    O.oracle_cis_table(b.ctypes.data_as(ctypes.c_void_p))
    assert np.array_equal(_u(a), _u(b))
    for nfft in (8192, 16384):
        tw, twi, r, ri = (np.zeros(2 * nfft) for _ in range(4))
        hc.hc_twiddles(nfft, tw.ctypes.data_as(ctypes.c_void_p), twi.ctypes.data_as(ctypes.c_void_p))
        O.oracle_twiddles(nfft, 0, r.ctypes.data_as(ctypes.c_void_p))
        O.oracle_twiddles(nfft, 1, ri.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(_u(tw), _u(r)) and np.array_equal(_u(twi), _u(ri)), nfft
    for alpha, n, fs, sf in ((1.0, 55, 48000.0, 5250.0), (0.35, 81, 48000.0, 5250.0), (0.6, 111, 24000.0, 1200.0)):
        p, q = np.zeros(n), np.zeros(n)
        m = hc.hc_rrc(alpha, n, fs, sf, p.ctypes.data_as(ctypes.c_void_p))
        O.oracle_rrc_design(ctypes.c_double(alpha), n, ctypes.c_double(fs), ctypes.c_double(sf),
                            q.ctypes.data_as(ctypes.c_void_p))
        assert m == n and np.array_equal(_u(p), _u(q)), (alpha, n)
    for sps in (20, 40, 80):
        p, q = np.zeros(2 * sps), np.zeros(2 * sps)
        hc.hc_msk_taps(sps, p.ctypes.data_as(ctypes.c_void_p))
        O.oracle_msk_taps(sps, q.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(_u(p), _u(q)), sps
    s8, si = np.zeros(5000, np.uint8), np.zeros(5000, np.int32)
    hc.hc_scrambler(s8.ctypes.data_as(ctypes.c_void_p))
    O.oracle_scrambler_bits(si.ctypes.data_as(ctypes.c_void_p), 5000)
    assert np.array_equal(s8.astype(np.int32), si)


def test_channeliser_designs_equal_oracle(hc):
    O = tl.Oracle.lib()
    O.oracle_pub_low_pass.restype = ctypes.c_int
    for gain, fs, cut, tw in ((1.0, 192000.0, 5000.0, 2000.0), (1.0, 48000.0, 6000.0, 1000.0)):
        a, b = np.zeros(4096, np.float32), np.zeros(4096, np.float32)
        n = hc.hc_pub_low_pass(gain, fs, cut, tw, a.ctypes.data_as(ctypes.c_void_p), 4096)
        m = O.oracle_pub_low_pass(ctypes.c_double(gain), ctypes.c_double(fs), ctypes.c_double(cut),
                                  ctypes.c_double(tw), b.ctypes.data_as(ctypes.c_void_p), 4096)
        assert n == m > 0 and np.array_equal(_u(a[:n]), _u(b[:m]))
    for ln, fs in ((255, 48000), (511, 12000)):
        a, b = np.zeros(ln, np.float32), np.zeros(ln, np.float32)
        hc.hc_pub_hilbert(ln, fs, a.ctypes.data_as(ctypes.c_void_p))
        O.oracle_pub_hilbert(ln, fs, b.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(_u(a), _u(b)), ln
    for fs, f in ((48000.0, 12000.0), (1536000.0, -250000.0)):
        n = hc.hc_pub_osc_len(fs)
        a, b = np.zeros(2 * n, np.float32), np.zeros(2 * int(fs), np.float32)
        hc.hc_pub_osc(fs, f, a.ctypes.data_as(ctypes.c_void_p))
        O.oracle_pub_osc(ctypes.c_double(fs), ctypes.c_double(f), b.ctypes.data_as(ctypes.c_void_p))
        assert n == int(fs) and np.array_equal(_u(a), _u(b[:2 * n])), fs
