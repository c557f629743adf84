"""The oracle against the reference itself, where the reference's path
compiles without Qt or other external libraries: decode/jfft.cpp (JFFT, the
coarse estimator's transforms; its real FFT, the burst trident check's
FFTrWrapper; JFastFir, the burst front end's Hilbert filter) and
publish/oscillator.cpp (the channeliser's mixer), built from /root/reference into oracle/_ref/libref.so by
oracle/Makefile's `ref` target (oracle/ref_shim.cpp is the C ABI over them).
Bit-exact comparisons on seeded inputs.  The reference tree exists only in
the build container: without it these tests skip (the GPU box never has it)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import aero_testlib as tl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, 'oracle', '_ref', 'libref.so')
REFERENCE = '/root/reference'


@pytest.fixture(scope='module')
def ref():
    if not os.path.isdir(REFERENCE):
        pytest.skip('reference tree not present (GPU box)')
    subprocess.run(['make', '-s', '-C', os.path.join(ROOT, 'oracle'), 'ref'], check=True, capture_output=True)
    L = ctypes.CDLL(REF_SO)
    L.ref_jfft.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.ref_osc.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_void_p, ctypes.c_int]
    L.ref_fft_real.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.ref_fastfir.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return L


def _oracle(cpu_libs):
    L = tl.Oracle.lib()
    L.oracle_fft.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.oracle_pub_osc.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
    L.oracle_fftr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.oracle_hilbert.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    return L


@pytest.mark.parametrize('nfft', [8192, 16384])
@pytest.mark.parametrize('inverse', [0, 1])
def test_jfft_matches_reference(ref, cpu_libs, nfft, inverse):
    O = _oracle(cpu_libs)
    rng = np.random.default_rng(nfft + inverse)
    for trial in range(3):
        # the coarse estimator's inputs: CIS * pcm / 32768 (trial 0), wide-range values (1, 2)
        if trial == 0:
            ang = rng.uniform(0, 2 * np.pi, nfft)
            pcm = rng.integers(-32768, 32768, nfft) / 32768.0
            x = np.empty(2 * nfft)
            x[0::2], x[1::2] = np.cos(ang) * pcm, np.sin(ang) * pcm
        else:
            x = rng.standard_normal(2 * nfft) * 10.0 ** rng.uniform(-6, 6, 2 * nfft)
        a, b = x.copy(), x.copy()
        O.oracle_fft(a.ctypes.data, nfft, inverse)
        ref.ref_jfft(b.ctypes.data, nfft, inverse)
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), 'JFFT differs from the reference'


@pytest.mark.parametrize('fs,freq', [(48000.0, 10500.0), (192000.0, -37000.0), (1536000.0, 123456.5),
                                     (96000.0, 0.0)])
def test_oscillator_matches_reference(ref, cpu_libs, fs, freq):
    O = _oracle(cpu_libs)
    L = int(fs)
    q = np.zeros(2 * L, dtype=np.float32)
    O.oracle_pub_osc(fs, freq, q.ctypes.data)          # the oracle's queue[0 .. L-1]
    seq = np.zeros(2 * (L + 1), dtype=np.float32)
    ref.ref_osc(fs, freq, seq.ctypes.data, L + 1)       # _vector before ticks 0 .. L
    # the reference's _vector: queue[L-1] after construction, then queue[1], queue[2], ..., queue[0]
    want = np.empty(2 * L, dtype=np.float32)
    want[2:] = seq[2:2 * L]                  # queue[1 .. L-1]
    want[0:2] = seq[2 * L:2 * L + 2]         # queue[0] (after L ticks)
    assert np.array_equal(q.view(np.uint32), want.view(np.uint32))
    assert np.array_equal(seq[0:2].view(np.uint32), q[2 * L - 2:].view(np.uint32))


@pytest.mark.parametrize('n', [32768, 16384, 8192])
def test_fft_real_matches_reference(ref, cpu_libs, n):
    """FFTr (the burst trident check's FFTrWrapper<double>(32768),
    decode/fftrwrapper.cpp:13-23) against the reference's JFFT::fft_real
    (decode/jfft.cpp:54-76) with FFTrWrapper's kissfft zeroing of the upper
    half applied to the reference output."""
    O = _oracle(cpu_libs)
    rng = np.random.default_rng(n)
    for trial in range(3):
        if trial == 0:  # the trident buffer: |analytic sample| values of a burst, >= 0
            x = np.abs(rng.standard_normal(n)) * rng.uniform(0.01, 3.0)
        else:
            x = rng.standard_normal(n) * 10.0 ** rng.uniform(-6, 6, n)
        a = np.zeros(2 * n)
        b = np.zeros(2 * n)
        O.oracle_fftr(x.ctypes.data, a.ctypes.data, n)
        ref.ref_fft_real(x.ctypes.data, b.ctypes.data, n)
        b[2 * (n // 2 + 1):] = 0.0  # fftrwrapper.cpp:19-22
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), 'real FFT differs from the reference'


def test_hilbert_fastfir_matches_reference(ref, cpu_libs):
    """The oracle's HilbertFir (overlap-add fast convolution, 8192-point
    blocks) against the reference's JFastFir::update (decode/jfft.cpp:322-495)
    with the same 2048 taps (the taps restate QJHilbertFilter::setSize,
    decode/DSP.cpp:732-759, which is Qt code and not built)."""
    O = _oracle(cpu_libs)
    rng = np.random.default_rng(0x4B)
    n = 3 * 6145 + 777  # several overlap-add blocks and a partial one
    x = np.empty(2 * n)
    x[0::2] = rng.integers(-32768, 32768, n) / 32768.0
    x[1::2] = 0.0  # the burst front end filters the real PCM
    x[2 * 5000:2 * 5100] = 0.0  # a stretch of silence
    a = np.zeros(2 * n)
    k = np.zeros(2 * 2048)
    O.oracle_hilbert(x.ctypes.data, a.ctypes.data, n, k.ctypes.data)
    b = np.zeros(2 * n)
    ref.ref_fastfir(k.ctypes.data, 2048, x.ctypes.data, b.ctypes.data, n)
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), 'Hilbert fast FIR differs from the reference'
