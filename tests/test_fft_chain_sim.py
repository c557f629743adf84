"""The coarse kernel's chained-FFT index arithmetic on the CPU
(aero-cli_amd/csrc/fft_layout.h, modelled lane by lane in
tools/fft_chain_sim.cpp): the three transforms of CoarseFreqEstimate
(forward, boxcar, inverse, square, forward; decode/coarsefreqestimate.cpp:
134-160) through the register stages, the wave-local LDS transpose, the
v_permlane16/32_swap steps and the G exchange equal the oracle's JFFT chain
(decode/jfft.cpp:114-212) value for value, up to the sign of exact zeros
(the kernel skips the exact (1, +-0) twiddle products), with
the G-layout stages past the LDS twiddles reading the permuted copy the
kernel reads (fft_layout.h twg_build)."""
import ctypes
import os

import numpy as np
import pytest

import aero_testlib as tl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIM = os.path.join(ROOT, 'tools', 'libfft_chain_sim.so')


def _sim():
    L = ctypes.CDLL(SIM)
    L.fft_chain_sim.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return L


@pytest.mark.parametrize('log2n,start,stop', [(14, 3584, 12800), (13, 614, 7578), (13, 307, 7885)])
def test_chain_matches_jfft(log2n, start, stop, cpu_libs):
    n = 1 << log2n
    O = tl.Oracle.lib()
    tw = np.zeros(2 * n)
    twi = np.zeros(2 * n)
    O.oracle_twiddles(n, 0, tw.ctypes.data)
    O.oracle_twiddles(n, 1, twi.ctypes.data)
    rng = np.random.default_rng(log2n)
    # coarse-estimator-like input: CIS * pcm / 32768, some leading zeros
    cis = np.exp(1j * rng.uniform(0, 2 * np.pi, n))
    pcm = rng.integers(-32768, 32767, n) / 32768.0
    pcm[:100] = 0
    x = (cis * pcm).astype(np.complex128)
    out = np.zeros(n, dtype=np.complex128)
    assert _sim().fft_chain_sim(log2n, tw.ctypes.data, twi.ctypes.data, x.ctypes.data, start, stop,
                                out.ctypes.data) == 0
    ref = x.copy()
    O.oracle_fft(ref.ctypes.data, n, 0)
    ref[start:stop + 1] = 0
    O.oracle_fft(ref.ctypes.data, n, 1)
    ref = ref * n  # FFTWrapper: x 1/N in JFFT, then x N (exact here)
    re, im = ref.real.copy(), ref.imag.copy()  # x * x as GCC expands it (numpy's complex product may fuse)
    ref = np.empty(n, dtype=np.complex128)
    ref.real, ref.imag = re * re - im * im, re * im + im * re
    O.oracle_fft(ref.ctypes.data, n, 0)
    assert np.array_equal(out.real, ref.real) and np.array_equal(out.imag, ref.imag)
