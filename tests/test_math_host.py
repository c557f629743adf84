"""aero_math.h (the device libm) compiled for the host vs glibc 2.35, the
library the reference links: every function bit-exact.  hypot and tanh are
glibc's SSE2 code; atan2 and log restate the __atan2_fma / __log_fma
instruction sequences the ifunc selects on this (FMA + AVX2) host; sincos
is glibc's SSE2 sincos, which the reference's cos(x)/sin(x) pairs and
std::exp(i x) reach.  Inputs cover the demods' argument ranges (loop
corrections, phase errors, |X| of the coarse FFT) and every branch of the
restated code (table rows, small-ratio series, quadrants, the range
reduction, near-1 log, extreme exponents)."""
import numpy as np
import pytest

pytestmark = pytest.mark.filterwarnings('ignore::RuntimeWarning')

import mathhost


def _inputs(n=1000000, seed=11):
    r = np.random.default_rng(seed)
    a = r.uniform(-1, 1, n) * np.exp(r.normal(0, 2, n))
    b = r.uniform(-1, 1, n) * np.exp(r.normal(0, 2, n))
    return a, b


def _same(fn, x, y=None):
    h = mathhost.evaluate(fn, x, y).view(np.int64)
    g = mathhost.glibc(fn, x, y).view(np.int64)
    bad = np.flatnonzero(h != g)
    assert bad.size == 0, (fn, bad.size, x[bad[:3]], None if y is None else y[bad[:3]])


@pytest.mark.parametrize('fn', ['hypot', 'tanh', 'atan2'])
def test_bit_exact_generic(fn):
    a, b = _inputs()
    _same(fn, a, b)


def test_atan2_every_branch():
    rng = np.random.default_rng(3)
    n = 400_000
    x = rng.standard_normal(n)
    cases = [
        x * (1 + rng.standard_normal(n) * 1e-9),                               # |y/x| near 1
        x * rng.uniform(0, 1 / 16, n),                                         # the small-ratio series
        x * rng.uniform(1 / 16 - 1e-6, 1 / 16 + 1e-6, n),                      # its edge
        x * (rng.integers(16, 257, n) / 256) * (1 + rng.standard_normal(n) * 1e-12),  # table rows' centres
        rng.standard_normal(n) * np.exp(rng.uniform(-745, 709, n)),            # extreme ratios, scaling, inf
    ]
    for y in cases:
        _same('atan2', y, x)
        _same('atan2', x, y)
        _same('atan2', -y, -x)


@pytest.mark.parametrize('scale', [1e-9, 0.1, 0.25, 0.86, 2.43, 2.0, 7.0, 40.0, 1e5, 1e8])
def test_sincos_bit_exact(scale):
    """Both outputs of sincos over the ranges of s_sincos.c's branches:
    tiny, |x| < 0.855 (Taylor below 0.126), pi/2 - |x| up to 2.43, the
    Cody-Waite reduction up to 105414350."""
    rng = np.random.default_rng(int(scale * 1000) % 2 ** 31)
    x = rng.uniform(-scale, scale, 400_000)
    _same('sincos_s', x)
    _same('sincos_c', x)


def test_sincos_huge_arguments_bit_exact():
    """|x| >= 105414350: sincos reduces through __branred (g_branred, restated
    from libm's SSE2 build with its 2/pi digit table read out of libm):
    log-uniform over the whole finite range, both signs, the threshold, powers
    of two, integers around 2^52..2^53, the largest doubles."""
    rng = np.random.default_rng(41)
    n = 1_000_000
    x = rng.choice([-1.0, 1.0], n) * np.exp2(rng.uniform(np.log2(105414350.0), 1023.0, n)) * rng.uniform(1, 1.99, n)
    edge = np.array([105414350.0, -105414350.0, 105414351.0, 2.0 ** 27, 2.0 ** 30, 2.0 ** 52, 2.0 ** 53 + 2,
                     281474976710656.0, 1e22, 1e100, 2.0 ** 1000, 1.7976931348623157e308, -1.7976931348623157e308])
    for xs in (x, edge, np.round(rng.uniform(2.0 ** 52, 2.0 ** 53, n))):
        _same('sincos_s', xs)
        _same('sincos_c', xs)


def test_log_and_log10_bit_exact():
    rng = np.random.default_rng(11)
    for x in (np.exp(rng.uniform(0, 28, 1_000_000)),                      # coarse-estimator |X| range
              1 + rng.uniform(-0.07, 0.07, 400_000),                        # the near-1 polynomial and its edges
              np.exp(rng.uniform(-744, 709, 400_000)),                      # wide exponents, subnormals
              np.abs(_inputs(200_000)[0]) * 1e3 + 1.0):
        _same('log', x)
        _same('log10', x)


def test_special_values():
    v = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, 5e-324, -5e-324, 1e308, -1e308, 2.0 ** -1022, 3.0])
    x, y = np.meshgrid(v, v)
    x, y = x.ravel(), y.ravel()
    for fn in ('atan2', 'hypot'):
        h, g = mathhost.evaluate(fn, y, x), mathhost.glibc(fn, y, x)
        assert np.array_equal(h.view(np.int64), g.view(np.int64)), fn
    for fn in ('tanh', 'sincos_s', 'sincos_c', 'log', 'log10'):
        xs = v[np.isfinite(v)]
        h, g = mathhost.evaluate(fn, xs), mathhost.glibc(fn, xs)
        assert np.array_equal(np.isnan(h), np.isnan(g)), fn
        ok = ~np.isnan(g)
        assert np.array_equal(h[ok].view(np.int64), g[ok].view(np.int64)), fn


def test_sincos_is_not_sin_fma():
    """Why sincos, not sin/cos: glibc 2.35's separate sin and cos are the
    ifunc'd FMA builds and round differently from sincos on some arguments,
    so the kernels must follow whichever entry the reference reaches
    (sincos, for its cos(x)/sin(x) pairs)."""
    x = np.random.default_rng(2).uniform(-3, 3, 1_000_000)
    s = mathhost.glibc('sincos_s', x).view(np.int64)
    f = mathhost.glibc('glibc_sin', x).view(np.int64)
    assert 0 < np.count_nonzero(s != f) < x.size // 100
