"""aero_math.h (the device libm) compiled for the host vs glibc 2.35, the
library the reference links.  hypot and tanh are glibc's algorithms and must
be bit-exact; atan2/sin/cos/log10 are correctly rounded and may differ from
glibc only where glibc itself is not (<= 1 ulp, rare)."""
import numpy as np
import pytest

import mathhost


def _inputs(n=1000000, seed=11):
    r = np.random.default_rng(seed)
    a = r.uniform(-1, 1, n) * np.exp(r.normal(0, 2, n))
    b = r.uniform(-1, 1, n) * np.exp(r.normal(0, 2, n))
    return a, b


@pytest.mark.parametrize('fn', ['hypot', 'tanh'])
def test_bit_exact_with_glibc(fn):
    a, b = _inputs()
    assert np.array_equal(mathhost.evaluate(fn, a, b).view(np.int64), mathhost.glibc(fn, a, b).view(np.int64))


@pytest.mark.parametrize('fn,scale,rate', [('atan2', None, 0.002), ('sin', 2.0, 0.003), ('cos', 2.0, 0.003),
                                           ('log10', 'pos', 0.001)])
def test_correctly_rounded_vs_glibc(fn, scale, rate):
    a, b = _inputs()
    x = a
    if scale == 'pos':
        x = np.abs(a) * 1e3 + 1.0
    elif scale:
        x = a * scale
    d = mathhost.evaluate(fn, x, b).view(np.int64) - mathhost.glibc(fn, x, b).view(np.int64)
    assert np.abs(d).max() <= 1
    assert np.count_nonzero(d) / d.size < rate


def test_special_values():
    x = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, 5e-324, 1e308])
    y = np.array([0.0, 0.0, -0.0, np.inf, 1.0, -np.inf, 1.0, -1e308])
    for fn in ('atan2', 'hypot'):
        h, g = mathhost.evaluate(fn, x, y), mathhost.glibc(fn, x, y)
        assert np.array_equal(np.signbit(h), np.signbit(g)) and np.allclose(h, g, equal_nan=True), fn
    for fn in ('tanh', 'sin', 'cos'):
        xs = x[np.isfinite(x) & (np.abs(x) < 2.0 ** 20)]
        assert np.allclose(mathhost.evaluate(fn, xs), mathhost.glibc(fn, xs), rtol=1e-15, atol=0), fn


def test_atan2_fast_path_equals_double_double():
    """The Ziv fast path of aero_atan2 must return exactly what the
    double-double path returns (it falls back whenever its bound is unsure)."""
    rng = np.random.default_rng(7)
    n = 1_000_000
    x = rng.standard_normal(n)
    ys = [rng.standard_normal(n),                                   # generic
          x * (1 + rng.standard_normal(n) * 1e-9),                  # |t| near 1
          rng.integers(0, 65, n) / 64 * x * (1 + rng.standard_normal(n) * 1e-13),  # t near k/64
          rng.standard_normal(n) * np.exp(rng.uniform(-700, 700, n))]            # extreme ratios
    for y in ys:
        a = mathhost.evaluate('atan2', y, x).view(np.int64)
        b = mathhost.evaluate('atan2_dd', y, x).view(np.int64)
        assert np.array_equal(a, b)


def test_log_fast_path_equals_double_double():
    rng = np.random.default_rng(11)
    for x in (np.exp(rng.uniform(0, 28, 1_000_000)),                      # coarse-estimator |X| range
              1 + rng.uniform(0, 1e-6, 200_000),                            # near 1
              np.exp(rng.uniform(-700, 700, 500_000)),                      # wide exponents
              (1 + rng.integers(0, 65, 500_000) / 64) * (1 + rng.standard_normal(500_000) * 1e-13)):
        a = mathhost.evaluate('log', x).view(np.int64)
        b = mathhost.evaluate('log_dd', x).view(np.int64)
        assert np.array_equal(a, b)


def test_sincos_fast_path_equals_double_double():
    """aero_sincos's Ziv fast path (|x| <= 1/4) returns exactly what the
    double-double path returns, for the loop corrections the demods pass it
    (rotator frequency, PLL steps, averaged phase errors) and around the
    range's edges."""
    rng = np.random.default_rng(5)
    xs = [rng.uniform(-0.25, 0.25, 1_000_000),
          rng.standard_normal(1_000_000) * 1e-4,
          np.exp(rng.uniform(np.log(2.0 ** -27), np.log(0.3), 1_000_000)) * rng.choice([-1.0, 1.0], 1_000_000),
          rng.uniform(-0.6, 0.6, 200_000)]
    for x in xs:
        for a, b in (('sincos_s', 'sincos_dd_s'), ('sincos_c', 'sincos_dd_c')):
            assert np.array_equal(mathhost.evaluate(a, x).view(np.int64), mathhost.evaluate(b, x).view(np.int64)), a
