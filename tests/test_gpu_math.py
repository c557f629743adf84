"""Device libm (aero_math.h on gfx950) vs the same code compiled for the host
and vs glibc; IEEE sqrt/fmod/division on the device vs the host."""
import numpy as np
import pytest

import aero_testlib as tl  # noqa: F401  (puts the package on sys.path)


def _inputs(n=400000, seed=5):
    r = np.random.default_rng(seed)
    a = r.uniform(-1, 1, n) * np.exp(r.normal(0, 2, n))
    b = r.uniform(-1, 1, n) * np.exp(r.normal(0, 2, n))
    return a, b


@pytest.mark.gpu
def test_device_ieee_ops_exact(engine_lib):
    import aero_engine as ae
    eng = ae.Engine(max_channels=1)
    a, b = _inputs()
    pa = np.abs(a)
    assert np.array_equal(eng.device_math('sqrt', pa), np.sqrt(pa))
    assert np.array_equal(eng.device_math('div', a, b), a / b)
    ph = a * 400.0
    assert np.array_equal(eng.device_math('fmod360', ph), np.fmod(ph, 360.0))
    eng.close()


@pytest.mark.gpu
def test_device_math_matches_host_build(engine_lib):
    import aero_engine as ae
    import mathhost
    eng = ae.Engine(max_channels=1)
    a, b = _inputs()
    for fn in ('hypot', 'atan2', 'tanh', 'sin', 'cos', 'log10'):
        x, y = a, b
        if fn in ('sin', 'cos'):
            x = a * 2.0
        if fn == 'log10':
            x = np.abs(a) * 1e3 + 1.0
        dev = eng.device_math(fn, x, y)
        host = mathhost.evaluate(fn, x, y)
        assert np.array_equal(dev.view(np.uint64), host.view(np.uint64)), fn
    eng.close()


def _edge_values(rng, n):
    """Random magnitudes over the whole double range, plus zeros, subnormals,
    the fast paths' range edges, infinities and NaN."""
    e = rng.uniform(-1074, 1023, n)
    x = rng.choice([-1.0, 1.0], n) * np.exp2(e) * rng.uniform(1, 2, n)
    special = np.array([0.0, -0.0, 5e-324, -5e-324, 2.0 ** -1022, 2.0 ** -500, 2.0 ** 500, 2.0 ** -767,
                        np.nextafter(2.0 ** -500, 0), np.nextafter(2.0 ** 500, np.inf), np.inf, -np.inf, np.nan,
                        1.7976931348623157e308, 1.0, -1.0, 3.0])
    return np.concatenate([x, special, rng.standard_normal(n) * 1e3])


@pytest.mark.gpu
def test_short_division_and_sqrt_sequences_are_ieee(engine_lib):
    """div_c (constant divisor, Markstein), div_n (the compiler's sequence
    without div_scale / div_fixup, zero numerators by select) and sqrt_n
    (without the 2^-767 scaling) equal IEEE a / b and sqrt bit for bit,
    including the operands that take their IEEE fallbacks."""
    import aero_engine as ae
    eng = ae.Engine(max_channels=1)
    rng = np.random.default_rng(17)
    a = _edge_values(rng, 300000)
    b = rng.permutation(a)
    with np.errstate(all='ignore'):
        for fn, ref in (('div_c48000', a / 48000.0), ('div_c360', a / 360.0), ('div_c192000', a / 192000.0),
                        ('div_n', a / b), ('sqrt_n', np.sqrt(np.abs(a)))):
            x = np.abs(a) if fn == 'sqrt_n' else a
            got = eng.device_math(fn, x, b)
            same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
            assert same.all(), (fn, x[~same][:4], b[~same][:4], got[~same][:4], ref[~same][:4])
        # the demods' operand ranges, densely
        m = rng.uniform(-1, 1, 400000) * np.exp(rng.uniform(-30, 30, 400000))
        d = rng.uniform(0.5, 2, 400000) * np.exp(rng.uniform(-30, 30, 400000))
        for fn, x, y, ref in (('div_n', m, d, m / d), ('div_c360', m, d, m / 360.0),
                              ('sqrt_n', np.abs(m), d, np.sqrt(np.abs(m)))):
            assert np.array_equal(eng.device_math(fn, x, y).view(np.uint64), ref.view(np.uint64)), fn
    eng.close()


@pytest.mark.gpu
def test_hypot_normal_range_variant_is_glibc(engine_lib):
    """aero_hypot_nr (the coarse kernel's branch-free |X| for waves whose
    values are all in [2^-200, 2^200]) equals glibc hypot bit for bit there,
    including ratios below 2^-54, exact cases and equal components."""
    import aero_engine as ae
    import mathhost
    eng = ae.Engine(max_channels=1)
    rng = np.random.default_rng(23)
    n = 500000
    a = rng.choice([-1.0, 1.0], n) * np.exp2(rng.uniform(-199, 199, n)) * rng.uniform(1, 2, n)
    ints = rng.integers(1, 1 << 20, (2, n)).astype(np.float64)                  # exact cases (3, 4 -> 5, ...)
    cases = [(a, rng.choice([-1.0, 1.0], n) * np.exp2(rng.uniform(-199, 199, n))),   # any ratio
             (a, a * np.exp2(rng.uniform(-70, 0, n))),                                  # around the 2^-54 cut
             (a, a * (1 + rng.standard_normal(n) * 1e-9)),                              # |x| ~ |y|
             (ints[0], ints[1])]
    for x, b in cases:
        got = eng.device_math('hypot_nr', x, b)
        ref = mathhost.glibc('hypot', x, b)
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))
    eng.close()
