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
    # sincos beyond 105414350 (__branred) on the device
    huge = np.sign(a) * np.exp2(np.abs(b) % 1 * 996 + 27) * (1 + np.abs(a) % 1)
    for fn in ('sin', 'cos'):
        dev = eng.device_math(fn, huge)
        assert np.array_equal(dev.view(np.uint64), mathhost.glibc(fn, huge).view(np.uint64)), fn + ' huge'
    eng.close()


@pytest.mark.gpu
def test_short_division_sequences_are_ieee(engine_lib):
    """div_c (constant divisor, Markstein's correction) and div_n (the
    compiler's division sequence without div_scale / div_fixup, zero
    numerators by select) equal the IEEE quotient bit for bit inside their
    contract (aero_math.h): zero or |a| >= 2^-969 with a normal quotient,
    divisors and their reciprocals normal; dense sampling of the demods'
    operand ranges, the contract's edges and signed zeros."""
    import aero_engine as ae
    eng = ae.Engine(max_channels=1)
    rng = np.random.default_rng(17)
    n = 400000
    sgn = rng.choice([-1.0, 1.0], n)
    wide = sgn * np.exp2(rng.uniform(-960, 1000, n)) * rng.uniform(1, 2, n)
    dem = rng.uniform(-1, 1, n) * np.exp(rng.uniform(-30, 30, n))
    edge = np.concatenate([[0.0, -0.0, 2.0 ** -969, -2.0 ** -969, 1.0, 360.0, 48000.0, 1e308],
                           sgn[:1000] * np.exp2(rng.uniform(-969, -950, 1000))])
    for a in (wide, dem, edge):
        for fn, c in (('div_c48000', 48000.0), ('div_c360', 360.0), ('div_c192000', 192000.0)):
            got = eng.device_math(fn, a)
            assert np.array_equal(got.view(np.uint64), (a / c).view(np.uint64)), fn
    # div_n: divisor and quotient normal, numerator zero or >= 2^-969
    b = sgn * np.exp2(rng.uniform(-500, 500, n)) * rng.uniform(1, 2, n)
    a = rng.permutation(sgn) * np.exp2(rng.uniform(-460, 460, n)) * rng.uniform(1, 2, n)
    a[:64] = 0.0
    a[64:128] = -0.0
    d = rng.uniform(1e-6, 10.0, n)  # the AGC gain's divisor
    for x, y in ((a, b), (dem, d), (np.full(n, 1.414213562), d), (np.full(n, 2.84), 2.84 + np.abs(dem))):
        got = eng.device_math('div_n', x, y)
        assert np.array_equal(got.view(np.uint64), (x / y).view(np.uint64))
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


@pytest.mark.gpu
def test_atan2_branch_free_main_path_is_glibc(engine_lib):
    """aero_atan2_bf (the demods' per-sample atan2: the main path's six forms
    side by side, selected per lane, the general code when any lane of the
    wave is special) equals glibc's __atan2_fma bit for bit: every quadrant,
    |y/x| on both sides of 1 and of 1/16, table-row centres, equal
    magnitudes, and waves mixing special lanes (zeros, infinities, NaN,
    extreme ratios) with normal ones."""
    import aero_engine as ae
    import mathhost
    eng = ae.Engine(max_channels=1)
    rng = np.random.default_rng(29)
    n = 600000
    x = rng.standard_normal(n) * np.exp(rng.uniform(-20, 20, n))
    cases = [rng.standard_normal(n) * np.exp(rng.uniform(-20, 20, n)),
             x * rng.uniform(-1 / 16, 1 / 16, n),
             x * (rng.integers(16, 257, n) / 256) * (1 + rng.standard_normal(n) * 1e-12) * rng.choice([-1, 1], n),
             x * rng.choice([-1.0, 1.0], n),
             x * np.exp2(rng.uniform(-60, 60, n))]
    # whole waves in one form (the wave-uniform shortcuts): x > 0, |y| < |x|,
    # on the small-ratio series or on the table rows
    xp = np.abs(x)
    cases.append(xp * rng.uniform(-1 / 16, 1 / 16, n) * 0.999)
    cases.append(xp * rng.uniform(1 / 16, 1.0, n) * rng.choice([-1, 1], n))
    mixed = cases[0].copy()
    mixed[::97] = 0.0
    mixed[1::89] = np.inf
    mixed[2::83] = np.nan
    mixed[3::79] = 1e-300
    cases.append(mixed)
    for y in cases:
        for xx, yy in ((x, y), (y, x), (-x, y), (x, -y), (xp, y)):
            got = eng.device_math('atan2_bf', yy, xx)
            ref = mathhost.glibc('atan2', yy, xx)
            same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
            assert same.all(), (yy[~same][:3], xx[~same][:3])
    eng.close()


@pytest.mark.gpu
def test_tanh_and_sincos_branch_free_paths_are_glibc(engine_lib):
    """aero_tanh_bf (2^-55 <= |x| < 22 in every lane of the wave: one expm1
    with its five tail forms selected, div_n / div_r divisions) and
    aero_sincos_bf (|x| < 0.855: the Taylor and table forms of do_sin and
    do_cos selected) equal glibc's tanh and sincos bit for bit; whole waves
    in range (the branch-free path runs), the form boundaries (|x| = 1,
    expm1's k = 0 / -1 / general cuts at 2|x| = 0.3466 and 1.0397, the k < 20
    and k > 56 forms, 0.126, 2^-27, table rows), and waves that mix special
    or out-of-range lanes in (the general code runs)."""
    import aero_engine as ae
    import mathhost
    eng = ae.Engine(max_channels=1)
    rng = np.random.default_rng(31)
    n = 1 << 19
    sg = rng.choice([-1.0, 1.0], n)

    def near(v, rel=1e-12):
        return np.repeat(v, n // len(v) + 1)[:n] * (1 + rng.standard_normal(n) * rel) * sg

    ln2 = np.log(2.0)
    th_cases = [rng.uniform(-4, 4, n),                                            # soft values
                sg * np.exp2(rng.uniform(-55, np.log2(21.9), n)),                  # the whole range
                near(np.array([1.0, 0.3466 / 2, 1.0397 / 2, 0.1733, 0.51985])),
                near(np.array([(k + 0.5) * ln2 / 2 for k in list(range(-4, 0)) + list(range(2, 64))]), 1e-15),
                near(np.array([19.5 * ln2 / 2, 20.5 * ln2 / 2, 56.5 * ln2 / 2, 21.99, 2.0 ** -55]), 1e-15)]
    mixed = th_cases[1].copy()
    mixed[::61] = 0.0
    mixed[1::67] = -0.0
    mixed[2::71] = np.inf
    mixed[3::73] = np.nan
    mixed[4::79] = 30.0
    mixed[5::83] = 1e-20
    th_cases.append(mixed)
    for x in th_cases:
        got = eng.device_math('tanh_bf', x)
        ref = mathhost.glibc('tanh', x)
        same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
        assert same.all(), (x[~same][:4], got[~same][:4], ref[~same][:4])
    sc_cases = [rng.uniform(-0.855, 0.855, n),
                sg * np.exp2(rng.uniform(-40, np.log2(0.8554), n)),
                near(np.array([0.126, 2.0 ** -27, 0.855])),
                near(np.arange(1, 110) / 128.0, 1e-13),
                sg * rng.uniform(0, 1e-300, n)]
    mixed = sc_cases[1].copy()
    mixed[::61] = 0.0
    mixed[1::67] = -0.0
    mixed[2::71] = np.inf
    mixed[3::73] = np.nan
    mixed[4::79] = 2.0
    mixed[5::83] = 1e6  # the Cody-Waite reduction (below 105414350)
    mixed[6::89] = 1e10  # __branred (g_branred)
    sc_cases.append(mixed)
    for x in sc_cases:
        for fn in ('sin', 'cos'):
            got = eng.device_math(fn + '_bf', x)
            ref = mathhost.glibc(fn, x)
            same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
            assert same.all(), (fn, x[~same][:4], got[~same][:4], ref[~same][:4])
    eng.close()


@pytest.mark.gpu
def test_phase_pointer_helpers_are_exact(engine_lib):
    """div_cw (div_c behind a wave-uniform test of its contract, the IEEE
    division otherwise) and set_phase_ptr (SetPhaseDeg's fmod(x, 360), its
    add-while-negative loop and (phase / 360) W, DSP.cpp:177-187, with fmod
    by one conditional subtraction on -360 < x < 720) equal the host's IEEE
    arithmetic bit for bit: the carrier steps' phases, the edges of the fast
    range, signed zeros, and waves with tiny, huge or NaN lanes."""
    import aero_engine as ae
    eng = ae.Engine(max_channels=1)
    rng = np.random.default_rng(37)
    n = 1 << 19
    W = 19999.0
    ptr = rng.uniform(0, W, n)
    tiny = ptr.copy()
    tiny[::67] = rng.uniform(0, 1, n)[::67] * 2.0 ** -1000
    tiny[1::71] = 0.0
    for a in (360.0 * ptr, tiny, -360.0 * ptr):
        got = eng.device_math('div_cw_wt', a)
        assert np.array_equal(got.view(np.uint64), (a / W).view(np.uint64))
    x = rng.uniform(-1.6, 361.6, n)
    edge = np.repeat(np.array([-360.0, -359.99999999999994, -0.0, 0.0, 359.99999999999994, 360.0,
                               719.9999999999999, 720.0, 1e-310, -1e-310]), n // 10 + 1)[:n]
    wide = rng.uniform(-1e4, 1e4, n)
    mixed = x.copy()
    mixed[::97] = np.nan
    mixed[1::89] = 1e6
    mixed[2::83] = -5e3
    for x in (x, edge, wide, mixed):
        r = np.fmod(x, 360.0)
        r = np.where(r < 0, r + 360.0, r)
        ref = (r / 360.0) * W
        got = eng.device_math('set_phase_ptr', x)
        same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
        assert same.all(), (x[~same][:4], got[~same][:4], ref[~same][:4])
    eng.close()
