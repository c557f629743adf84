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
