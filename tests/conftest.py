import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'aero-cli_amd'))


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU')


@pytest.fixture(scope='session')
def cpu_libs():
    import aero_testlib
    aero_testlib.build_cpu_only()
    return True


@pytest.fixture(scope='session')
def engine_lib():
    import aero_testlib
    aero_testlib.build_all()
    import aero_engine
    return aero_engine.load_library()


@pytest.fixture(params=['few', 'one'])
def msk_kernel(request, monkeypatch):
    """Both continuous-MSK kernel shapes (demod_msk.hip): the few-channel one
    (16 lanes per channel, the default up to 4096 channels) and the
    one-lane-per-channel kernels (AERO_MSK_WIDE=0, what C3's 65536 channels
    run); the engine reads the variable when it creates a group."""
    if request.param == 'one':
        monkeypatch.setenv('AERO_MSK_WIDE', '0')
    else:
        monkeypatch.delenv('AERO_MSK_WIDE', raising=False)
    return request.param


@pytest.fixture(params=['few', 'one'])
def oqpsk_kernel(request, monkeypatch):
    """Both continuous-OQPSK kernel shapes (demod_oqpsk.hip): the few-channel
    one (16 lanes per channel, the default up to 4096 channels) and the
    chain + FIR helper-wave kernel (AERO_OQPSK_WIDE=0, what C2's 65536
    channels run)."""
    if request.param == 'one':
        monkeypatch.setenv('AERO_OQPSK_WIDE', '0')
    else:
        monkeypatch.delenv('AERO_OQPSK_WIDE', raising=False)
    return request.param
