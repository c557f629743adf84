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
