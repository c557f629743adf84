"""A broken chain/FIR wave hand-off in the OQPSK demod is an error, not
silence (demod_oqpsk.hip, SPIN_LIMIT): the diagnostic build
libaero_engine_handoff_fail.so (AERO_X_HANDOFF_FAIL: the FIR waves return at
once, the chain waves' wait gives up after 2^12 polls) must make aero_run
fail with AERO_E_DEVICE, where the product build decodes the same input."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG_SO = os.path.join(ROOT, 'aero-cli_amd', 'libaero_engine_handoff_fail.so')

CHILD = r'''
import sys
sys.path[:0] = [%r, %r]
import aero_engine as ae, aero_testlib as tl
pcm = tl.synth(seconds=2.0, seed=0xAE20)
eng = ae.Engine(max_channels=4)
chs = [eng.open_channel(10500, 48000) for _ in range(4)]
rc = 0
try:  # the error surfaces at the first call that waits for a demod pass
    for c in chs:
        eng.push(c, pcm)
    eng.run()
    eng.flush()
except ae.AeroError as ex:
    rc = ex.rc
print('RC', rc)
''' % (os.path.join(ROOT, 'aero-cli_amd'), os.path.join(ROOT, 'tests'))


def _run(so):
    env = dict(os.environ)
    env.pop('AERO_ENGINE_SO', None)
    # the hand-off exists in the chain + FIR-wave kernel only: four channels
    # would otherwise run the few-channel kernel (engine.hip wide_max)
    env['AERO_OQPSK_WIDE'] = '0'
    if so:
        env['AERO_ENGINE_SO'] = so
    r = subprocess.run([sys.executable, '-c', CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return int([l for l in r.stdout.splitlines() if l.startswith('RC')][-1].split()[1])


@pytest.mark.gpu
def test_handoff_timeout_fails_the_run(engine_lib):
    assert os.path.exists(DIAG_SO), 'diagnostic build missing (aero-cli_amd/build.py build_diag)'
    import aero_engine as ae
    assert _run(DIAG_SO) == ae.AERO_E_DEVICE
    assert _run(None) == 0
