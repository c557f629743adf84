"""One HIP runtime per process, whatever the import order.

PyTorch-ROCm bundles its own libamdhip64 / libhsa-runtime64 in torch/lib;
the engine links /opt/rocm's.  Loading the engine before torch used to map
both copies, and a torch device pointer was then unknown to the engine's
runtime.  aero_engine.load_library preloads torch's copy, so either order
maps exactly one.  The CPU test checks the mappings (no GPU call); the GPU
test pushes torch device memory through the engine in both orders."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_MAPS = r'''
import sys
sys.path.insert(0, %r)
order = sys.argv[1]
import aero_engine as ae
if order == 'engine_first':
    ae.load_library()
    import torch
else:
    import torch
    ae.load_library()
libs = sorted({l.split()[-1] for l in open('/proc/self/maps')
               if 'libamdhip64' in l or 'libhsa-runtime64' in l})
print('\n'.join(libs))
'''

_PUSH = r'''
import sys
sys.path.insert(0, %r)
sys.path.insert(0, %r)
order = sys.argv[1]
import numpy as np
import aero_engine as ae
if order == 'engine_first':
    eng = ae.Engine(max_channels=1, flags=ae.F_TRACE_HOPS)
    import torch
else:
    import torch
    torch.cuda.init()
    eng = ae.Engine(max_channels=1, flags=ae.F_TRACE_HOPS)
ch = eng.open_channel(10500, 48000)
x = torch.zeros(3 * 4096 + 1, dtype=torch.int16, device='cuda')
torch.cuda.synchronize()
eng.push_device(ch, x.data_ptr(), x.numel())
eng.flush()
print('hops', len(eng.hops(ch)))
eng.close()
'''


def _run(code, order):
    r = subprocess.run([sys.executable, '-c', code, order], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


@pytest.mark.parametrize('order', ['engine_first', 'torch_first'])
def test_one_hip_runtime_mapped(engine_lib, order):
    libs = _run(_MAPS % os.path.join(ROOT, 'aero-cli_amd'), order).split()
    hip = [l for l in libs if 'libamdhip64' in l]
    hsa = [l for l in libs if 'libhsa-runtime64' in l]
    assert len(hip) == 1 and len(hsa) == 1, libs


@pytest.mark.gpu
@pytest.mark.parametrize('order', ['engine_first', 'torch_first'])
def test_device_push_any_import_order(engine_lib, order):
    out = _run(_PUSH % (os.path.join(ROOT, 'aero-cli_amd'), os.path.join(ROOT, 'tests')), order)
    assert 'hops 3' in out, out
