"""The N>1 path of bench.py under RCCL, rehearsed on one
GPU: `bench.py --dist` runs a one-rank `nccl` process group through the same
calls a multi-GPU run makes (init with device_id, the barriers around the
timed region, the MAX / SUM all-reduces of the timings and counts, C5's
broadcast of each wideband read).  The 8-GPU run itself is the driver's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, timeout):
    env = dict(os.environ)
    for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--dist', '--no-cpu-baseline'] + args,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_rccl_group_c2():
    out = _bench(['--channels', '4096', '--steps', '3', '--warmup', '1', '--h2d-steps', '1'], 240)
    assert out['process_group'] == 'nccl' and out['n_gpus'] == 1
    assert out['config']['total_channels'] == 4096
    assert out['value'] > 0 and out['h2d']['value'] > 0
    # the SUM all-reduce carried the counters through
    assert out['timed_region']['frames'] > 0 and out['timed_region']['su_crc_ok'] > 0


def test_bench_rccl_group_c5():
    out = _bench(['--mode', 'c5', '--steps', '2', '--warmup', '0'], 300)
    assert out['process_group'] == 'nccl' and out['n_gpus'] == 1
    assert out['value'] > 0
