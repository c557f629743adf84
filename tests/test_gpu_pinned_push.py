"""Batch pushes from pinned host memory (a torch pin_memory() tensor): with
64 or more channels aero_push_pcm_batch DMAs the caller's rows straight into
the PCM ring on the input stream, each copy waiting only for the demod launch
that consumed the rows it overwrites (engine.hip push_common /
note_consumed).  The bench's H2D-inclusive region runs this path; here its
decoded output is compared with the oracle, channel by channel, through
several PCM-ring wraps (32768 rows), both for whole ring rows (one 1-D copy:
the batch covers every channel of the group) and for a batch narrower than
the group with idle channels beside it (2-D copy)."""
import concurrent.futures as cf

import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu


def _oracle(pcm):
    o = tl.Oracle()
    o.push_chunked(pcm, 12000)
    return o.softbits(), o.item_lines('A')


@pytest.mark.parametrize('nch,max_channels,chunk', [(64, 64, 4096), (64, 70, 7000)])
def test_pinned_batch_push_matches_oracle(engine_lib, nch, max_channels, chunk):
    import torch
    import aero_engine as ae
    seconds = 8.0
    streams = [tl.synth(seconds=seconds, seed=0xB100 + k, carrier=12030.0 + 0.25 * k, ebn0=12.0, phase0=0.05 * k)
               for k in range(nch)]
    x = np.stack(streams, axis=1)  # time-major [n][nch]
    L = x.shape[0] // chunk * chunk
    eng = ae.Engine(max_channels=max_channels, flags=ae.F_TRACE_SOFT)
    chans = [eng.open_channel(10500, 48000) for _ in range(max_channels)]
    assert chans[:nch] == list(range(nch))
    # two pinned buffers used alternately, refilled while the engine runs
    bufs = [torch.empty((chunk, nch), dtype=torch.int16).pin_memory() for _ in range(2)]
    for k, t in enumerate(range(0, L, chunk)):
        b = bufs[k % 2]
        b.copy_(torch.from_numpy(np.ascontiguousarray(x[t:t + chunk])))
        eng.push_batch_host(b.data_ptr(), chunk, nch, nch)
        eng.run()
    eng.flush()
    assert L > 3 * 32768
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        refs = list(ex.map(_oracle, [s[:L] for s in streams]))
    for k in range(nch):
        sb, ritems = eng.softbits(k), refs[k][1]
        assert len(refs[k][0]) > 1000, 'oracle did not lock on channel %d' % k
        assert np.array_equal(sb, refs[k][0]), 'channel %d soft bits differ' % k
        assert ritems and eng.items(k) == ritems, 'channel %d items differ' % k
    for k in range(nch, max_channels):  # idle channels stay empty
        assert len(eng.softbits(k)) == 0 and eng.items(k) == []
    eng.close()
