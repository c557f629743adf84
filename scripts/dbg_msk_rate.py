"""Debug: MSK rate-change parity per rate sequence (first differing soft bit
and hop record) on the GPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'aero-cli_amd'), os.path.join(ROOT, 'tests')]
import aero_testlib as tl  # noqa: E402
import aero_engine as ae  # noqa: E402

SEQS = {
    '12k': (600, [(12000, 12.0, 0xE100, 1800.0, 14.0)]),
    '48k_open': (600, [(48000, 8.0, 0xE101, 1800.0, 14.0)]),
    '24k_open600': (600, [(24000, 12.0, 0xE102, 1800.0, 14.0)]),
    '12k_48k': (600, [(12000, 12.0, 0xE100, 1800.0, 14.0), (48000, 6.0, 0xE101, 1800.0, 14.0)]),
    '12k_24k': (600, [(12000, 12.0, 0xE100, 1800.0, 14.0), (24000, 12.0, 0xE102, 1800.0, 14.0)]),
    '24k_12k_1200': (1200, [(24000, 10.0, 0xE120, 1800.0, 14.0), (12000, 12.0, 0xE121, 1800.0, 14.0)]),
}
for name, (br, segs) in SEQS.items():
    msgs = []
    for fs, sec, seed, car, eb in segs:
        x = tl.synth_msk(seconds=sec, bitrate=br, baud=600, seed=seed, carrier=car, ebn0=eb, fs=fs)
        st = fs // 4
        msgs += [(x[i:i + st], fs) for i in range(0, len(x), st)]
    eng = ae.Engine(max_channels=2, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS)
    ch = eng.open_channel(br, segs[0][0] if name.endswith('open') or 'open' in name else None)
    o = tl.Oracle(bitrate=br)
    for pcm, fs in msgs:
        eng.push(ch, pcm, fs=fs)
        eng.run()
        o.push(pcm, fs=fs)
    eng.flush()
    sb, rsb = eng.softbits(ch), o.softbits()
    h, rh = eng.hops(ch), o.hops()
    n = min(len(sb), len(rsb))
    d = np.nonzero(sb[:n] != rsb[:n])[0]
    m = min(len(h), len(rh))
    dh = [i for i in range(m) if not np.array_equal(h[i].view(np.int64), rh[i].view(np.int64))]
    print(name, 'soft', len(sb), len(rsb), 'first diff', d[:3], 'hops', len(h), len(rh), 'first hop diff', dh[:2])
    if dh:
        i = dh[0]
        print('   eng', h[i], '\n   ref', rh[i])
    eng.close()
