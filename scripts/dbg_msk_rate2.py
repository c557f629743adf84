"""Debug: pt_msk trace around an MSK rate change (engine vs oracle)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'aero-cli_amd'), os.path.join(ROOT, 'tests')]
import aero_testlib as tl  # noqa: E402
import aero_engine as ae  # noqa: E402

np.set_printoptions(precision=17, linewidth=200)
br, segs = 600, [(12000, 12.0, 0xE100, 1800.0, 14.0), (24000, 4.0, 0xE102, 1800.0, 14.0)]
msgs = []
for fs, sec, seed, car, eb in segs:
    x = tl.synth_msk(seconds=sec, bitrate=br, baud=600, seed=seed, carrier=car, ebn0=eb, fs=fs)
    st = fs // 4
    msgs += [(x[i:i + st], fs) for i in range(0, len(x), st)]
eng = ae.Engine(max_channels=2, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_PT)
ch = eng.open_channel(br)
o = tl.Oracle(bitrate=br, trace_pt=True)
npt_switch = None
for k, (pcm, fs) in enumerate(msgs):
    if fs != 12000 and npt_switch is None:
        eng.flush()
        npt_switch = len(eng.pt(ch))
        o_pre = len(o.pt())
        print('pt before switch: eng', npt_switch, 'oracle', o_pre)
    eng.push(ch, pcm, fs=fs)
    eng.run()
    o.push(pcm, fs=fs)
eng.flush()
p, rp = eng.pt(ch), o.pt()
rp = rp[npt_switch:] if npt_switch else rp
print('after switch: eng', len(p), 'oracle', len(rp))
n = min(len(p), len(rp))
d = np.nonzero(np.any(p[:n] != rp[:n], axis=1))[0]
print('first pt diffs (relative to the switch):', d[:5])
for i in range(max(0, (d[0] if len(d) else 0) - 2), min(n, (d[0] if len(d) else 0) + 3)):
    print(i, p[i], rp[i])
