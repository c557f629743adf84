"""Diagnostic: where the burst OQPSK demod's time goes (AERO_X_BSTAMPS build,
burst.hip), at the bench configuration: per-section cycles per sample-step
of a wave, samples per launch, findmaxpos scans, active lanes.
Usage: AERO_ENGINE_SO=aero-cli_amd/libaero_engine_bstamps.so \\
       python scripts/burst_stamps.py [channels] [steps] [mode]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'aero-cli_amd'), os.path.join(ROOT, 'tests'), ROOT]
import bench  # noqa: E402
import shard  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 6
MODE = sys.argv[3] if len(sys.argv) > 3 else 'burst10500'
M = bench.MODES[MODE]
HOP, P, PRE = M['hop'], min(64, C), M.get('preroll', 4)
offs = shard.channel_offsets(C, P, 0)
pool_host = bench.make_pool(M, P, (PRE + STEPS) * HOP + int(offs.max()) + 1, 0xAE20)
import torch  # noqa: E402
import aero_engine as ae  # noqa: E402
pool = torch.from_numpy(pool_host).to('cuda')
eng = ae.Engine(max_channels=C, flags=ae.F_TIMING)
for _ in range(C):
    eng.open_channel(M['bitrate'], M['fs'], burst=True)
lib = ae.load_library()
fn = lib.aero_x_burst_stamps
fn.argtypes = [ctypes.c_void_p]
out = (ctypes.c_ulonglong * 16)()
names = ['loop control', 'val_to_demod', 'symbol timing (OQPSK)', 'trident decision', 'part B loads + RRC',
         'PLL, rotators, AGC2', 'symbol step + NCOs', 'entry/exit state']


def step_input(s):
    views = [pool[:, int(o) + s * HOP:int(o) + (s + 1) * HOP] for o in offs]
    return torch.stack(views).permute(2, 0, 1).reshape(HOP, C).contiguous()


for s in range(PRE + STEPS):
    x = step_input(s)
    torch.cuda.synchronize()
    if s == PRE:
        fn(out)  # reset after the pre-roll
        eng.timing_reset()
    eng.push_batch_device(x.data_ptr(), HOP, C, C)
    eng.run()
    eng.drain_items()
eng.sync()
fn(out)
it = max(out[12], 1)
tot = sum(out[:8])
res = {'channels': C, 'steps': STEPS, 'waves_launched_active': int(out[11]), 'lanes_active': int(out[10]),
       'samples': int(out[8]), 'findmaxpos_scans': int(out[9]), 'wave_iterations': int(out[12]),
       'active_lane_fraction': round(out[8] / (64.0 * it), 4),
       'cycles_per_wave_iteration': round(tot / it, 1),
       'sections_cycles_per_iteration': {names[k]: round(out[k] / it, 1) for k in range(8)},
       'kernel_ms_per_step': {k: round(eng.timing('burst_' + k)[0] / STEPS, 3)
                              for k in ('hilbert', 'demod', 'trident', 'frame', 'viterbi')},
       'launches_per_step': {k: round(eng.timing('burst_' + k)[1] / STEPS, 2) for k in ('demod', 'trident')}}
print(json.dumps(res, indent=1))
eng.close()
