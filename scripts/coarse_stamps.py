"""Diagnostic: per-section cycle totals of the coarse FFT kernel (wave 0 of
every workgroup that ran a hop) from the AERO_X_STAMPS build.
Usage: AERO_ENGINE_SO=aero-cli_amd/libaero_engine_stamps.so python scripts/coarse_stamps.py [channels]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'aero-cli_amd'), os.path.join(ROOT, 'tests'), ROOT]
import bench  # noqa: E402
import shard  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
M = bench.MODES['oqpsk10500']
P = min(64, C)
steps = 56
offs = shard.channel_offsets(C, P, 0)
pool_host = bench.make_pool(M, P, steps * 4096 + int(offs.max()) + 1, 0xAE20)
import torch  # noqa: E402
import aero_engine as ae  # noqa: E402
pool = torch.from_numpy(pool_host).to('cuda')
eng = ae.Engine(max_channels=C)
for _ in range(C):
    eng.open_channel(10500, 48000)
lib = ae.load_library()
fn = lib.aero_x_coarse_stamps
fn.argtypes = [ctypes.c_void_p]
out = (ctypes.c_ulonglong * 12)()
vfn = lib.aero_x_viterbi_stamps
vfn.argtypes = [ctypes.c_void_p]
vout = (ctypes.c_ulonglong * 4)()
names = ['prologue', 'ring to LDS + twiddles', 'table gathers + mix', 'FFT 1', 'boxcar+iFFT+square', 'FFT 3',
         'hypot', 'log10 smoothing', 'fold search']
order = list(range(9))
for s in range(steps):
    views = [pool[:, int(o) + s * 4096:int(o) + (s + 1) * 4096] for o in offs]
    x = torch.stack(views).permute(2, 0, 1).reshape(4096, C).contiguous()
    torch.cuda.synchronize()
    eng.push_batch_device(x.data_ptr(), 4096, C, C)
    eng.run()
    eng.sync()
    if s == 47:
        fn(out)  # reset after the lock-in pre-roll
        vfn(vout)
fn(out)
vfn(vout)
tot = sum(out[:9])
n = out[11]
print('channels %d, hops %d, s_memtime cycles per hop (wave 0) %.0f' % (C, n, tot / max(n, 1)))
for k in order:
    print('  %-20s %9.0f  %5.1f %%' % (names[k], out[k] / max(n, 1), 100.0 * out[k] / max(tot, 1)))
eng.close()
vn = vout[3]
print('viterbi jobs %d, s_memtime cycles per job %.0f' % (vn, sum(vout[:3]) / max(vn, 1)))
for k, nm in enumerate(['load + deinterleave', 'decode', 'delay line, descramble, CRC, record']):
    print('  %-38s %9.0f' % (nm, vout[k] / max(vn, 1)))
