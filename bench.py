"""Aero demodulation benchmark (BASELINE.json metric: Msamples/s of 10500-bps
OQPSK demod + Viterbi on 1/2/4/8 MI355X).

One step = one coarse-estimator hop (4096 samples at 48 kHz) pushed for every
channel of the batch and run through the whole hot path: demod segment,
coarse FFT estimate + hop decision, AeroL framing, Viterbi + delay line +
descrambler + CRC, frame records back to the host and ACARS parsing.

Workload: C independent single-VFO 10500-bps OQPSK channels per GPU
(BASELINE configs[1] replicated across the batch; one VFO cannot fill a GPU
because its recurrence is sequential).  Inputs: synthetic 48 kHz P-channel
PCM (tools/aero_synth.cpp), materialised in HBM before the timed region.
Multi-GPU: one process per GPU, channels sharded (weak scaling), no
data-path collective; barrier + max-over-ranks timing only.
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, 'aero-cli_amd'), os.path.join(ROOT, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)

HOP = 4096
FS = 48000
BYTES_PER_SAMPLE = 18.22   # 2 B int16 in + 16 B AGC ring r/w + 0.22 B soft bits out
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6    # MI355X vector FP64 (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=48, help='hops before timing (hunter scan + lock)')
    ap.add_argument('--channels', type=int, default=65536, help='VFO channels per GPU (one lane each: 65536 fill the 1024 SIMDs at one wave each)')
    ap.add_argument('--pool', type=int, default=64, help='distinct synthetic streams per GPU')
    ap.add_argument('--cpu-seconds', type=float, default=240.0, help='signal seconds per CPU-baseline process (~10 s CPU each)')
    ap.add_argument('--cpu-procs', type=int, default=8)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--pmc', default=os.path.join(ROOT, 'profiles', 'pmc_demod.json'),
                    help='rocprofv3 PMC summary for the roofline traffic field')
    return ap.parse_args()


def make_pool(n_streams, length, seed0):
    import aero_testlib as tl
    tl.build_cpu_only() if not os.path.exists(tl.SYNTH_SO) else None

    def one(k):
        # seed 0xAE20+k, carrier 12000 + 37.5 + 0.5 k Hz, Eb/N0 12 dB
        return tl.synth(seconds=length / FS, seed=seed0 + k, carrier=12037.5 + 0.5 * (k % 64), ebn0=12.0,
                        phase0=0.1 * k, lead_in=0)
    with cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
        return np.stack(list(ex.map(one, range(n_streams))))


def cpu_baseline(seconds, procs):
    """The oracle (CPU port of the reference path) on host cores, one process
    per channel as aero-decode is deployed (one VFO per process); bounded
    sample: each process decodes `seconds` of its own synthetic stream."""
    import multiprocessing as mp
    ctx = mp.get_context('fork')
    with ctx.Pool(procs) as p:
        res = p.map(_cpu_one, [(seconds, 0xBE00 + k) for k in range(procs)])
    total = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    cpu = sum(r[1] for r in res)
    return {'value': round(total / wall / 1e6, 4), 'unit': 'Msamples/s', 'cores': procs, 'kind': 'port',
            'sample': '%d processes x %.0f s of synthetic 10500-bps P-channel (48 kHz int16) through '
                      'oracle/liboracle.so (demod + coarse + hunter + AeroL + Viterbi + ACARS), '
                      '12000-sample messages; %.1f s CPU total' % (procs, seconds, cpu),
            'per_core_msps': round(total / cpu / 1e6, 4)}


def _cpu_one(arg):
    seconds, seed = arg
    import aero_testlib as tl
    pcm = tl.synth(seconds=seconds, seed=seed, carrier=12037.5, ebn0=12.0)
    o = tl.Oracle()
    t = time.perf_counter()
    o.push_chunked(pcm, 12000)
    return len(pcm), time.perf_counter() - t


def main():
    a = parse()
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    import shard
    C, P = a.channels, a.pool
    steps_total = a.warmup + a.steps
    span = steps_total * HOP
    offsets = shard.channel_offsets(C, P, rank)
    pool_host = make_pool(P, span + int(offsets.max()) + 1, 0xAE20 + 1000 * rank)
    # CPU baseline first, in worker processes forked before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a.cpu_seconds, a.cpu_procs)

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    import aero_engine as ae
    pool = torch.from_numpy(pool_host).to('cuda')

    def step_input(s):
        # [HOP, C] time-major; channel c = g*P + p reads stream p at offset off[g]
        views = [pool[:, int(o) + s * HOP:int(o) + (s + 1) * HOP] for o in offsets]
        return torch.stack(views).permute(2, 0, 1).reshape(HOP, C).contiguous()

    eng = ae.Engine(max_channels=C, device=local, flags=ae.F_TIMING)
    for _ in range(C):
        eng.open_channel(10500, FS)
    # warmup: hunter scan, AFC and lock (untimed)
    for s in range(a.warmup):
        x = step_input(s)
        torch.cuda.synchronize()
        eng.push_batch_device(x.data_ptr(), HOP, C, C)
        eng.run()
        eng.drain_items()
    timed_inputs = [step_input(a.warmup + s) for s in range(a.steps)]
    eng.sync()
    torch.cuda.synchronize()
    eng.timing_reset()
    s0 = eng.samples_processed()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    items = 0
    for x in timed_inputs:
        eng.push_batch_device(x.data_ptr(), HOP, C, C)
        eng.run()
        items += eng.drain_items()  # ACARS items leave every step, as a serving host would take them
    eng.sync()
    items += eng.drain_items()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    samples = eng.samples_processed() - s0
    t = torch.tensor([elapsed, float(samples)], dtype=torch.float64, device='cuda')
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, samples = float(tmax[0]), float(t[1])
    kt = {k: eng.timing(k) for k in ('demod', 'coarse', 'frame', 'viterbi')}
    ht = {k: eng.timing(k) for k in ('host_push', 'host_run', 'host_wait_njobs', 'host_wait_jobs', 'host_frames')}
    if rank == 0:
        value = samples / elapsed / 1e6
        dm_ms, dm_n = kt['demod']
        per_launch_s = dm_ms / 1e3 / max(dm_n, 1)
        samples_per_launch = C * HOP
        achieved = BYTES_PER_SAMPLE * samples_per_launch / per_launch_s / 1e9
        traffic = None
        if os.path.exists(a.pmc):
            try:
                traffic = json.load(open(a.pmc)).get('hbm_bytes_per_launch')
            except Exception:
                traffic = None
        out = {
            'metric': 'Msamples/s demod+Viterbi, 10500bps OQPSK, 1/2/4/8 GPU; ACARS frames bit-exact vs ref',
            'value': round(value, 3), 'unit': 'Msamples/s', 'n_gpus': world, 'steps': a.steps,
            'warmup': a.warmup, 'ms_per_step': round(elapsed / a.steps * 1e3, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic',
            'config': {'workload': 'C2 x %d: independent single-VFO 10500-bps continuous OQPSK P-channels '
                                   'per GPU, 48 kHz int16, one 4096-sample hop per step' % C,
                       'channels_per_gpu': C, 'total_channels': C * world, 'hop_samples': HOP,
                       'parallelism': 'channel-sharded x%d' % world},
            'roofline': {'bound': 'hbm', 'kernel': 'demod_oqpsk_kernel', 'achieved': round(achieved, 2),
                         'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 5),
                         'traffic': traffic, 'bytes_per_sample': BYTES_PER_SAMPLE,
                         'avg_launch_ms': round(per_launch_s * 1e3, 3)},
            'kernel_ms_per_step': {k: round(v[0] / max(a.steps, 1), 3) for k, v in kt.items()},
            'acars_items': items,
            'host_ms_per_step': {k: round(v[0] / max(a.steps, 1), 3) for k, v in ht.items()},
        }
        if cpu is not None:
            out['cpu_baseline'] = cpu
            out['vs_cpu'] = round(value / cpu['value'], 1)
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
