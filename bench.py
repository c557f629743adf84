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

# The engine runs one HIP stream per channel kind (and the channeliser one
# more); HIP deals streams round-robin over GPU_MAX_HW_QUEUES hardware
# queues (4 by default, and the GPU boxes set 4), so the C5 receiver's kinds
# shared a queue and ran one after the other.  At least 8,
# set before anything initialises HIP.
# The effective value is recorded in every bench line's config
# (config.gpu_max_hw_queues); --hw-queues 4 measures at the box default.
HWQ_DEFAULT = int(os.environ.get('GPU_MAX_HW_QUEUES', '4'))
if '--hw-queues' in sys.argv[1:-1]:
    os.environ['GPU_MAX_HW_QUEUES'] = sys.argv[sys.argv.index('--hw-queues') + 1]
elif HWQ_DEFAULT < 8:
    os.environ['GPU_MAX_HW_QUEUES'] = '8'


ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, 'aero-cli_amd'), os.path.join(ROOT, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)

# per channel kind: hop (samples per step), input rate, SURVEY.md §8(d) algorithmic
# bytes per input sample, synthetic carrier range, CPU-baseline signal seconds
MODES = {
    # 2 B int16 in + 16 B AGC ring r/w (192000-deep, cannot stay on chip) + 0.22 B soft bits out
    'oqpsk10500': dict(bitrate=10500, hop=4096, fs=48000, bytes=18.22, timing='demod',
                       metric='Msamples/s demod+Viterbi, 10500bps OQPSK, 1/2/4/8 GPU; ACARS frames bit-exact vs ref',
                       cpu_seconds=240.0, config='C2', flops=1300.0, nfft_log2=14,
                       # the coarse kernel's own algorithmic bytes per channel-hop: the
                       # 16384-entry uint32 snapshot ring read once, the y history of
                       # bins 2815..13568 (coarse.hip CoarseK<OQPSK>) read and written
                       coarse_hop_bytes=16384 * 4 + 2 * (13568 - 2815 + 1) * 8,
                       kernels={'demod': 'demod_oqpsk_kernel', 'coarse': 'coarse_kernel', 'frame': 'frame_kernel',
                                'viterbi': 'viterbi_kernel'}),
    # 2 B int16 in + 0.05 B soft bits out
    'msk600': dict(bitrate=600, hop=2048, fs=12000, bytes=2.05, timing='msk600_demod',
                   metric='Msamples/s demod+Viterbi, 600bps MSK (C3); ACARS frames bit-exact vs ref',
                   cpu_seconds=2400.0, config='C3', flops=1050.0, nfft_log2=13,
                   kernels={'demod': 'demod_msk_kernel', 'coarse': 'coarse_kernel', 'frame': 'frame_msk_kernel',
                            'viterbi': 'viterbi_kernel'}),
    # burst OQPSK (C4): 2 B int16 in + 16 B AGC ring r/w (48000-deep) + soft bits out;
    # a step is one 12000-sample message per channel (burst output follows message boundaries)
    'burst10500': dict(bitrate=10500, hop=12000, fs=48000, bytes=18.22,
                       timing='burst_demod', burst=True, preroll=4,
                       metric='Msamples/s demod+Viterbi, 10500bps burst OQPSK (C4); R/T packets bit-exact vs ref',
                       cpu_seconds=240.0, config='C4', flops=1300.0,
                       kernels={'hilbert': 'hilbert_kernel', 'front': 'front_burst_kernel', 'demod': 'demod_burst_kernel',
                                'trident': 'trident_kernel', 'frame': 'frame_burst_kernel',
                                'viterbi': 'rt_viterbi_kernel'}),
    # burst MSK (aero-decode -b 1200 --burst: one fb = 1200 demodulator at 48 kHz), the C4
    # accounting: 2 B int16 in + 16 B AGC ring r/w (48000-deep) + soft bits out; a step is one
    # 12000-sample message per channel
    'burstmsk1200': dict(bitrate=1200, hop=12000, fs=48000, bytes=18.05,
                         timing='burst_demod', burst=True, preroll=4,
                         metric='Msamples/s demod+Viterbi, 1200bps burst MSK; R/T packets bit-exact vs ref',
                         cpu_seconds=240.0, config='f1 (burst MSK 1200)', flops=900.0,
                         kernels={'hilbert': 'hilbert_kernel', 'front': 'front_bmsk_kernel', 'demod': 'demod_bmsk_kernel',
                                  'trident': 'trident_bmsk_kernel', 'frame': 'frame_bmsk_kernel',
                                  'viterbi': 'rt_viterbi_kernel'}),
    # the C channel: OQPSK 8400 with its per-message JFastFir prefilter, AeroL::DecodeC;
    # 2 B int16 in + 16 B AGC ring r/w + soft bits out as C2 (the prefilter's down-mix words and
    # outputs, 4 + 16 B per sample written and read, are this engine's); a step is one 12000-sample
    # message per channel (the prefilter follows message boundaries, oqpskdemodulator.cpp:292-324)
    'c8400': dict(bitrate=8400, hop=12000, fs=48000, bytes=18.22, timing='c8400_demod', preroll=8,
                  metric='Msamples/s demod+Viterbi, 8400bps C channel (f4); SUs and voice bit-exact vs ref',
                  cpu_seconds=240.0, config='f4 (C channel 8400)', flops=1300.0, nfft_log2=14, kind='C-channel',
                  kernels={'prefilter': 'prefilter_dn_kernel + prefilter_blk_kernel', 'demod': 'demod_c_kernel', 'coarse': 'coarse_kernel',
                           'frame': 'frame_c_kernel', 'viterbi': 'viterbi_c_kernel'}),
    # 2 B int16 in + 0.025 B soft bits out (fb stays 600 at 24 kHz, decode/decode.cpp:142-150)
    'msk1200': dict(bitrate=1200, hop=2048, fs=24000, bytes=2.025,
                    timing='msk1200_demod', metric='Msamples/s demod+Viterbi, 1200bps MSK; ACARS frames bit-exact vs ref',
                    cpu_seconds=1200.0, config='C3 (1200 variant)', flops=1050.0, nfft_log2=13,
                    kernels={'demod': 'demod_msk_kernel', 'coarse': 'coarse_kernel', 'frame': 'frame_msk_kernel',
                             'viterbi': 'viterbi_kernel'}),
}
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6    # MI355X vector FP64 (spec)
# Untimed pre-roll before the warmup steps: the hunter's scan and the carrier
# lock take ~30 hops on the synthetic streams; 48 hops leave every channel
# locked (mse < threshold) however small --warmup is, so the timed steps
# always run the locked path (soft bits -> frames -> Viterbi -> ACARS)
PREROLL_HOPS = 48
# CPU-baseline calibration: the oracle's
# per-core rate on the survey container's Intel Xeon (8 vCPU) against the
# reference's own -O2 build probed on that same host
CALIBRATION = {'oqpsk10500': {'port_msps_per_core': 0.967, 'reference_msps_per_core': 0.996},
               'msk600': {'port_msps_per_core': 1.114, 'reference_msps_per_core': 1.387}}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--mode', default='oqpsk10500', choices=sorted(MODES) + ['c1', 'c5', 'c5bin'],
                    help='channel kind (default: the BASELINE.json headline, C2 10500-bps OQPSK)')
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5,
                    help='untimed steps after the fixed %d-hop lock-in pre-roll' % PREROLL_HOPS)
    ap.add_argument('--channels', type=int, default=65536, help='VFO channels per GPU (one lane each: 65536 fill the 1024 SIMDs at one wave each)')
    ap.add_argument('--pool', type=int, default=64, help='distinct synthetic streams per GPU')
    ap.add_argument('--cpu-seconds', type=float, default=None,
                    help='signal seconds per CPU-baseline process (default per mode: ~5-10 s CPU each)')
    ap.add_argument('--cpu-procs', type=int, default=None,
                    help='CPU-baseline processes (default: the host cores this process may use, at most 16 = '
                         'the GPU box CPU share)')
    ap.add_argument('--cpu-runs', type=int, default=3, help='CPU-baseline repetitions (the median is reported)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-dcd-tick', action='store_true',
                    help="continuous OQPSK without AeroL's 1 s DCD timer (AERO_F_DCD_TICK, on by default as in "
                         'bin/aero-decode, whose reference runs the Qt event loop)')
    ap.add_argument('--hw-queues', type=int, default=None,
                    help='GPU_MAX_HW_QUEUES for this run (default: at least 8; applied before HIP initialises)')
    ap.add_argument('--h2d-steps', type=int, default=None,
                    help='continuous modes: steps of the second, H2D-inclusive timed region (int16 blocks pushed '
                         'from pinned host memory inside it; default: as many as --steps, so both regions carry '
                         'the same pipeline fill and drain); 0 skips it')
    ap.add_argument('--dist', action='store_true',
                    help='run under an RCCL process group even with one rank (rehearses the N>1 path: init, '
                         'barriers, max / sum all-reduces, on a one-GPU box)')
    ap.add_argument('--pmc', default=None,
                    help='rocprofv3 PMC summary for the roofline traffic field (default profiles/pmc_<mode>.json; '
                         'used only when it was captured at this mode and channel count)')
    return ap.parse_args()


def synth_one(M, seconds, seed, k=0, lead_in=0):
    import aero_testlib as tl
    if M.get('burst') and M['bitrate'] != 10500:
        # 1200-baud MSK R/T bursts every 1-3 s near 2.5 kHz
        return tl.synth_burst_msk(seconds=seconds, bitrate=M['bitrate'], seed=seed, carrier=2500.0 + 3.0 * (k % 64),
                                  ebn0=14.0, phase0=0.1 * k, lead_in=lead_in or 24000)
    if M.get('burst'):
        # C4: R/T bursts every 1-3 s on a carrier near 12 kHz (the burst demod has no hunter)
        return tl.synth_burst(seconds=seconds, seed=seed, carrier=12000.0 + 0.5 * (k % 64), ebn0=14.0,
                              phase0=0.1 * k, lead_in=lead_in or 24000)
    if M['bitrate'] == 8400:
        return tl.synth_c(seconds=seconds, seed=seed, carrier=12000.0 + 0.5 * (k % 64), ebn0=12.0, phase0=0.1 * k,
                          lead_in=lead_in)
    if M['bitrate'] == 10500:
        # seed 0xAE20+k, carrier 12000 + 37.5 + 0.5 k Hz, Eb/N0 12 dB
        return tl.synth(seconds=seconds, seed=seed, carrier=12037.5 + 0.5 * (k % 64), ebn0=12.0, phase0=0.1 * k,
                        lead_in=lead_in)
    # MSK: carriers inside the first coarse-search window (mixer centre 0 Hz, +-450 Hz)
    return tl.synth_msk(seconds=seconds, bitrate=M['bitrate'], baud=600, seed=seed, carrier=300.0 + 2.0 * (k % 64),
                        ebn0=12.0, phase0=0.1 * k, lead_in=lead_in)


def make_pool(M, n_streams, length, seed0):
    import aero_testlib as tl
    tl.build_cpu_only() if not os.path.exists(tl.SYNTH_SO) else None

    def one(k):
        return synth_one(M, length / M['fs'], seed0 + k, k)
    with cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
        return np.stack(list(ex.map(one, range(n_streams))))


def host_cores():
    """Cores this process may run on, capped at the GPU box's per-GPU CPU
    share (16): os.cpu_count() there reports the whole machine."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cgroup_cpus():
    """CPUs the cgroup quota grants this process (cpu.max), or None."""
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        return None if q == 'max' else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def _cpu_run(M, seconds, procs, seed0):
    import multiprocessing as mp
    ctx = mp.get_context('fork')
    with ctx.Pool(procs) as p:
        res = p.map(_cpu_one, [(M, seconds, seed0 + k) for k in range(procs)])
    total = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    cpu = sum(r[1] for r in res)
    return total / wall / 1e6, total / cpu / 1e6, cpu


def cpu_baseline(mode, M, seconds, procs, runs=3):
    """The oracle (CPU port of the reference path) on host cores, one process
    per channel as aero-decode is deployed (one VFO per process); bounded
    sample: each process decodes `seconds` of its own synthetic stream.
    `value` is the median of `runs` runs at `procs` processes (the GPU box's
    per-GPU CPU share); one more run at the visible CPU count (nproc) with
    the same total work split across that many processes.  The 1-core figure
    is samples per CPU-second of the same runs."""
    rates, ones, cpus = [], [], []
    for r in range(max(1, runs)):
        v, one, cpu = _cpu_run(M, seconds, procs, 0xBE00 + 1000 * r)
        rates.append(v)
        ones.append(one)
        cpus.append(cpu)
    try:
        nvis = len(os.sched_getaffinity(0))
    except AttributeError:
        nvis = os.cpu_count() or 1
    med = sorted(rates)[len(rates) // 2]
    out = {'value': round(med, 4), 'unit': 'Msamples/s', 'cores': procs, 'kind': 'port',
           'sample': ('%d processes x %.0f s of synthetic %d-bps ' + M.get('kind', 'P-channel') + ' (%d Hz int16) '
                      'through oracle/liboracle.so (demod + coarse + hunter + AeroL + Viterbi + ACARS), '
                      '%d-sample messages; median of %d runs (%.1f s CPU each)') % (
                         procs, seconds, M['bitrate'], M['fs'], M['fs'] // 4, len(rates), sorted(cpus)[len(cpus) // 2]),
           'runs_msps': [round(v, 4) for v in rates],
           'one_core_msps': round(sorted(ones)[len(ones) // 2], 4), 'cpu_model': cpu_model(),
           'host_cpus_visible': os.cpu_count(), 'affinity_cpus': nvis, 'cgroup_cpus': cgroup_cpus()}
    if nvis != procs:
        # the same total CPU work spread over nproc processes
        v, one, cpu = _cpu_run(M, max(1.0, seconds * procs / nvis), min(nvis, 512), 0xBF00)
        out['nproc'] = {'value': round(v, 4), 'processes': min(nvis, 512),
                        'seconds_per_process': round(max(1.0, seconds * procs / nvis), 2)}
    if mode in CALIBRATION:
        out['calibration'] = dict(CALIBRATION[mode], host='survey container Intel Xeon, 8 vCPU, 1 thread')
    return out


def _cpu_one(arg):
    M, seconds, seed = arg
    import aero_testlib as tl
    pcm = synth_one(M, seconds, seed, lead_in=1000)
    o = tl.Oracle(bitrate=M['bitrate'], burst=bool(M.get('burst')), dcd_tick=bool(M.get('dcd_tick')))
    t = time.perf_counter()
    o.push_chunked(pcm, M['fs'] // 4)
    return len(pcm), time.perf_counter() - t


def spawn_ranks(n):
    """--gpus N without a launcher: one child process per GPU with the
    torch.distributed env a launcher would set (rendezvous on 127.0.0.1).
    This process never touches the GPU; it exits with the worst child code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def pmc_traffic(path, mode, channels, kernel):
    """HBM bytes per launch of `kernel` (name prefix) from a rocprofv3 PMC
    capture of this same bench configuration (tools/pmc_json.py over
    scripts/profile_round.sh's FETCH_SIZE / WRITE_SIZE passes); None otherwise."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    cfg = d.get('config', {})
    if cfg.get('mode') != mode or int(cfg.get('channels', -1)) != channels:
        return None, None
    for k, v in d.get('kernels', {}).items():
        if k.startswith(kernel):
            return v.get('hbm_bytes_per_launch'), os.path.relpath(path, ROOT)
    return None, None


C5_SECONDS = 6.0  # synthetic wideband held in HBM, read after read in a loop


def _c5_cpu_one(arg):
    cfg, v, audio, spb = arg
    import aero_testlib as tl
    import aero_engine as ae
    o = tl.Oracle(bitrate=ae.vfo_bitrate(cfg['vfos'][v]['data_rate']))
    t = time.perf_counter()
    o.push_chunked(audio, spb)
    return len(audio), time.perf_counter() - t


def c5_cpu_baseline(cfg, x, procs):
    """aero-publish + one aero-decode per VFO, as the reference deploys C5:
    the oracle publisher on one core over the whole sample, then the 64 oracle
    decoders on `procs` processes; wideband Msamples/s and channel
    Msamples/s of the bounded sample."""
    import multiprocessing as mp
    import aero_testlib as tl
    ref = tl.OraclePublisher(cfg['sample_rate'], cfg['center_frequency'], cfg['mains'], cfg['vfos'])
    nb = len(x) // ref.block_len
    t = time.perf_counter()
    ref.process(x[:nb * ref.block_len])
    t_pub = time.perf_counter() - t
    jobs = [(cfg, v, ref.usb(v), ref.info(v)['samples_per_block']) for v in range(len(cfg['vfos']))]
    t = time.perf_counter()
    with mp.get_context('fork').Pool(procs) as p:
        res = p.map(_c5_cpu_one, jobs)
    t_dec = time.perf_counter() - t
    ch_samples = sum(r[0] for r in res)
    wall = t_pub + t_dec  # the publisher feeds the decoders: sequential lower bound on one host
    return {'value': round(ch_samples / wall / 1e6, 4), 'unit': 'Msamples/s', 'cores': procs, 'kind': 'port',
            'sample': '%.1f s of the C5 wideband (%d reads): oracle publisher on 1 core (%.2f s) then 64 oracle '
                      'decoders on %d processes (%.2f s)' % (nb * ref.block_len / cfg['sample_rate'], nb, t_pub,
                                                              procs, t_dec),
            'wideband_msps': round(nb * ref.block_len / wall / 1e6, 4), 'cpu_model': cpu_model()}


def run_c5(a, rank, world, local):
    use_dist = world > 1 or a.dist
    """C5: one 1.536 Msps receiver (3 main VFOs, 64 [vfos], BASELINE
    configs[4]); the wideband CF32 sits in HBM on rank 0, every read is
    broadcast to all ranks (RCCL over xGMI, the path's one exchange step,
    shard.broadcast_reads), and each rank channelises and decodes the VFOs
    shard.shard_vfos gives it.  A step is one 0.25 s read."""
    import aero_testlib as tl
    import shard
    cfg = tl.c5_config()
    owner = shard.shard_vfos(cfg['vfos'], world)
    mine = [owner[v] == rank for v in range(len(cfg['vfos']))]
    x = tl.c5_wideband(cfg, C5_SECONDS) if rank == 0 else None
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = c5_cpu_baseline(cfg, x[:int(cfg['sample_rate'] * 4.0)], a.cpu_procs or host_cores())
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if use_dist:
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    import aero_engine as ae
    ch = ae.Channeliser(cfg['sample_rate'], cfg['center_frequency'], cfg['mains'], cfg['vfos'], max_blocks=1,
                        device=local, skip=[not m for m in mine])
    B = ch.block_len
    nread = int(cfg['sample_rate'] * C5_SECONDS) // B
    wb = torch.empty((nread, B * 2), dtype=torch.float32, device='cuda')
    if rank == 0:
        wb.copy_(torch.from_numpy(x[:nread * B].view(np.float32).reshape(nread, B * 2)))
    rd = torch.empty((B * 2,), dtype=torch.float32, device='cuda')
    eng = ae.Engine(max_channels=max(1, sum(mine)), device=local,
                    flags=ae.F_TIMING | (0 if a.no_dcd_tick else ae.F_DCD_TICK))
    chans = [eng.open_channel(ae.vfo_bitrate(v['data_rate'])) if m else -1 for v, m in zip(cfg['vfos'], mine)]
    per_read = sum(ch.vfo_info(v)['samples_per_block'] for v in range(len(cfg['vfos'])) if mine[v])

    def step(s):
        if rank == 0:
            rd.copy_(wb[s % nread])
        shard.broadcast_reads(rd)
        torch.cuda.synchronize()
        ch.push_device(rd.data_ptr(), 1)
        ch.run()
        ch.feed(eng, chans)
        eng.run()
        return eng.drain_items()

    pre = 16 + a.warmup  # 4 s of audio: every hunter has locked
    for s in range(pre):
        step(s)
    eng.sync()
    ch.sync()
    torch.cuda.synchronize()
    eng.timing_reset()
    s0 = eng.samples_processed()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    items = 0
    for s in range(a.steps):
        items += step(pre + s)
    eng.sync()
    ch.sync()
    items += eng.drain_items()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    samples = eng.samples_processed() - s0
    t = torch.tensor([elapsed, float(samples), float(items)], dtype=torch.float64, device='cuda')
    if use_dist:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, samples, items = float(tmax[0]), float(t[1]), int(t[2])
    if rank == 0:
        value = samples / elapsed / 1e6
        wideband = a.steps * B / elapsed / 1e6
        audio_s = a.steps * 0.25
        # algorithmic bytes of a step: the CF32 read (8 B per wideband sample,
        # SURVEY §8(d) C5) plus every channel's demod bytes per audio sample
        vb = {600: 2.05, 1200: 2.025}
        ch_bytes = sum(ch.vfo_info(v)['samples_per_block'] * vb.get(cfg['vfos'][v]['data_rate'], 18.22)
                       for v in range(len(cfg['vfos'])))
        step_bytes = 8.0 * B * world + ch_bytes
        achieved = step_bytes * a.steps / elapsed / 1e9
        out = {
            'metric': 'Msamples/s demod+Viterbi, C5 64-VFO channeliser + mixed 600/1200/10500 (channel samples)',
            'value': round(value, 3), 'unit': 'Msamples/s', 'n_gpus': world,
            'process_group': 'nccl' if use_dist else None, 'steps': a.steps, 'warmup': a.warmup,
            'preroll_reads': 16, 'ms_per_step': round(elapsed / a.steps * 1e3, 3), 'higher_is_better': True,
            'scaling': 'strong', 'vs_baseline': None, 'dtype': 'f32 channeliser / f64 demod', 'data': 'synthetic',
            'config': {'gpu_max_hw_queues': int(os.environ['GPU_MAX_HW_QUEUES']), 'workload': 'C5: 1.536 Msps receiver, 3 main VFOs, 64 [vfos] (6 x 10500, 29 x 600/1200 '
                                   'alternating), one 0.25 s read per step, reads broadcast to %d rank(s)' % world,
                       'vfos': len(cfg['vfos']), 'vfos_per_rank': per_read and sum(mine),
                       'parallelism': 'vfo-sharded x%d + read broadcast' % world},
            'wideband_msps': round(wideband, 3), 'realtime_factor': round(audio_s / elapsed, 2),
            'roofline': {'bound': 'hbm', 'kernel': 'whole step', 'achieved': round(achieved, 3),
                         'peak': HBM_PEAK_GBS * world, 'unit': 'GB/s',
                         'frac': round(achieved / (HBM_PEAK_GBS * world), 7), 'traffic': None,
                         'bytes_per_step': round(step_bytes)},
            'acars_items': items,
        }
        if cpu is not None:
            out['cpu_baseline'] = cpu
        print(json.dumps(out), flush=True)
    eng.close()
    ch.close()
    if use_dist:
        dist.destroy_process_group()


C1_SECONDS = 60.0  # one VFO of synthetic 10500-bps audio, published as fast as ZeroMQ takes it


def run_c1(a):
    """C1 end to end: the drop-in binaries on one VFO, ZeroMQ
    loopback PUB (tools/zmq_pcm_pub, aero-publish's wire format) -> SUB
    bin/aero-decode -> ACARS JSON lines, timed from the publisher's first
    message to the last expected item; beside it the oracle decoding the same
    audio on one core (the reference runs one process per VFO).  A single VFO
    is one lane of one wave on the GPU: this measures the binary path and its
    per-sample latency, not GPU throughput (that is the C2 line)."""
    import signal
    import socket
    import subprocess
    import tempfile
    import threading
    import aero_testlib as tl
    M = MODES['oqpsk10500']
    pcm = tl.synth(seconds=C1_SECONDS, seed=0xC100, carrier=12037.5, ebn0=12.0)
    o = tl.Oracle()
    t = time.perf_counter()
    o.push_chunked(pcm, 12000)
    t_cpu = time.perf_counter() - t
    want = len(o.item_lines('A'))
    bindir = os.path.join(ROOT, 'aero-cli_amd', 'bin')
    pub = os.path.join(ROOT, 'tools', 'zmq_pcm_pub')
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    tmp = tempfile.mkdtemp(prefix='aero_c1_')
    f = os.path.join(tmp, 'vfo.pcm')
    pcm.astype('<i2').tofile(f)
    dec = subprocess.Popen([os.path.join(bindir, 'aero-decode'), '-p', 'tcp://127.0.0.1:%d' % port, '-t', 'VFO01',
                            '-b', '10500', '--format', 'jsondump', '-s', 'BENCH', '-v'],
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    lines, stamps = [], []

    def pump():
        for raw in dec.stderr:
            lines.append(raw.decode('utf-8', 'replace'))
            stamps.append(time.perf_counter())
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    t_wait = time.perf_counter()
    while not any('Listening for samples' in l for l in lines):
        if dec.poll() is not None or time.perf_counter() - t_wait > 180:
            sys.exit('bench c1: aero-decode did not start:\n' + ''.join(lines[-20:]))
        time.sleep(0.05)
    wait_ms = 1000
    t_pub = time.perf_counter()
    pp = subprocess.Popen([pub, '--bind', 'tcp://127.0.0.1:%d' % port, '--topic', 'VFO01', '--rate', '48000',
                           '--chunk', '12000', '--wait-ms', str(wait_ms), f], stderr=subprocess.PIPE)
    t0 = t_pub + wait_ms / 1000.0  # the publisher sends its first message after the slow-joiner wait
    deadline = time.perf_counter() + 600
    while sum(l.startswith('{') for l in lines) < want and time.perf_counter() < deadline and dec.poll() is None:
        time.sleep(0.01)
    got = [s for l, s in zip(lines, stamps) if l.startswith('{')]
    t_end = got[-1] if got else time.perf_counter()
    dec.send_signal(signal.SIGTERM)
    dec.wait(timeout=120)
    pp.wait(timeout=60)
    th.join(timeout=10)
    os.remove(f)
    os.rmdir(tmp)
    if len(got) < want:
        sys.exit('bench c1: %d of %d ACARS items arrived' % (len(got), want))
    elapsed = t_end - t0
    out = {'metric': 'Msamples/s end-to-end ZeroMQ PUB -> aero-decode -> ACARS JSON, single 10500-bps VFO (C1)',
           'value': round(len(pcm) / elapsed / 1e6, 4), 'unit': 'Msamples/s', 'n_gpus': 1, 'steps': 1, 'warmup': 0,
           'ms_per_step': round(elapsed * 1e3, 1), 'higher_is_better': True, 'scaling': 'none', 'vs_baseline': None,
           'dtype': 'f64', 'data': 'synthetic',
           'config': {'gpu_max_hw_queues': int(os.environ['GPU_MAX_HW_QUEUES']), 'workload': 'C1: one VFO, %.0f s of synthetic 48 kHz int16 10500-bps P-channel in 12000-sample '
                                  'ZeroMQ messages, published without pacing' % C1_SECONDS,
                      'binary': 'aero-cli_amd/bin/aero-decode --format jsondump', 'items': len(got)},
           'realtime_factor': round(C1_SECONDS / elapsed, 2),
           'timing_note': 'first message (publisher start + %d ms slow-joiner wait) to the last ACARS JSON line; '
                          'the audio after the last frame is counted as processed' % wait_ms,
           'roofline': None,
           'cpu_baseline': {'value': round(len(pcm) / t_cpu / 1e6, 4), 'unit': 'Msamples/s', 'cores': 1,
                            'kind': 'port', 'sample': 'the same %.0f s through oracle/liboracle.so in one process'
                                                      % C1_SECONDS, 'cpu_model': cpu_model()}}
    print(json.dumps(out), flush=True)


C5BIN_SECONDS = 12.0  # wideband CF32 file the publisher reads without pacing


def _is_item(line):
    """a jsondump ACARS line of aero-decode (not its AERO_HOST_TIMING summary)"""
    return line.startswith('{') and not line.startswith('{"aero_host_timing"')


def run_c5bin(a):
    """C5 through the drop-in binaries on one GPU: bin/aero-publish (GPU
    channeliser, CF32 file source, the generated 64-VFO INI) -> ZeroMQ ->
    ONE bin/aero-decode subscribed to all 64 topics (one engine channel per
    topic, one aero_run per batch of queued messages).  Timed from the
    publisher's first read to the last ACARS line; the item count is checked
    against the oracle publisher + 64 oracle decoders on the same wideband,
    which is also the CPU baseline (the reference's deployment: one
    aero-publish, one aero-decode process per VFO)."""
    import signal
    import socket
    import subprocess
    import tempfile
    import threading
    import aero_testlib as tl
    import aero_engine as ae
    cfg = tl.c5_config()
    x = tl.c5_wideband(cfg, C5BIN_SECONDS)
    nv = len(cfg['vfos'])
    # reference chain on the host: expected items, channel samples, CPU time
    ref = tl.OraclePublisher(cfg['sample_rate'], cfg['center_frequency'], cfg['mains'], cfg['vfos'])
    nb = len(x) // ref.block_len
    t = time.perf_counter()
    ref.process(x[:nb * ref.block_len])
    t_pub = time.perf_counter() - t
    import multiprocessing as mp
    jobs = [(cfg, v, ref.usb(v), ref.info(v)['samples_per_block']) for v in range(nv)]
    procs = a.cpu_procs or host_cores()
    t = time.perf_counter()
    with mp.get_context('fork').Pool(procs) as p:
        res = p.map(_c5_items_one, jobs)
    t_dec = time.perf_counter() - t
    want = sum(r[1] for r in res)
    ch_samples = sum(r[0] for r in res)
    bindir = os.path.join(ROOT, 'aero-cli_amd', 'bin')
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    tmp = tempfile.mkdtemp(prefix='aero_c5bin_')
    wb = os.path.join(tmp, 'wideband.cf32')
    x[:nb * ref.block_len].astype(np.complex64).tofile(wb)
    ini = os.path.join(tmp, 'c5.ini')
    open(ini, 'w').write(tl.c5_ini(cfg).replace('tcp://*:6004', 'tcp://127.0.0.1:%d' % port))
    args = [os.path.join(bindir, 'aero-decode'), '-p', 'tcp://127.0.0.1:%d' % port, '--format', 'jsondump', '-v']
    for v in range(nv):
        args += ['-t', 'VFO%02d' % (v + 1), '-b', str(cfg['vfos'][v]['data_rate']), '-s', 'BENCH']
    # the publisher reads the file without pacing: unbounded ZeroMQ queues on
    # both ends (AERO_ZMQ_HWM=0) so nothing is dropped while the decoder catches up
    env = dict(os.environ, AERO_ZMQ_HWM='0', AERO_HOST_TIMING='1')
    dec = subprocess.Popen(args, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env)
    lines, stamps = [], []

    def pump(pipe, out, st):
        for raw in pipe:
            out.append(raw.decode('utf-8', 'replace'))
            st.append(time.perf_counter())
    th = threading.Thread(target=pump, args=(dec.stderr, lines, stamps), daemon=True)
    th.start()
    t_wait = time.perf_counter()
    while not any('Listening for samples' in l for l in lines):
        if dec.poll() is not None or time.perf_counter() - t_wait > 180:
            sys.exit('bench c5bin: aero-decode did not start:\n' + ''.join(lines[-20:]))
        time.sleep(0.05)
    pub = subprocess.Popen([os.path.join(bindir, 'aero-publish'), '-v', '-d',
                            'driver=file,path=%s,start_delay_ms=1500' % wb, ini], stdout=subprocess.DEVNULL,
                           stderr=subprocess.PIPE, env=env)
    plines, pstamps = [], []
    tp = threading.Thread(target=pump, args=(pub.stderr, plines, pstamps), daemon=True)
    tp.start()
    pub.wait(timeout=300)
    tp.join(timeout=10)
    t0 = next((s for l, s in zip(plines, pstamps) if 'Starting concurrent reader' in l), None)
    if pub.returncode != 0 or t0 is None:
        dec.kill()
        sys.exit('bench c5bin: aero-publish failed:\n' + ''.join(plines[-20:]))
    # wait for the decoder to go quiet (every queued message decoded)
    n_last, t_last = -1, time.perf_counter()
    while time.perf_counter() - t_last < 3.0 and time.perf_counter() - t0 < 600:
        n = sum(_is_item(l) for l in lines)
        if n != n_last:
            n_last, t_last = n, time.perf_counter()
        time.sleep(0.1)
    got = [s for l, s in zip(lines, stamps) if _is_item(l)]
    t_end = got[-1] if got else time.perf_counter()
    n_run = len(got)
    dec.send_signal(signal.SIGTERM)
    dec.wait(timeout=120)
    th.join(timeout=10)
    n_all = sum(_is_item(l) for l in lines)  # with the flushed tail
    os.remove(wb)
    os.remove(ini)
    os.rmdir(tmp)
    if n_all != want:
        sys.exit('bench c5bin: %d ACARS items, the oracle chain gives %d' % (n_all, want))
    elapsed = t_end - t0
    # where the binaries' wall time went (AERO_HOST_TIMING section totals)
    split = {}
    for l in plines + lines:
        if l.startswith('{"aero_host_timing"'):
            try:
                d = json.loads(l)
                split[d['aero_host_timing']] = dict(d['ms'], **{'n_' + k: v for k, v in d['counts'].items()})
            except ValueError:
                pass
    out = {'metric': 'Msamples/s end-to-end aero-publish -> ZeroMQ -> one 64-topic aero-decode -> ACARS JSON (C5)',
           'value': round(ch_samples / elapsed / 1e6, 4), 'unit': 'Msamples/s', 'n_gpus': 1, 'steps': 1,
           'warmup': 0, 'ms_per_step': round(elapsed * 1e3, 1), 'higher_is_better': True, 'scaling': 'none',
           'vs_baseline': None, 'dtype': 'f32 channeliser / f64 demod', 'data': 'synthetic',
           'config': {'gpu_max_hw_queues': int(os.environ['GPU_MAX_HW_QUEUES']), 'workload': 'C5 through the binaries: %.0f s of 1.536 Msps CF32 (3 main VFOs, 64 [vfos]) read '
                                  'without pacing by bin/aero-publish; one bin/aero-decode with 64 -t topics'
                                  % C5BIN_SECONDS, 'vfos': nv, 'items': n_all, 'items_before_sigterm': n_run},
           'wideband_msps': round(nb * ref.block_len / elapsed / 1e6, 3),
           'realtime_factor': round(C5BIN_SECONDS / elapsed, 2),
           'host_split_ms': split,
           'timing_note': "publisher's first read to the last ACARS JSON line before SIGTERM; audio after the "
                          'last frame counts as processed',
           'roofline': None,
           'cpu_baseline': {'value': round(ch_samples / (t_pub + t_dec) / 1e6, 4), 'unit': 'Msamples/s',
                            'cores': procs, 'kind': 'port',
                            'sample': 'the same %.0f s: oracle publisher on 1 core (%.2f s) then 64 oracle decoders '
                                      'on %d processes (%.2f s)' % (C5BIN_SECONDS, t_pub, procs, t_dec),
                            'cpu_model': cpu_model()}}
    print(json.dumps(out), flush=True)


def _c5_items_one(arg):
    cfg, v, audio, spb = arg
    import aero_testlib as tl
    import aero_engine as ae
    o = tl.Oracle(bitrate=ae.vfo_bitrate(cfg['vfos'][v]['data_rate']))
    o.push_chunked(audio, spb)
    return len(audio), len(o.item_lines('A'))


def main():
    a = parse()
    if (a.gpus > 1 or a.dist) and 'RANK' not in os.environ:
        sys.exit(spawn_ranks(a.gpus))
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    use_dist = world > 1 or a.dist
    if a.mode == 'c5':
        return run_c5(a, rank, world, local)
    if a.mode == 'c1':
        if rank == 0:
            run_c1(a)
        return None
    if a.mode == 'c5bin':
        if rank == 0:
            run_c5bin(a)
        return None
    import shard
    M = MODES[a.mode]
    HOP, FS = M['hop'], M['fs']
    C, P = a.channels, a.pool
    preroll = M.get('preroll', PREROLL_HOPS)  # burst channels have no hunter to lock
    pre = preroll + a.warmup  # untimed hops: lock-in pre-roll + warmup
    burst = bool(M.get('burst'))
    h2d_steps = 0 if burst else max(0, a.steps if a.h2d_steps is None else a.h2d_steps)
    steps_total = pre + a.steps + h2d_steps
    span = steps_total * HOP
    offsets = shard.channel_offsets(C, P, rank)
    pool_host = make_pool(M, P, span + int(offsets.max()) + 1, 0xAE20 + 1000 * rank)
    # CPU baseline first, in worker processes forked before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        # the oracle runs what the GPU runs: the DCD timer on the P channel unless --no-dcd-tick
        Mc = dict(M, dcd_tick=M['bitrate'] == 10500 and not M.get('burst') and not a.no_dcd_tick)
        cpu = cpu_baseline(a.mode, Mc, a.cpu_seconds or M['cpu_seconds'], a.cpu_procs or host_cores(), a.cpu_runs)

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if use_dist:
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    import aero_engine as ae
    pool = torch.from_numpy(pool_host).to('cuda')

    def step_input(s):
        # [HOP, C] time-major; channel c = g*P + p reads stream p at offset off[g]
        views = [pool[:, int(o) + s * HOP:int(o) + (s + 1) * HOP] for o in offsets]
        return torch.stack(views).permute(2, 0, 1).reshape(HOP, C).contiguous()

    eng = ae.Engine(max_channels=C, device=local, flags=ae.F_TIMING | (0 if a.no_dcd_tick else ae.F_DCD_TICK))
    for _ in range(C):
        eng.open_channel(M['bitrate'], FS, burst=burst)
    stat_names = ('rt_tests', 'rt_packets') if burst else ('viterbi_jobs', 'frames', 'su_crc_ok')
    # pre-roll (hunter scan, AFC and lock) + warmup, untimed
    for s in range(pre):
        x = step_input(s)
        torch.cuda.synchronize()
        eng.push_batch_device(x.data_ptr(), HOP, C, C)
        eng.run()
        eng.drain_items()
    timed_inputs = [step_input(pre + s) for s in range(a.steps)]
    eng.sync()
    eng.drain_items()
    torch.cuda.synchronize()
    eng.timing_reset()
    s0 = eng.samples_processed()
    st0 = {k: eng.stat(k) for k in stat_names}
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    items = 0
    for x in timed_inputs:
        eng.push_batch_device(x.data_ptr(), HOP, C, C)
        eng.run()
        items += eng.drain_items()  # ACARS items leave every step, as a serving host would take them
    t_tail = time.perf_counter()
    eng.sync()
    items += eng.drain_items()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    t_end = time.perf_counter()
    elapsed = t_end - t0
    tail_ms = (t_end - t_tail) * 1e3  # final drain: the last passes' decode, copy-back and host items
    samples = eng.samples_processed() - s0
    stats = {k: eng.stat(k) - v for k, v in st0.items()}
    tag = M['timing'][:-len('demod')]
    if burst:  # the burst path's kernels: Hilbert fast FIR, demod, trident FFT check, framing, R/T Viterbi
        kt = {k: eng.timing('burst_' + k) for k in ('hilbert', 'front', 'demod', 'trident', 'frame', 'viterbi')}
    else:
        kt = {k: eng.timing(tag + k) for k in ('demod', 'coarse', 'frame', 'viterbi')}
        if 'prefilter' in M['kernels']:
            kt['prefilter'] = eng.timing(tag + 'prefilter')
    ht = {k: eng.timing(k) for k in ('host_push', 'host_run', 'host_wait_njobs', 'host_wait_jobs', 'host_frames')}
    del timed_inputs
    h2d = None
    if h2d_steps:
        # the same step loop with every int16 block pushed from pinned host
        # memory inside the timed region (H2D-inclusive), the
        # blocks DMA'd straight into the PCM ring while the previous step runs
        host_inputs = [step_input(pre + a.steps + s).cpu().pin_memory() for s in range(h2d_steps)]
        eng.sync()
        eng.drain_items()
        torch.cuda.synchronize()
        s1 = eng.samples_processed()
        if use_dist:
            dist.barrier()
        eng.timing_reset()
        t1 = time.perf_counter()
        tp = [0.0, 0.0, 0.0]  # host seconds in push (incl. the wait for its DMA), run, item drain
        for xh in host_inputs:
            ta = time.perf_counter()
            eng.push_batch_host(xh.data_ptr(), HOP, C, C)
            tb = time.perf_counter()
            eng.run()
            tc = time.perf_counter()
            eng.drain_items()
            td = time.perf_counter()
            tp[0] += tb - ta
            tp[1] += tc - tb
            tp[2] += td - tc
        eng.sync()
        eng.drain_items()
        torch.cuda.synchronize()
        if use_dist:
            dist.barrier()
        h_el = time.perf_counter() - t1
        h_smp = eng.samples_processed() - s1
        th = torch.tensor([h_el, float(h_smp)], dtype=torch.float64, device='cuda')
        if use_dist:
            dist.all_reduce(th[:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(th[1:], op=dist.ReduceOp.SUM)
        h_el, h_smp = float(th[0]), float(th[1])
        h2d = {'value': round(h_smp / h_el / 1e6, 3), 'unit': 'Msamples/s', 'steps': h2d_steps,
               'ms_per_step': round(h_el / h2d_steps * 1e3, 3),
               'pcie_bytes_per_step': 2 * HOP * C * world,
               'host_ms_per_step': {k: round(v / h2d_steps * 1e3, 3) for k, v in zip(('push', 'run', 'drain'), tp)},
               'engine_host_ms_per_step': {k: round(eng.timing(k)[0] / h2d_steps, 3)
                                           for k in ('host_push', 'host_push_copy', 'host_push_pin', 'host_run',
                                                     'host_wait_jobs')},
               'note': 'same steps, int16 [hop, channels] blocks pushed from pinned host memory '
                       '(aero_push_pcm_batch, dev=0) inside the timed region'}
        del host_inputs
    stats['acars_items'] = items
    keys = sorted(stats)
    t = torch.tensor([elapsed, float(samples)] + [float(stats[k]) for k in keys], dtype=torch.float64,
                     device='cuda')
    if use_dist:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, samples = float(tmax[0]), float(t[1])
        stats = {k: int(t[2 + i]) for i, k in enumerate(keys)}
    if rank == 0:
        value = samples / elapsed / 1e6
        # roofline of the dominant kernel (the most device time per step) on
        # the SURVEY.md §8(d) / BASELINE.md basis: the path's algorithmic bytes
        # (bytes per input sample x the samples one step processes) over that
        # kernel's summed device time per step.  The coarse kernel's own
        # algorithmic bytes (snapshot ring + y history per channel-hop) are
        # reported beside it as roofline.kernel_traffic, the demodulator's
        # figure as roofline.path and the whole step as roofline.step.
        steps = max(a.steps, 1)
        dom = max(kt, key=lambda k: kt[k][0])
        dom_ms = kt[dom][0] / steps
        path_bytes = M['bytes'] * C * HOP
        step_bytes = path_bytes
        unit = {'bytes_per_sample': M['bytes'], 'samples_per_step': C * HOP}
        kernel_traffic = None
        if dom == 'coarse' and 'coarse_hop_bytes' in M:
            kb = M['coarse_hop_bytes'] * C * (kt[dom][1] / steps)
            kernel_traffic = {'bytes_per_channel_hop': M['coarse_hop_bytes'], 'bytes_per_step': int(kb),
                              'achieved': round(kb / (dom_ms / 1e3) / 1e9, 2),
                              'frac': round(kb / (dom_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5),
                              'note': "the coarse kernel's own algorithmic bytes: 16384-entry uint32 snapshot "
                                      'ring read + y history of the searched bins read and written'}
        achieved = step_bytes / (dom_ms / 1e3) / 1e9
        step_achieved = path_bytes / (elapsed / steps) / 1e9
        path_kernel = 'demod' if 'demod' in kt else dom
        path_ms = kt[path_kernel][0] / steps
        traffic, traffic_src = pmc_traffic(a.pmc or os.path.join(ROOT, 'profiles', 'pmc_%s.json' % a.mode),
                                           a.mode, C, M['kernels'][dom])
        total_ms = sum(v[0] for v in kt.values()) / steps
        kernels = {}
        for k, (ms, n) in kt.items():
            kernels[M['kernels'][k]] = {'ms_per_step': round(ms / steps, 3), 'launches_per_step': round(n / steps, 2),
                                        'share_of_device_time': round(ms / steps / total_ms, 3) if total_ms else None}
        if 'nfft_log2' in M and kt['coarse'][1]:
            # the coarse estimator's three radix-2 transforms, 5 N log2 N real flops each, per channel-hop
            nf = 1 << M['nfft_log2']
            fl = 3 * 5 * nf * M['nfft_log2']
            kc = kernels[M['kernels']['coarse']]
            tf = fl * C / (kc['ms_per_step'] / 1e3) / 1e12
            kc['fp64'] = {'flop_per_channel_hop': fl, 'achieved_tflops': round(tf, 2), 'peak_tflops': FP64_PEAK_TFLOPS,
                          'frac': round(tf / FP64_PEAK_TFLOPS, 4)}
        # the dominant kernel's algorithmic FP64 flops per step: the coarse
        # estimator's three radix-2 transforms (5 N log2 N each per
        # channel-hop); another kernel carries the path's SURVEY.md §8(d)
        # flops per input sample
        if dom == 'coarse' and 'nfft_log2' in M:
            nf = 1 << M['nfft_log2']
            dom_fl = 3 * 5 * nf * M['nfft_log2'] * C * (kt[dom][1] / steps)
            basis = '3 x 5 N log2 N per channel-hop (N = %d), %d channel-hops per step' % (
                nf, round(C * kt[dom][1] / steps))
        else:
            dom_fl = M['flops'] * C * HOP
            basis = '%g flop per input sample (SURVEY.md §8(d)) x %d samples per step' % (M['flops'], C * HOP)
        dom_tf = dom_fl / (dom_ms / 1e3) / 1e12
        dom_fp64 = {'achieved': round(dom_tf, 3), 'frac': round(dom_tf / FP64_PEAK_TFLOPS, 5), 'basis': basis}
        out = {
            'metric': M['metric'],
            'value': round(value, 3), 'unit': 'Msamples/s', 'n_gpus': world,
            'process_group': 'nccl' if use_dist else None, 'steps': a.steps,
            'warmup': a.warmup, 'preroll_hops': preroll, 'ms_per_step': round(elapsed / a.steps * 1e3, 3),
            'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic',
            'config': {'gpu_max_hw_queues': int(os.environ['GPU_MAX_HW_QUEUES']), 'workload': ('%s x %d: independent single-VFO %d-bps burst %s R/T channels per GPU, '
                                    '%d Hz int16, one %d-sample message per channel per step' % (
                                        M['config'], C, M['bitrate'], 'OQPSK' if M['bitrate'] == 10500 else 'MSK',
                                        FS, HOP)) if burst else (
                                   '%s x %d: independent single-VFO %d-bps continuous %s %ss '
                                   'per GPU, %d Hz int16, one %d-sample %s per step' % (
                                       M['config'], C, M['bitrate'],
                                       'OQPSK' if M['bitrate'] in (10500, 8400) else 'MSK',
                                       M.get('kind', 'P-channel'), FS, HOP,
                                       'message' if M['bitrate'] == 8400 else 'hop')),
                       'channels_per_gpu': C, 'total_channels': C * world, 'hop_samples': HOP,
                       'dcd_tick': (not a.no_dcd_tick) and not burst and M['bitrate'] == 10500,
                       'parallelism': 'channel-sharded x%d' % world},
            # the dominant kernel is bound by FP64 VALU dependency latency, not
            # HBM: its FP64 fraction is the
            # primary figure, the HBM fraction BASELINE.json quotes is
            # roofline.hbm beside it
            'roofline': dict({'bound': 'fp64', 'kernel': M['kernels'][dom], 'achieved': dom_fp64['achieved'],
                              'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s', 'frac': dom_fp64['frac'],
                              'flop_basis': dom_fp64['basis'],
                              'binding': 'FP64 dependency latency of one resident channel per CU (barrier-coupled '
                                         'transforms, exact libm); neither HBM nor the FP64 pipe is saturated',
                              'traffic': traffic, 'traffic_source': traffic_src,
                              'hbm': {'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                                      'frac': round(achieved / HBM_PEAK_GBS, 5),
                                      'basis': 'SURVEY.md §8(d) bytes per input sample x samples per step over '
                                               "the dominant kernel's device time per step"}},
                             **unit, **{'kernel_traffic': kernel_traffic,
                              'bytes_per_step': int(step_bytes), 'kernel_ms_per_step': round(dom_ms, 3),
                              'launches_per_step': round(kt[dom][1] / steps, 2),
                              'path': {'kernel': M['kernels'][path_kernel], 'bytes_per_sample': M['bytes'],
                                       'bytes_per_step': int(path_bytes),
                                       'achieved': round(path_bytes / (path_ms / 1e3) / 1e9, 2),
                                       'frac': round(path_bytes / (path_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5)},
                              'step': {'achieved': round(step_achieved, 2),
                                       'frac': round(step_achieved / HBM_PEAK_GBS, 5),
                                       'ms_per_step': round(elapsed / steps * 1e3, 3)}}),
            'kernels': kernels,
            # SURVEY §8(d) / BASELINE.md: the path is FP64-VALU bound, so the whole-path FP64
            # rate (algorithmic flop per input sample x samples/s) is reported beside the HBM one
            'fp64_roofline': {'flop_per_sample': M['flops'], 'achieved': round(value * 1e6 * M['flops'] / 1e12, 3),
                              'peak': FP64_PEAK_TFLOPS * world, 'unit': 'TFLOP/s',
                              'frac': round(value * 1e6 * M['flops'] / 1e12 / (FP64_PEAK_TFLOPS * world), 5)},
            'timed_region': stats,
            'host_ms_per_step': {k: round(v[0] / max(a.steps, 1), 3) for k, v in ht.items()},
            'drain_ms': round(tail_ms, 3),
        }
        if h2d is not None:
            out['h2d'] = h2d
        if cpu is not None:
            out['cpu_baseline'] = cpu
            out['vs_cpu'] = round(value / cpu['value'], 1)
        print(json.dumps(out), flush=True)
    eng.close()
    if use_dist:
        dist.destroy_process_group()
    decoded = stats['su_crc_ok'] if M['bitrate'] == 8400 else stats['acars_items']  # C: SUs, no ACARS
    if rank == 0 and (stats[stat_names[0]] <= 0 or decoded <= 0):
        # the metric names demod + Viterbi: a timed region without decoded frames measured something else
        print('bench: timed region decoded no Viterbi jobs / ACARS items (%s)' % stats, file=sys.stderr)
        sys.exit(3)


if __name__ == '__main__':
    main()
