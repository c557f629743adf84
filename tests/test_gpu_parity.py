"""GPU parity: the HIP engine vs the CPU oracle on the same synthetic VFO
streams.  Integer outputs (soft bits, coarse-hop decisions, Viterbi blocks,
CRC-checked frames, ACARS items) must be bit-exact; the rotated pt_qpsk
soft-metric floats within 1e-5 (BASELINE.json north_star)."""
import numpy as np
import pytest

import aero_testlib as tl

PT_TOL = 1e-5

CASES = [
    # seed, carrier Hz, Eb/N0 dB, seconds, message size (samples)
    (0xAE20, 12037.5, 12.0, 14.0, 12000),
    (0xAE21, 12038.0, 9.0, 14.0, 12000),
    (0xAE22, 7020.0, 12.0, 12.0, 3000),
    (0xAE23, 15500.0, 10.0, 12.0, 48000),
]


def _run_engine(streams, chunks, flags):
    import aero_engine as ae
    eng = ae.Engine(max_channels=len(streams), flags=flags)
    chans = [eng.open_channel(10500, 48000) for _ in streams]
    pos = [0] * len(streams)
    while any(p < len(s) for p, s in zip(pos, streams)):
        for k, (s, ch) in enumerate(zip(streams, chans)):
            if pos[k] < len(s):
                eng.push(ch, s[pos[k]:pos[k] + chunks[k]])
                pos[k] += chunks[k]
        eng.run()
    eng.flush()
    return eng, chans


@pytest.mark.gpu
def test_engine_matches_oracle(engine_lib, oqpsk_kernel):
    import aero_engine as ae
    streams = [tl.synth(seconds=sec, seed=seed, carrier=f, ebn0=eb) for seed, f, eb, sec, _ in CASES]
    chunks = [c[4] for c in CASES]
    eng, chans = _run_engine(streams, chunks, ae.F_TRACE_ALL)
    for k, (s, ch) in enumerate(zip(streams, chans)):
        o = tl.Oracle(trace_pt=True)
        o.push_chunked(s, chunks[k])
        sb_o, sb_e = o.softbits(), eng.softbits(ch)
        assert len(sb_o) > 1000, 'oracle did not lock on case %d' % k
        assert len(sb_e) == len(sb_o), 'case %d soft-bit count %d vs %d' % (k, len(sb_e), len(sb_o))
        assert np.array_equal(sb_e, sb_o), 'case %d soft bits differ at %s' % (
            k, np.nonzero(sb_e != sb_o)[0][:10])
        h_o, h_e = o.hops(), eng.hops(ch)
        assert h_o.shape == h_e.shape
        assert np.array_equal(h_e, h_o), 'case %d hop records differ' % k
        p_o, p_e = o.pt(), eng.pt(ch)
        assert p_o.shape == p_e.shape
        assert np.max(np.abs(p_o - p_e)) <= PT_TOL
        assert np.array_equal(eng.blocks(ch), o.blocks()), 'case %d Viterbi blocks differ' % k
        assert np.array_equal(eng.frames(ch), o.frames()), 'case %d frames differ' % k
        items_o = o.item_lines('A')
        assert len(items_o) > 0
        assert eng.items(ch) == items_o, 'case %d ACARS items differ' % k
    eng.close()


@pytest.mark.gpu
def test_fragment_items_disable_reassembly(engine_lib):
    import aero_engine as ae
    s = tl.synth(seconds=12.0, seed=0xAE30, carrier=12040.0, ebn0=12.0)
    eng = ae.Engine(max_channels=1, flags=0)
    ch = eng.open_channel(10500, 48000, disable_reassembly=True)
    for i in range(0, len(s), 12000):
        eng.push(ch, s[i:i + 12000])
        eng.run()
    eng.flush()
    o = tl.Oracle()
    o.push_chunked(s, 12000)
    assert eng.items(ch) == o.item_lines('F')
    eng.close()


@pytest.mark.gpu
def test_batch_push_equals_channel_push(engine_lib, oqpsk_kernel):
    """Lockstep batch ingest (bench path) == per-channel ZMQ-message ingest."""
    import aero_engine as ae
    nch = 6
    streams = [tl.synth(seconds=9.0, seed=0xAE40 + k, carrier=12037.5 + 0.5 * k, ebn0=11.0) for k in range(nch)]
    pcm = np.stack(streams, axis=1)
    e1 = ae.Engine(max_channels=nch, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS)
    for _ in range(nch):
        e1.open_channel()
    drained = []
    for i in range(0, pcm.shape[0], 4096):
        e1.push_batch(pcm[i:i + 4096])
        e1.run()
        drained += e1.drain_items(lines=True)  # aero_pop_items_all between runs
    e1.flush()
    drained += e1.drain_items(lines=True)
    e2, chans = _run_engine(streams, [12000] * nch, ae.F_TRACE_SOFT | ae.F_TRACE_HOPS)
    for c in range(nch):
        assert np.array_equal(e1.softbits(c), e2.softbits(chans[c]))
        assert np.array_equal(e1.hops(c), e2.hops(chans[c]))
        assert [line for ch, line in drained if ch == c] == e2.items(chans[c])
    assert drained
    e1.close()
    e2.close()


@pytest.mark.gpu
def test_many_channels_multiple_waves(engine_lib, oqpsk_kernel):
    """70 channels (three wavefronts, out of step with each other: different
    carriers, phases, noise and push sizes) against the oracle, channel by
    channel: soft bits and ACARS items."""
    import aero_engine as ae
    nch = 70
    rng = np.random.default_rng(3)
    streams = [tl.synth(seconds=6.0, seed=0xAE60 + k, carrier=float(rng.uniform(11900, 12100)),
                        ebn0=float(rng.uniform(9, 14)), phase0=float(rng.uniform(0, 6.28)))
               for k in range(nch)]
    chunks = [int(rng.choice([1000, 4096, 12000, 30000])) for _ in range(nch)]
    eng, chans = _run_engine(streams, chunks, ae.F_TRACE_SOFT)
    for k in range(nch):
        o = tl.Oracle()
        o.push_chunked(streams[k], 12000)
        assert np.array_equal(eng.softbits(chans[k]), o.softbits()), 'channel %d soft bits differ' % k
        assert eng.items(chans[k]) == o.item_lines('A'), 'channel %d items differ' % k
    eng.close()


@pytest.mark.gpu
def test_documented_channel_config_per_bitrate(engine_lib):
    """INTEGRATION.md's binding: aero_channel_open with the rate each bit
    rate's audio arrives at (decode/decode.cpp:145, 152-159) for every
    aero-decode bit rate; AERO_E_INVALID for 10500 bps at another rate,
    AERO_E_RATE for MSK at a rate outside [12000, 96000] Hz, and any MSK rate
    inside it (a generic-rate group)."""
    import ctypes
    import aero_engine as ae
    eng = ae.Engine(max_channels=4)
    lib = ae.load_library()
    for bitrate in (10500, 600, 1200):
        fs = 12000 if bitrate == 600 else (24000 if bitrate == 1200 else 48000)
        cfg = ae.ChannelCfg(bitrate, 0, fs, 0)
        ch = ctypes.c_int()
        assert lib.aero_channel_open(eng.h, ctypes.byref(cfg), ctypes.byref(ch)) == ae.AERO_OK, bitrate
        bad = ae.ChannelCfg(bitrate, 0, 11025, 0)
        want = ae.AERO_E_INVALID if bitrate == 10500 else ae.AERO_E_RATE
        assert lib.aero_channel_open(eng.h, ctypes.byref(bad), ctypes.byref(ch)) == want, bitrate
    cfg = ae.ChannelCfg(600, 0, 16000, 0)
    assert lib.aero_channel_open(eng.h, ctypes.byref(cfg), ctypes.byref(ch)) == ae.AERO_OK
    eng.close()


@pytest.mark.gpu
def test_queued_host_messages_between_runs(engine_lib):
    """Host messages are queued in pinned staging and reach the PCM rings as
    one gather launch per run (engine.hip hostq_flush): several messages per
    channel between two runs (the multi-topic aero-decode batch), of
    different sizes, a device push on another channel in between (which
    flushes the queue first), and a message larger than half the ring (the
    overrun guard runs the group mid-queue).  Soft bits, hops and items equal
    the oracle fed the same messages."""
    import torch
    import aero_engine as ae
    streams = [tl.synth(seconds=9.0, seed=0xAE60 + k, carrier=9000.0 + 1500.0 * k) for k in range(3)]
    eng = ae.Engine(max_channels=3, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS)
    chans = [eng.open_channel(10500, 48000) for _ in streams]
    sizes = [(1000, 2500, 700, 4096), (12000,), (5000, 20000)]
    pos = [0, 0, 0]
    dev = torch.from_numpy(streams[1]).to('cuda')
    rnd = 0
    while any(p < len(s) for p, s in zip(pos, streams)):
        for k in (0, 2):
            for sz in sizes[k] * 2:  # several messages of each channel before one run
                if pos[k] < len(streams[k]):
                    eng.push(chans[k], streams[k][pos[k]:pos[k] + sz])
                    pos[k] += sz
            if k == 0 and pos[1] < len(streams[1]):
                n = min(12000, len(streams[1]) - pos[1])
                torch.cuda.synchronize()
                eng.push_device(chans[1], dev[pos[1]:pos[1] + n].data_ptr(), n)
                pos[1] += n
        if rnd % 3 == 2 and pos[0] < len(streams[0]):  # larger than half the PCM ring
            eng.push(chans[0], streams[0][pos[0]:pos[0] + 40000])
            pos[0] += 40000
        eng.run()
        rnd += 1
    eng.flush()
    for k, s in enumerate(streams):
        o = tl.Oracle()
        o.push_chunked(s, 4096)
        assert len(o.softbits()) > 1000
        assert np.array_equal(eng.softbits(chans[k]), o.softbits()), 'channel %d soft bits differ' % k
        h = eng.hops(chans[k])
        assert np.array_equal(h.view(np.int64), o.hops().view(np.int64)), 'channel %d hops differ' % k
        assert eng.items(chans[k]) == o.item_lines('A') and o.item_lines('A'), 'channel %d items differ' % k
    eng.close()
