"""Decoder status events and item latency on the GPU.

- aero_channel_get_events against the oracle: the data-carrier-detect
  changes SignalHunter::handleDcd passes to Decoder::handleDcdChange and
  the centres of SignalHunter::newFreqCenter (decode/hunter.cpp:14-40,
  decode/decode.cpp:429-439), for continuous OQPSK / MSK channels with and
  without a signal and for burst OQPSK / MSK channels (DCD per burst).
- aero_run launches the decode of its last pass before returning: the items
  of every frame completed by the samples a run consumed come out of
  aero_pop_items without more audio, aero_sync or aero_flush (the reference
  emits them as soon as they are decoded).
"""
import time

import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu


def _noise(seconds, seed, fs=48000):
    return (np.random.default_rng(seed).normal(0, 300, int(fs * seconds))).astype(np.int16)


def test_events_continuous(engine_lib, cpu_libs):
    import aero_engine as ae
    cases = [  # bitrate, fs, pcm, chunk
        (10500, 48000, tl.synth(seconds=10.0, seed=0xAE50, carrier=12037.5, ebn0=12.0), 12000),
        (10500, 48000, _noise(14.0, 1), 12000),
        (600, 12000, tl.synth_msk(seconds=12.0, bitrate=600, baud=600, seed=0xAE51, carrier=300.0, ebn0=12.0), 3000),
        (600, 12000, _noise(20.0, 2, 12000), 3000),
    ]
    eng = ae.Engine(max_channels=len(cases))
    chans = [eng.open_channel(b, fs) for b, fs, _, _ in cases]
    pos = [0] * len(cases)
    while any(p < len(c[2]) for p, c in zip(pos, cases)):
        for k, (b, fs, pcm, chunk) in enumerate(cases):
            if pos[k] < len(pcm):
                eng.push(chans[k], pcm[pos[k]:pos[k] + chunk])
                pos[k] += chunk
        eng.run()
    eng.flush()
    for (b, fs, pcm, chunk), ch in zip(cases, chans):
        ref = tl.Oracle(bitrate=b)
        ref.push_chunked(pcm, chunk)
        want_dcd, want_fc = ref.events()
        dcd, steps, fcs = eng.channel_events(ch)
        assert dcd == want_dcd, (b, dcd, want_dcd)
        assert steps == len(want_fc), (b, steps, len(want_fc))
        assert fcs == want_fc[-8:], (b, fcs, want_fc[-8:])
    # the noise channels scanned, the signal channels locked
    assert eng.channel_events(chans[1])[1] >= 4 and eng.channel_events(chans[3])[1] >= 4
    assert eng.channel_events(chans[0])[0] == 1 and eng.channel_events(chans[2])[0] == 1
    eng.close()


def test_events_burst(engine_lib, cpu_libs):
    import aero_engine as ae
    cases = [
        (10500, tl.synth_burst(seconds=12.0, seed=0xAE52, carrier=12000.0, ebn0=14.0)),
        (1200, tl.synth_burst_msk(seconds=12.0, bitrate=1200, seed=0xAE53, carrier=2500.0, ebn0=14.0)),
    ]
    eng = ae.Engine(max_channels=len(cases))
    chans = [eng.open_channel(b, 48000, burst=True) for b, _ in cases]
    for (b, pcm), ch in zip(cases, chans):
        for i in range(0, len(pcm), 12000):
            eng.push(ch, pcm[i:i + 12000])
            eng.run()
    eng.flush()
    for (b, pcm), ch in zip(cases, chans):
        ref = tl.Oracle(bitrate=b, burst=True)
        ref.push_chunked(pcm, 12000)
        want_dcd, want_fc = ref.events()
        dcd, steps, _ = eng.channel_events(ch)
        # the burst window (10500 bits) only ends after many bursts, so the
        # carrier usually stays detected after the first one
        assert want_dcd >= 1, 'the synthetic stream carries bursts'
        assert (dcd, steps) == (want_dcd, 0), (b, dcd, want_dcd)
    eng.close()


def test_items_leave_without_more_audio(engine_lib, cpu_libs):
    """the last pass's Viterbi used to wait for the next pass."""
    import aero_engine as ae
    pcm = tl.synth(seconds=12.0, seed=0xAE54, carrier=12037.5, ebn0=12.0)
    eng = ae.Engine(max_channels=1)
    ch = eng.open_channel(10500, 48000)
    got, late = [], []
    for i in range(0, len(pcm), 12000):
        eng.push(ch, pcm[i:i + 12000])
        eng.run()
        # poll until nothing new arrives for 300 ms (the GPU and host work of
        # one message take a few ms)
        last, t_last = len(got), time.time()
        while time.time() - t_last < 0.3:
            got += eng.items(ch)
            if len(got) != last:
                last, t_last = len(got), time.time()
            time.sleep(0.02)
        eng.sync()  # would launch a deferred decode: nothing may be left
        late += eng.items(ch)
    eng.flush()
    tail = eng.items(ch)
    eng.close()
    assert not late, '%d items waited for aero_sync' % len(late)
    ref = tl.Oracle()
    ref.push_chunked(pcm, 12000)
    assert got + tail == ref.item_lines('A') and len(got) >= 10
