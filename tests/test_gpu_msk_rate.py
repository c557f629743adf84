"""MSK rate change at the boundary: MskDemodulator::dataReceived re-applies
setSettings at a message's sample rate when it differs from the current one
(decode/mskdemodulator.cpp:473-481, settings :94-218), so a 600-bps VFO that
aero-publish emits at an explicit INI out_rate (publish/publisher.cpp:160-176)
still decodes.  The engine moves such a channel to the group of the new rate
with the state setSettings keeps (engine.hip msk_migrate); the oracle
re-applies setSettings (oracle_push_rate).  Soft bits, hop records (f64
bitwise, sample index counted from the channel's first sample), frames and
ACARS items must equal the oracle's, for rate sequences through 12, 24 and 48
kHz and with channels that keep their rate beside them."""
import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu

# (bitrate, [(fs, seconds, seed, carrier Hz, Eb/N0 dB)], message seconds)
CHANNELS = [
    (600, [(12000, 12.0, 0xE100, 1800.0, 14.0), (48000, 6.0, 0xE101, 1800.0, 14.0),
           (24000, 30.0, 0xE102, 1800.0, 14.0)], 0.25),
    (600, [(12000, 24.0, 0xE110, 1500.0, 12.0)], 0.25),                       # stays at 12 kHz
    (1200, [(24000, 10.0, 0xE120, 1800.0, 14.0), (12000, 24.0, 0xE121, 1800.0, 14.0)], 0.5),
    (1200, [(24000, 6.0, 0xE130, 2100.0, 14.0), (48000, 6.0, 0xE131, 2100.0, 14.0),
            (24000, 12.0, 0xE132, 2100.0, 14.0)], 0.125),
]


def _messages(bitrate, segs, msg_s):
    out = []
    for fs, sec, seed, car, eb in segs:
        x = tl.synth_msk(seconds=sec, bitrate=bitrate, baud=600, seed=seed, carrier=car, ebn0=eb, fs=fs)
        step = int(fs * msg_s)
        out += [(x[i:i + step], fs) for i in range(0, len(x), step)]
    return out


def test_msk_rate_change_matches_oracle(engine_lib, msk_kernel):
    import aero_engine as ae
    msgs = [_messages(br, segs, m) for br, segs, m in CHANNELS]
    eng = ae.Engine(max_channels=8, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    chans = [eng.open_channel(br) for br, _, _ in CHANNELS]
    pos = [0] * len(msgs)
    while any(p < len(m) for p, m in zip(pos, msgs)):
        for k, ch in enumerate(chans):
            if pos[k] < len(msgs[k]):
                pcm, fs = msgs[k][pos[k]]
                eng.push(ch, pcm, fs=fs)
                pos[k] += 1
        eng.run()
    eng.flush()
    items_total = 0
    for k, ((br, segs, _), ch) in enumerate(zip(CHANNELS, chans)):
        o = tl.Oracle(bitrate=br)
        for pcm, fs in msgs[k]:
            o.push(pcm, fs=fs)
        sb, rsb = eng.softbits(ch), o.softbits()
        assert len(rsb) > 1000
        assert len(sb) == len(rsb) and np.array_equal(sb, rsb), 'channel %d soft bits differ (%d vs %d)' % (
            k, len(sb), len(rsb))
        h, rh = eng.hops(ch), o.hops()
        assert h.shape == rh.shape and np.array_equal(h.view(np.int64), rh.view(np.int64)), \
            'channel %d hop records differ' % k
        assert np.array_equal(eng.frames(ch), o.frames()), 'channel %d frames differ' % k
        items = eng.items(ch)
        assert items == o.item_lines('A'), 'channel %d items differ' % k
        items_total += len(items)
    assert items_total > 0
    eng.close()


# rates without a fixed-rate group: the generic-rate kernels (demod_msk.hip
# demod_mskg_kernel, coarse bins from MskGen).  16000 and 15000 are what
# aero-publish emits for a 12 kHz out_rate from 2.048 / 1.92 Msps receivers
# (Fs / 2^int(log2(Fs / out_rate)), publish/publisher.cpp:196-210); 18750
# has an odd SPS (31: delayt8 of 15.5 samples, weights 0.5 / 0.5); 96000 is
# the largest rate served
GENERIC = [
    (600, [(16000, 20.0, 0xE300, 1800.0, 14.0)], 0.25),
    (600, [(12000, 6.0, 0xE310, 1500.0, 14.0), (18750, 12.0, 0xE311, 1500.0, 14.0),
           (15000, 8.0, 0xE312, 1500.0, 14.0), (24000, 6.0, 0xE313, 1500.0, 14.0)], 0.25),
    (1200, [(24000, 6.0, 0xE320, 2100.0, 14.0), (40000, 10.0, 0xE321, 2100.0, 14.0),
            (96000, 4.0, 0xE322, 2100.0, 14.0)], 0.25),
    (600, [(96000, 5.0, 0xE330, 1800.0, 14.0)], 0.125),
]


def _run_vs_oracle(eng, chans, spec, msgs):
    pos = [0] * len(msgs)
    while any(p < len(m) for p, m in zip(pos, msgs)):
        for k, ch in enumerate(chans):
            if pos[k] < len(msgs[k]):
                pcm, fs = msgs[k][pos[k]]
                eng.push(ch, pcm, fs=fs)
                pos[k] += 1
        eng.run()
    eng.flush()
    items_total = 0
    for k, ((br, _, _), ch) in enumerate(zip(spec, chans)):
        o = tl.Oracle(bitrate=br)
        for pcm, fs in msgs[k]:
            o.push(pcm, fs=fs)
        sb, rsb = eng.softbits(ch), o.softbits()
        assert len(rsb) > 500
        assert len(sb) == len(rsb) and np.array_equal(sb, rsb), 'channel %d soft bits differ (%d vs %d)' % (
            k, len(sb), len(rsb))
        h, rh = eng.hops(ch), o.hops()
        assert h.shape == rh.shape and np.array_equal(h.view(np.int64), rh.view(np.int64)), \
            'channel %d hop records differ' % k
        assert np.array_equal(eng.frames(ch), o.frames()), 'channel %d frames differ' % k
        items = eng.items(ch)
        assert items == o.item_lines('A'), 'channel %d items differ' % k
        items_total += len(items)
    return items_total


def test_msk_generic_rates_match_oracle(engine_lib, msk_kernel):
    """Channels at and through rates with no fixed-rate group, beside each
    other, against the oracle's setSettings at those rates."""
    import aero_engine as ae
    msgs = [_messages(br, segs, m) for br, segs, m in GENERIC]
    eng = ae.Engine(max_channels=8, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    chans = [eng.open_channel(br) for br, _, _ in GENERIC]
    assert _run_vs_oracle(eng, chans, GENERIC, msgs) > 0
    eng.close()


def test_msk_unsupported_rate_refused(engine_lib):
    import aero_engine as ae
    eng = ae.Engine(max_channels=2)
    ch = eng.open_channel(600)
    for fs in (11025, 96001):  # outside [MSK_FS_MIN, MSK_FS_MAX]
        with pytest.raises(ae.AeroError) as ex:
            eng.push(ch, np.zeros(1000, np.int16), fs=fs)
        assert ex.value.rc == ae.AERO_E_RATE
    eng.push(ch, np.zeros(1000, np.int16), fs=48000)  # a supported rate moves the channel
    eng.push(ch, np.zeros(1000, np.int16), fs=22050)  # and a generic one
    eng.close()


def test_msk_rate_change_in_a_full_group(engine_lib):
    """A group whose every slot is taken (64 channels at 12 kHz, groups hold
    max_channels rounded up to 64): one channel goes to 24 kHz and back.  The
    slot it left is reused on the way back (engine.hip free_slots /
    reset_slot) instead of the move failing with AERO_E_FULL, and the moving
    channel and a neighbour still equal the oracle."""
    import aero_engine as ae
    segs = [(12000, 8.0, 0xE200, 1800.0, 14.0), (24000, 8.0, 0xE201, 1800.0, 14.0),
            (12000, 16.0, 0xE202, 1800.0, 14.0)]
    mover = _messages(600, segs, 0.25)
    stay = _messages(600, [(12000, 32.0, 0xE210, 1500.0, 12.0)], 0.25)
    eng = ae.Engine(max_channels=64, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    chans = [eng.open_channel(600) for _ in range(64)]
    quiet = np.zeros(3000, np.int16)
    for c in chans[2:]:
        eng.push(c, quiet, fs=12000)
    for k in range(max(len(mover), len(stay))):
        if k < len(mover):
            eng.push(chans[0], mover[k][0], fs=mover[k][1])
        if k < len(stay):
            eng.push(chans[1], stay[k][0], fs=stay[k][1])
        eng.run()
    eng.flush()
    for ch, msgs in ((chans[0], mover), (chans[1], stay)):
        o = tl.Oracle(bitrate=600)
        for pcm, fs in msgs:
            o.push(pcm, fs=fs)
        sb, rsb = eng.softbits(ch), o.softbits()
        assert len(rsb) > 1000 and np.array_equal(sb, rsb), 'channel %d soft bits differ' % ch
        h, rh = eng.hops(ch), o.hops()
        assert h.shape == rh.shape and np.array_equal(h.view(np.int64), rh.view(np.int64)), ch
        assert eng.items(ch) == o.item_lines('A'), 'channel %d items differ' % ch
    eng.close()


def test_generic_groups_small_and_released(engine_lib):
    """A 65536-channel engine whose one MSK channel moves through generic
    rates: each generic-rate group holds at most 256 channels (a 96 kHz group
    sized for 65536 would ask for ~50 GB of AGC ring), a group is released
    when its last channel leaves, a rate's group is re-created when the
    channel comes back, and the channel still equals the oracle."""
    import aero_engine as ae
    segs = [(15000, 4.0, 0xE400, 1800.0, 14.0), (96000, 2.0, 0xE401, 1800.0, 14.0),
            (18750, 4.0, 0xE402, 1800.0, 14.0), (40000, 3.0, 0xE403, 1800.0, 14.0),
            (15000, 10.0, 0xE404, 1800.0, 14.0)]
    msgs = _messages(600, segs, 0.25)
    eng = ae.Engine(max_channels=65536, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_FRAMES)
    ch = eng.open_channel(600, 15000)
    last_fs, peak = None, 0
    for pcm, fs in msgs:
        eng.push(ch, pcm, fs=fs)
        eng.run()
        if fs != last_fs:
            # one group alive (the channel's), sized for 256 channels
            assert eng.stat('groups') == 1, 'a left generic group was kept'
            peak = max(peak, eng.stat('device_bytes'))
            last_fs = fs
    eng.flush()
    assert peak < (2 << 30), 'generic group pools too large: %d bytes' % peak
    o = tl.Oracle(bitrate=600)
    for pcm, fs in msgs:
        o.push(pcm, fs=fs)
    sb, rsb = eng.softbits(ch), o.softbits()
    assert len(rsb) > 1000 and np.array_equal(sb, rsb)
    h, rh = eng.hops(ch), o.hops()
    assert h.shape == rh.shape and np.array_equal(h.view(np.int64), rh.view(np.int64))
    assert np.array_equal(eng.frames(ch), o.frames())
    eng.close()
