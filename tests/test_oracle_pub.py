"""Oracle properties of the aero-publish channeliser restatement
(oracle/pub_oracle.cpp; publish/publisher.cpp, vfo.cpp, halfbanddecimator.*,
dsp.cpp, oscillator.cpp, firfilter.cpp).  The publisher needs QtCore and
SoapySDR, so the restatement is pinned by known answers and behaviour only:
parity unpinned against the compiled reference."""
import numpy as np
import pytest

import aero_testlib as tl

C = tl.CENTER


@pytest.mark.parametrize('fs,blk', [(288000, 57600), (1536000, 384000), (1920000, 480000)])
def test_read_length(cpu_libs, fs, blk):
    """buflen/2 complex samples per read: 4 reads a second, 5 when 2*Fs/4 is
    not a multiple of 512 (publish/publisher.cpp:92-100)."""
    p = tl.OraclePublisher(fs, C, [dict(frequency=C, out_rate=fs, publish=1)], [])
    assert p.block_len == blk


def test_vfo_plans(cpu_libs):
    """Decimation plans of publish/publisher.cpp:183-217 and vfo.cpp:57-88."""
    cfg = tl.PUB_CONFIGS['r1536k']
    p = tl.OraclePublisher(cfg['sample_rate'], C, cfg['mains'], cfg['vfos'])
    got = [p.info(v) for v in range(4)]
    assert [(g['main'], g['out_rate'], g['halfbands'], g['late']) for g in got] == [
        (0, 48000, 2, 0), (0, 12000, 4, 0), (1, 24000, 3, 0), (1, 48000, 2, 0)]
    assert [g['samples_per_block'] for g in got] == [12000, 3000, 6000, 12000]
    assert got[1]['usb_taps'] > 0 and got[0]['usb_taps'] == 0
    p = tl.OraclePublisher(1920000, C, [dict(frequency=C, out_rate=240000)],
                           [dict(frequency=C + 1000, data_rate=10500), dict(frequency=C, data_rate=600)])
    assert [(p.info(v)['halfbands'], p.info(v)['late'], p.info(v)['out_rate']) for v in range(2)] == [
        (0, 5, 48000), (2, 5, 12000)]
    assert p.info(0)['late_taps'] == 49  # ntaps = int(53*240000/(22*12000)) = 48 -> odd 49
    p = tl.OraclePublisher(288000, C, [dict(frequency=C, out_rate=288000)], [dict(frequency=C, data_rate=600)])
    assert (p.info(0)['halfbands'], p.info(0)['late'], p.info(0)['samples_per_block']) == (2, 6, 2400)


def test_uncovered_vfo_refused(cpu_libs):
    with pytest.raises(ValueError):
        tl.OraclePublisher(1536000, C, [dict(frequency=C, out_rate=192000)], [dict(frequency=C + 500000, data_rate=600)])


def _tone_bin(x, fs, f):
    spec = np.abs(np.fft.rfft(x.astype(np.float64) * np.hanning(len(x))))
    return spec[int(round(f * len(x) / fs))], spec


@pytest.mark.parametrize('sign', [1, -1])
def test_usb_selects_upper_sideband(cpu_libs, sign):
    """A tone f Hz above a VFO comes out as an f Hz audio tone; f Hz below is
    attenuated by the Hilbert USB demodulator (vfo.cpp:188-214).  Only by
    about 15 dB: FIRHilbert normalises its taps to unit energy, not unit
    passband gain (publish/dsp.cpp:210-214), so the arms do not cancel fully."""
    fs, f = 288000, 1500.0
    vfo = dict(frequency=C + 20000, data_rate=10500, gain=100.0)
    p = tl.OraclePublisher(fs, C, [dict(frequency=C, out_rate=fs)], [vfo])
    blk = p.block_len
    x = tl.wideband(fs, 4 * blk, 7, tones=[(20000.0 + sign * f, 0.3)], noise=0.001)
    p.process(x)
    a = p.usb(0)
    assert len(a) == 4 * 9600
    peak, spec = _tone_bin(a[9600:], 48000, f)
    if sign > 0:
        assert peak > 50 * np.median(spec)
    else:
        ref = tl.OraclePublisher(fs, C, [dict(frequency=C, out_rate=fs)], [vfo])
        ref.process(tl.wideband(fs, 4 * blk, 7, tones=[(20000.0 + f, 0.3)], noise=0.001))
        upper, _ = _tone_bin(ref.usb(0)[9600:], 48000, f)
        assert peak < upper / 4


def test_reads_are_processed_in_order(cpu_libs):
    """One call per read or all reads at once: identical audio (demodData per read)."""
    cfg = tl.PUB_CONFIGS['r288k']
    a = tl.OraclePublisher(cfg['sample_rate'], C, cfg['mains'], cfg['vfos'], correct_dc_bias=True)
    b = tl.OraclePublisher(cfg['sample_rate'], C, cfg['mains'], cfg['vfos'], correct_dc_bias=True)
    x = tl.wideband(cfg['sample_rate'], 3 * a.block_len, 3, cfg['tones'])
    a.process(x)
    for k in range(3):
        b.process(x[k * a.block_len:(k + 1) * a.block_len])
    for v in range(len(cfg['vfos'])):
        assert np.array_equal(a.usb(v), b.usb(v))


def test_main_vfo_iq_output(cpu_libs):
    """A main VFO without sub-VFOs publishes 4-bit packed IQ (vfo.cpp:262-274)."""
    cfg = tl.PUB_CONFIGS['r1536k']
    p = tl.OraclePublisher(cfg['sample_rate'], C, cfg['mains'], cfg['vfos'])
    p.process(tl.wideband(cfg['sample_rate'], p.block_len, 5, cfg['tones']))
    assert len(p.iq(2)) == 48000 and len(p.iq(0)) == 0
