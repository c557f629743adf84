"""Test helpers: synthetic VFO input (tools/libaero_synth.so) and the oracle
(oracle/liboracle.so, the checker).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg use the oracle."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'aero-cli_amd')
if PKG not in sys.path:
    sys.path.insert(0, PKG)

# AERO_ORACLE_SO / AERO_SYNTH_SO: the AddressSanitizer builds (tests/asan_check.sh)
ORACLE_SO = os.environ.get('AERO_ORACLE_SO') or os.path.join(ROOT, 'oracle', 'liboracle.so')
SYNTH_SO = os.environ.get('AERO_SYNTH_SO') or os.path.join(ROOT, 'tools', 'libaero_synth.so')


class SynthCfg(ctypes.Structure):
    _fields_ = [('fs', ctypes.c_double), ('carrier_hz', ctypes.c_double), ('phase0', ctypes.c_double),
                ('amplitude', ctypes.c_double), ('ebn0_db', ctypes.c_double), ('seed', ctypes.c_uint64),
                ('msg_rate', ctypes.c_double), ('lead_in', ctypes.c_int)]


def build_all():
    import build  # aero-cli_amd/build.py
    return build.build_all()


def build_cpu_only():
    import build
    build.build_oracle()
    build.build_synth()
    build.build_fftsim()


_synth = None


def synth(seconds=10.0, seed=0xAE20, carrier=12037.5, ebn0=12.0, amplitude=0.25, phase0=0.3, msg_rate=0.6,
          lead_in=1000, fs=48000.0, return_frames=False):
    """int16 PCM of an Aero P-channel (SURVEY.md §8(d) C1/C2 input) + the
    transmitted 312-byte information fields per frame."""
    global _synth
    if _synth is None:
        _synth = ctypes.CDLL(SYNTH_SO)
        _synth.aero_synth_p10500.restype = ctypes.c_size_t
    n = int(fs * seconds)
    pcm = np.zeros(n, dtype=np.int16)
    maxf = int(seconds * 2) + 8
    frames = np.zeros(312 * maxf, dtype=np.uint8)
    cfg = SynthCfg(fs, carrier, phase0, amplitude, ebn0, seed, msg_rate, lead_in)
    nf = _synth.aero_synth_p10500(ctypes.byref(cfg), pcm.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                                  frames.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(maxf))
    if return_frames:
        return pcm, frames[:312 * min(nf, maxf)].reshape(-1, 312)
    return pcm


def synth_msk(seconds=10.0, bitrate=600, seed=0xAE40, carrier=1800.0, ebn0=12.0, amplitude=0.25, phase0=0.3,
              msg_rate=0.6, lead_in=500, baud=None, return_frames=False, fs=None):
    """int16 PCM of a 600/1200-bps MSK P-channel at 12/24 kHz (SURVEY.md §8(d)
    C3 input; `fs` overrides the rate) + the transmitted 72-byte information
    fields per frame.  `baud` (default = bitrate) is the modulation rate; the
    frame layout follows `bitrate`."""
    global _synth
    if _synth is None:
        _synth = ctypes.CDLL(SYNTH_SO)
    _synth.aero_synth_msk.restype = ctypes.c_size_t
    fs = float(fs) if fs else (12000.0 if bitrate == 600 else 24000.0)
    n = int(fs * seconds)
    pcm = np.zeros(n, dtype=np.int16)
    maxf = int(seconds * (baud or bitrate) / 1200) + 8
    frames = np.zeros(72 * maxf, dtype=np.uint8)
    cfg = SynthCfg(fs, carrier, phase0, amplitude, ebn0, seed, msg_rate, lead_in)
    nf = _synth.aero_synth_msk(ctypes.byref(cfg), ctypes.c_int(bitrate), ctypes.c_int(baud or bitrate),
                               pcm.ctypes.data_as(ctypes.c_void_p),
                               ctypes.c_size_t(n), frames.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(maxf))
    if return_frames:
        return pcm, frames[:72 * min(nf, maxf)].reshape(-1, 72)
    return pcm


def synth_c(seconds=10.0, seed=0xAEC0, carrier=12000.0, ebn0=12.0, amplitude=0.25, phase0=0.3, lead_in=1000,
            return_frames=False):
    """int16 48 kHz PCM of an 8400-bps C channel (tools/aero_synth.cpp
    aero_synth_c8400) + per frame the 36 transmitted SU bytes and 300 voice bytes."""
    global _synth
    if _synth is None:
        _synth = ctypes.CDLL(SYNTH_SO)
    _synth.aero_synth_c8400.restype = ctypes.c_size_t
    n = int(48000 * seconds)
    pcm = np.zeros(n, dtype=np.int16)
    maxf = int(seconds * 2) + 8
    frames = np.zeros(336 * maxf, dtype=np.uint8)
    cfg = SynthCfg(48000.0, carrier, phase0, amplitude, ebn0, seed, 0.6, lead_in)
    nf = _synth.aero_synth_c8400(ctypes.byref(cfg), pcm.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                                 frames.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(maxf))
    if return_frames:
        return pcm, frames[:336 * min(nf, maxf)].reshape(-1, 336)
    return pcm


def synth_burst(seconds=10.0, seed=0xAE50, carrier=12000.0, ebn0=14.0, amplitude=0.25, phase0=0.3, lead_in=24000,
                return_packets=False):
    """int16 48 kHz PCM of 10500-bps burst OQPSK R/T packets (SURVEY.md §8(d)
    C4 input) + the transmitted packets [(kind 'R'/'T', bytes)]."""
    global _synth
    if _synth is None:
        _synth = ctypes.CDLL(SYNTH_SO)
    _synth.aero_synth_burst.restype = ctypes.c_size_t
    n = int(48000 * seconds)
    pcm = np.zeros(n, dtype=np.int16)
    cap = int(seconds + 4) * 400
    buf = np.zeros(cap, dtype=np.uint8)
    npk = ctypes.c_size_t()
    cfg = SynthCfg(48000.0, carrier, phase0, amplitude, ebn0, seed, 0.6, lead_in)
    used = _synth.aero_synth_burst(ctypes.byref(cfg), pcm.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n),
                                   buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(cap), ctypes.byref(npk))
    if not return_packets:
        return pcm
    pk, i = [], 0
    while i < used:
        kind, ln = np.frombuffer(buf[i:i + 8].tobytes(), np.uint32)
        pk.append((chr(kind), bytes(buf[i + 8:i + 8 + ln])))
        i += 8 + int(ln)
    return pcm, pk


def synth_burst_msk(seconds=10.0, bitrate=1200, seed=0xAE70, carrier=2500.0, ebn0=14.0, amplitude=0.25, phase0=0.3,
                    lead_in=24000, p1=126, p2=74, alt_sign=1, return_packets=False):
    """int16 48 kHz PCM of 1200-baud burst MSK R/T packets for `aero-decode
    -b <bitrate> --burst` (p1 carrier / p2 alternating preamble bit periods)
    + the transmitted packets [(kind 'R'/'T', bytes)]."""
    global _synth
    if _synth is None:
        _synth = ctypes.CDLL(SYNTH_SO)
    _synth.aero_synth_burst_msk.restype = ctypes.c_size_t
    n = int(48000 * seconds)
    pcm = np.zeros(n, dtype=np.int16)
    cap = int(seconds + 4) * 400
    buf = np.zeros(cap, dtype=np.uint8)
    npk = ctypes.c_size_t()
    cfg = SynthCfg(48000.0, carrier, phase0, amplitude, ebn0, seed, 0.6, lead_in)
    used = _synth.aero_synth_burst_msk(ctypes.byref(cfg), ctypes.c_int(bitrate), ctypes.c_int(p1), ctypes.c_int(p2),
                                       ctypes.c_int(alt_sign), pcm.ctypes.data_as(ctypes.c_void_p),
                                       ctypes.c_size_t(n), buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(cap),
                                       ctypes.byref(npk))
    if not return_packets:
        return pcm
    pk, i = [], 0
    while i < used:
        kind, ln = np.frombuffer(buf[i:i + 8].tobytes(), np.uint32)
        pk.append((chr(kind), bytes(buf[i + 8:i + 8 + ln])))
        i += 8 + int(ln)
    return pcm, pk


class Oracle:
    """One reference channel (a whole `aero-decode -b <bitrate>` instance)."""
    _libs = {}

    @classmethod
    def lib(cls):
        if 'L' not in cls._libs:
            L = ctypes.CDLL(ORACLE_SO)
            L.oracle_create.restype = ctypes.c_void_p
            L.oracle_create.argtypes = [ctypes.c_int, ctypes.c_int]
            L.oracle_destroy.argtypes = [ctypes.c_void_p]
            L.oracle_push.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
            L.oracle_push_rate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            for f in ('oracle_softbits', 'oracle_blocks', 'oracle_frames', 'oracle_items'):
                getattr(L, f).restype = ctypes.c_size_t
                getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
            for f in ('oracle_hops', 'oracle_pt'):
                getattr(L, f).restype = ctypes.c_size_t
                getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
            L.oracle_conv_encode.restype = ctypes.c_size_t
            L.oracle_conv_encode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
            L.oracle_viterbi_decode_soft.restype = ctypes.c_size_t
            L.oracle_viterbi_decode_soft.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
            L.oracle_crc16_bytes.restype = ctypes.c_uint16
            L.oracle_crc16_bytes.argtypes = [ctypes.c_void_p, ctypes.c_int]
            L.oracle_scrambler_bits.argtypes = [ctypes.c_void_p, ctypes.c_int]
            L.oracle_deinterleave_perm.argtypes = [ctypes.c_int, ctypes.c_void_p]
            L.oracle_rrc_design.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                            ctypes.c_void_p]
            L.oracle_cis_table.argtypes = [ctypes.c_void_p]
            L.oracle_twiddles.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
            L.oracle_fft.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
            L.oracle_msk_taps.argtypes = [ctypes.c_int, ctypes.c_void_p]
            for f in ('oracle_softbits16', 'oracle_rt_tests', 'oracle_rt_packets', 'oracle_c_units', 'oracle_voice'):
                getattr(L, f).restype = ctypes.c_size_t
                getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
            L.oracle_events.restype = ctypes.c_size_t
            L.oracle_events.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_void_p,
                                        ctypes.c_size_t]
            cls._libs['L'] = L
        return cls._libs['L']

    def __init__(self, trace_pt=False, bitrate=10500, burst=False, dcd_tick=False):
        self.L = self.lib()
        self.bitrate = bitrate
        self.h = self.L.oracle_create(bitrate, (1 if trace_pt else 0) | (2 if burst else 0) | (4 if dcd_tick else 0))
        assert self.h, 'oracle_create(%d) failed' % bitrate

    def __del__(self):
        if getattr(self, 'h', None):
            self.L.oracle_destroy(self.h)
            self.h = None

    def push(self, pcm, fs=None):
        """One message; with `fs` the message's sample rate (an MSK channel
        re-applies its settings when it changes)."""
        pcm = np.ascontiguousarray(pcm, dtype=np.int16)
        if fs is None:
            self.L.oracle_push(self.h, pcm.ctypes.data, pcm.size)
        else:
            self.L.oracle_push_rate(self.h, pcm.ctypes.data, pcm.size, int(fs))

    def push_chunked(self, pcm, chunk=12000, fs=None):
        for i in range(0, len(pcm), chunk):
            self.push(pcm[i:i + chunk], fs)

    def _get(self, fn, dtype, rec=1):
        n = fn(self.h, None, 0)
        buf = np.zeros(n * rec, dtype=dtype)
        fn(self.h, buf.ctypes.data, n)
        return buf.reshape(-1, rec) if rec > 1 else buf

    def softbits(self):
        return self._get(self.L.oracle_softbits, np.uint8)

    def softbits16(self):
        """burst: delivered soft bits with the -1 start-of-packet markers"""
        return self._get(self.L.oracle_softbits16, np.int16)

    def rt_tests(self):
        """burst: (blockptr, result code) of every R/T test"""
        return self._get(self.L.oracle_rt_tests, np.uint8).view(np.uint32).reshape(-1, 2)

    def rt_packets(self):
        """burst: [(kind 'R'/'T', infofield bytes)] of every decoded R/T packet"""
        raw = self._get(self.L.oracle_rt_packets, np.uint8)
        return parse_rt_packets(raw)

    def c_units(self):
        """C channel: every CRC-valid Call_progress SU (12 bytes each)"""
        return self._get(self.L.oracle_c_units, np.uint8).reshape(-1, 12)

    def voice(self):
        """C channel: per frame (AES of its last Call_progress, 300 voice bytes)"""
        raw = self._get(self.L.oracle_voice, np.uint8).reshape(-1, 304)
        return [(int(np.frombuffer(r[:4].tobytes(), np.uint32)[0]), bytes(r[4:])) for r in raw]

    def hops(self):
        return self._get(self.L.oracle_hops, np.float64, 6)

    def pt(self):
        return self._get(self.L.oracle_pt, np.float64, 2)

    def blocks(self):
        return self._get(self.L.oracle_blocks, np.uint8)

    def frames(self):
        return self._get(self.L.oracle_frames, np.uint8)

    def events(self):
        """(dcd_edges, [centre of every SignalHunter step]) (decode/decode.cpp:429-439)"""
        e = ctypes.c_longlong()
        n = self.L.oracle_events(self.h, ctypes.byref(e), None, 0)
        fc = np.zeros(n, dtype=np.float64)
        self.L.oracle_events(self.h, ctypes.byref(e), fc.ctypes.data, n)
        return int(e.value), [float(v) for v in fc]

    def item_lines(self, kind='A'):
        n = self.L.oracle_items(self.h, None, 0)
        b = ctypes.create_string_buffer(n + 1)
        self.L.oracle_items(self.h, b, n)
        lines = b.raw[:n].decode().splitlines()
        return [l for l in lines if l.startswith(kind + ' ')]


def frame_records(raw):
    """320-byte frame records -> list of (info bytes, crc-ok mask)."""
    raw = np.asarray(raw, dtype=np.uint8).reshape(-1, 320)
    out = []
    for r in raw:
        L = int(np.frombuffer(r[312:316].tobytes(), np.uint32)[0])
        m = int(np.frombuffer(r[316:320].tobytes(), np.uint32)[0])
        out.append((bytes(r[:L]), m))
    return out


def parse_rt_packets(raw):
    raw = np.asarray(raw, dtype=np.uint8)
    out, i = [], 0
    while i < len(raw):
        kind, ln = np.frombuffer(raw[i:i + 8].tobytes(), np.uint32)
        out.append((chr(kind), bytes(raw[i + 8:i + 8 + int(ln)])))
        i += 8 + int(ln)
    return out


class OraclePublisher:
    """oracle/pub_oracle.cpp: aero-publish's channeliser restated sample by
    sample (the checker for aero-cli_amd/csrc/chan.hip)."""
    _ready = False

    @classmethod
    def lib(cls):
        L = Oracle.lib()
        if not cls._ready:
            c = ctypes
            L.oracle_pub_create.restype = c.c_void_p
            L.oracle_pub_create.argtypes = [c.c_int, c.c_int, c.c_int, c.c_int, c.c_void_p, c.c_int, c.c_void_p,
                                            c.c_void_p, c.c_int]
            L.oracle_pub_destroy.argtypes = [c.c_void_p]
            L.oracle_pub_block_len.argtypes = [c.c_void_p]
            L.oracle_pub_block_len.restype = c.c_int
            L.oracle_pub_process.argtypes = [c.c_void_p, c.c_void_p, c.c_int]
            for f in ('oracle_pub_usb', 'oracle_pub_iq'):
                getattr(L, f).argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_size_t]
                getattr(L, f).restype = c.c_size_t
            L.oracle_pub_info.argtypes = [c.c_void_p, c.c_int, c.c_void_p]
            L.oracle_pub_low_pass.argtypes = [c.c_double, c.c_double, c.c_double, c.c_double, c.c_void_p, c.c_int]
            L.oracle_pub_hilbert.argtypes = [c.c_int, c.c_int, c.c_void_p]
            L.oracle_pub_osc.argtypes = [c.c_double, c.c_double, c.c_void_p]
            cls._ready = True
        return L

    def __init__(self, sample_rate, center_frequency, mains, vfos, mix_offset=0, correct_dc_bias=False):
        L = self.lib()
        m = np.array([[d['frequency'], d.get('out_rate', 0), d.get('compress_scale', 0), d.get('publish', 0)]
                      for d in mains], dtype=np.int32).reshape(-1, 4)
        v = np.array([[d['frequency'], d.get('data_rate', 0), d.get('out_rate', 0), d.get('filter_bandwidth', 0)]
                      for d in vfos], dtype=np.int32).reshape(-1, 4)
        g = np.array([d.get('gain', 0.0) for d in vfos], dtype=np.float32)
        self._keep = (m, v, g)
        self.h = L.oracle_pub_create(sample_rate, center_frequency, mix_offset, int(bool(correct_dc_bias)),
                                     m.ctypes.data, len(mains), v.ctypes.data, g.ctypes.data, len(vfos))
        if not self.h:
            raise ValueError('invalid publisher configuration')
        self.block_len = L.oracle_pub_block_len(self.h)
        self.nvfo, self.nmain = len(vfos), len(mains)

    def __del__(self):
        if getattr(self, 'h', None):
            Oracle.lib().oracle_pub_destroy(self.h)
            self.h = None

    def process(self, iq):
        iq = np.ascontiguousarray(iq, dtype=np.complex64)
        nb = iq.size // self.block_len
        assert nb * self.block_len == iq.size
        Oracle.lib().oracle_pub_process(self.h, iq.ctypes.data, nb)

    def usb(self, v):
        L = Oracle.lib()
        n = L.oracle_pub_usb(self.h, v, None, 0)
        out = np.zeros(n, dtype=np.int16)
        L.oracle_pub_usb(self.h, v, out.ctypes.data, n)
        return out

    def iq(self, m):
        L = Oracle.lib()
        n = L.oracle_pub_iq(self.h, m, None, 0)
        out = np.zeros(n, dtype=np.int8)
        L.oracle_pub_iq(self.h, m, out.ctypes.data, n)
        return out

    def info(self, v):
        i = np.zeros(7, dtype=np.int32)
        assert Oracle.lib().oracle_pub_info(self.h, v, i.ctypes.data) == 0
        return dict(main=int(i[0]), out_rate=int(i[1]), samples_per_block=int(i[2]), halfbands=int(i[3]),
                    late=int(i[4]), late_taps=int(i[5]), usb_taps=int(i[6]))


def wideband(sample_rate, n, seed, tones=(), noise=0.05):
    """Synthetic CF32 wideband: complex Gaussian noise plus (offset_hz,
    amplitude) tones relative to the centre frequency."""
    rng = np.random.default_rng(seed)
    x = (rng.normal(0, noise, n) + 1j * rng.normal(0, noise, n)).astype(np.complex128)
    t = np.arange(n) / float(sample_rate)
    for f, a in tones:
        x += a * np.exp(2j * np.pi * f * t)
    return x.astype(np.complex64)


# C5-like channeliser configurations (SURVEY.md §8(d) C5 stand-in): one per
# SDR rate, exercising 2^k half-bands, late 1/5 and 1/6 decimation, the audio
# low-pass, int16 wrap-around (gain 5000 %), and a main VFO with IQ output
CENTER = 1545000000
PUB_CONFIGS = {
    'r1536k': dict(sample_rate=1536000, mains=[dict(frequency=CENTER - 300000, out_rate=192000),
                                               dict(frequency=CENTER + 100000, out_rate=192000),
                                               dict(frequency=CENTER + 600000, out_rate=192000, publish=1,
                                                    compress_scale=2)],
                   vfos=[dict(frequency=CENTER - 320000, data_rate=10500, gain=100.0),
                         dict(frequency=CENTER - 265000, data_rate=600, filter_bandwidth=2500, gain=150.0),
                         dict(frequency=CENTER + 60000, data_rate=1200, gain=80.0),
                         dict(frequency=CENTER + 130000, data_rate=10500, gain=5000.0)],
                   tones=[(-318500.0, 0.3), (-264000.0, 0.2), (61200.0, 0.25), (131000.0, 0.4), (600500.0, 0.5)]),
    'r288k': dict(sample_rate=288000, mains=[dict(frequency=CENTER, out_rate=288000)],
                  vfos=[dict(frequency=CENTER + 20000, data_rate=10500, gain=100.0),
                        dict(frequency=CENTER - 50000, data_rate=600, gain=100.0, filter_bandwidth=3000),
                        dict(frequency=CENTER + 90000, data_rate=1200, gain=100.0)],
                  tones=[(21500.0, 0.3), (-49000.0, 0.2), (91000.0, 0.2)]),
    'r1920k': dict(sample_rate=1920000, mains=[dict(frequency=CENTER, out_rate=240000)],
                   vfos=[dict(frequency=CENTER - 40000, data_rate=10500, gain=100.0),
                         dict(frequency=CENTER + 30000, data_rate=600, gain=100.0),
                         dict(frequency=CENTER + 70000, data_rate=1200, gain=100.0, filter_bandwidth=4000)],
                   tones=[(-38000.0, 0.3), (31000.0, 0.2), (72000.0, 0.2)]),
}


# ------------------------------------------------------------------ C5
# SURVEY.md §8(d) C5 stand-in for the absent sdr_54W_all.ini: a 1.536 Msps
# receiver, 3 main VFOs (VFOsub[3], publish/publisher.h:50) of 192 kHz, and
# 64 [vfos]: 6 x 10500 bps on the first main, 29 x 600 / 1200 on each of the
# other two.  Each VFO carries a synthetic Aero signal of its bit rate, put
# in as the upper sideband aero-publish's USB demodulator recovers
# (publish/vfo.cpp:188-258).
C5_RATE = 1536000
C5_MAIN_OFFSETS = (-300000, 0, 300000)


def c5_config(n_mains=3, per_main=(6, 29, 29)):
    mains = [dict(frequency=CENTER + off, out_rate=192000) for off in C5_MAIN_OFFSETS[:n_mains]]
    vfos = []
    for m, n in enumerate(per_main[:n_mains]):
        base = CENTER + C5_MAIN_OFFSETS[m]
        if m == 0:  # 10500 bps: audio band [f, f + 24 kHz], 26 kHz apart
            for k in range(n):
                vfos.append(dict(frequency=base - 78000 + 26000 * k, data_rate=10500, gain=100.0))
        else:  # 600 / 1200 alternating, 5 kHz apart
            for k in range(n):
                vfos.append(dict(frequency=base - 75000 + 5000 * k, data_rate=600 if (k + m) % 2 else 1200,
                                 gain=100.0, filter_bandwidth=3000 if (k % 3 == 0) else 0))
    return dict(sample_rate=C5_RATE, center_frequency=CENTER, mains=mains, vfos=vfos)


def c5_ini(cfg):
    """SDRReceiver-style INI (the keys publish/publisher.cpp:55-227 reads) for cfg."""
    lines = ['[General]', 'sample_rate=%d' % cfg['sample_rate'], 'center_frequency=%d' % cfg['center_frequency'],
             'tuner_gain=30', 'mix_offset=0', 'zmq_address=tcp://*:6004', 'correct_dc_bias=0', '',
             '[main_vfos]', 'size=%d' % len(cfg['mains'])]
    for i, m in enumerate(cfg['mains'], 1):
        lines += ['%d\\frequency=%d' % (i, m['frequency']), '%d\\out_rate=%d' % (i, m['out_rate'])]
    lines += ['', '[vfos]', 'size=%d' % len(cfg['vfos'])]
    for i, v in enumerate(cfg['vfos'], 1):
        lines += ['%d\\frequency=%d' % (i, v['frequency']), '%d\\data_rate=%d' % (i, v['data_rate']),
                  '%d\\gain=%g' % (i, v['gain']), '%d\\topic=VFO%02d' % (i, i)]
        if v.get('filter_bandwidth'):
            lines.append('%d\\filter_bandwidth=%d' % (i, v['filter_bandwidth']))
    return '\n'.join(lines) + '\n'


def c5_audio(v, seconds, seed):
    """The audio a VFO's decoder should see: synthetic Aero PCM of its rate."""
    if v['data_rate'] == 10500:
        return synth(seconds=seconds, seed=seed, carrier=12000.0 + 37.5 + (seed % 7), ebn0=30.0), 48000
    br = v['data_rate']
    return synth_msk(seconds=seconds, bitrate=br, baud=600, seed=seed, carrier=300.0 + 2.0 * (seed % 16),
                     ebn0=30.0), (12000 if br == 600 else 24000)


def c5_wideband(cfg, seconds, seed=0xC500, noise=0.02):
    """CF32 wideband at cfg's rate: every VFO's audio as an analytic
    (upper-sideband) signal at its frequency, built per main VFO at 192 kHz
    and then raised to the receiver rate, plus a complex noise floor."""
    from scipy import signal
    fs = cfg['sample_rate']
    n = int(fs * seconds)
    rng = np.random.default_rng(seed)
    out = (rng.normal(0, noise, n) + 1j * rng.normal(0, noise, n)).astype(np.complex128)
    for m, mv in enumerate(cfg['mains']):
        mrate = mv['out_rate']
        nm = int(mrate * seconds)
        acc = np.zeros(nm, dtype=np.complex128)
        tm = np.arange(nm) / mrate
        for k, v in enumerate(cfg['vfos']):
            if abs(v['frequency'] - mv['frequency']) >= mrate // 2:
                continue
            pcm, arate = c5_audio(v, seconds, seed + 17 * k + 1)
            x = signal.hilbert(pcm.astype(np.float64) / 32768.0)
            x = signal.resample_poly(x, mrate // arate, 1)[:nm]
            acc[:len(x)] += 0.25 * x * np.exp(2j * np.pi * (v['frequency'] - mv['frequency']) * tm[:len(x)])
        up = signal.resample_poly(acc, fs // mrate, 1)[:n]
        t = np.arange(len(up)) / fs
        out[:len(up)] += up * np.exp(2j * np.pi * (mv['frequency'] - cfg['center_frequency']) * t)
    return out.astype(np.complex64)
