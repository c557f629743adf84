"""Python host mirror of the C ABI in include/aero_engine.h (ctypes).

Mirrors aero-decode's per-VFO surface: a channel is opened per ZMQ topic
(decode/decode.cpp:117-241), each ZMQ message is pushed as int16 PCM
(Decoder::audioReceived -> OqpskDemodulator::dataReceived), and ACARS items
come back in emission order (AeroL::ACARSsignal).  The library is the HIP
build in this directory; there is no CPU fallback: loading fails loudly when
the native library is missing and engine creation fails without a gfx950 GPU.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libaero_engine.so')

AERO_OK = 0
AERO_E_INVALID = -1
AERO_E_NOMEM = -2
AERO_E_HIP = -3
AERO_E_NOGPU = -4
AERO_E_FULL = -5
AERO_E_RATE = -6
AERO_E_DEVICE = -7

F_TRACE_PT = 0x1
F_TRACE_BLOCKS = 0x2
F_TIMING = 0x4
F_TRACE_SOFT = 0x8
F_TRACE_HOPS = 0x10
F_TRACE_FRAMES = 0x20
F_DCD_TICK = 0x40  # AeroL's 1 s DCD timer on the sample clock (continuous OQPSK)
F_TRACE_ALL = F_TRACE_PT | F_TRACE_BLOCKS | F_TRACE_SOFT | F_TRACE_HOPS | F_TRACE_FRAMES

MATH_FN = {'hypot': 0, 'atan2': 1, 'tanh': 2, 'sin': 3, 'cos': 4, 'log10': 5, 'sqrt': 6, 'fmod360': 7,
           'div': 8, 'div_c48000': 9, 'div_c360': 10, 'div_n': 11, 'div_c192000': 13, 'hypot_nr': 14, 'atan2_bf': 15,
           'tanh_bf': 16, 'sin_bf': 17, 'cos_bf': 18,
           'div_cw_wt': 19, 'set_phase_ptr': 20}


class EngineCfg(ctypes.Structure):
    _fields_ = [('device', ctypes.c_int), ('max_channels', ctypes.c_int), ('flags', ctypes.c_int)]


class ChannelCfg(ctypes.Structure):
    _fields_ = [('bitrate', ctypes.c_int), ('burst', ctypes.c_int), ('fs', ctypes.c_uint32),
                ('disable_reassembly', ctypes.c_int)]


class AcarsItem(ctypes.Structure):
    _fields_ = [('aesid', ctypes.c_uint32),
                ('gesid', ctypes.c_uint8), ('qno', ctypes.c_uint8), ('refno', ctypes.c_uint8),
                ('seqno', ctypes.c_uint8),
                ('mode', ctypes.c_uint8), ('tak', ctypes.c_uint8), ('bi', ctypes.c_uint8),
                ('nonacars', ctypes.c_uint8),
                ('downlink', ctypes.c_uint8), ('valid', ctypes.c_uint8), ('hastext', ctypes.c_uint8),
                ('moretocome', ctypes.c_uint8),
                ('fragment', ctypes.c_uint8), ('label_len', ctypes.c_uint8), ('reg_len', ctypes.c_uint8),
                ('pad0', ctypes.c_uint8),
                ('label', ctypes.c_char * 4), ('reg', ctypes.c_char * 16),
                ('msg_len', ctypes.c_uint32), ('msg', ctypes.c_char * 3584)]


class ChanCfg(ctypes.Structure):
    _fields_ = [('device', ctypes.c_int), ('sample_rate', ctypes.c_int), ('center_frequency', ctypes.c_int),
                ('mix_offset', ctypes.c_int), ('correct_dc_bias', ctypes.c_int), ('max_blocks', ctypes.c_int),
                ('flags', ctypes.c_int)]


class ChanMain(ctypes.Structure):
    _fields_ = [('frequency', ctypes.c_int), ('out_rate', ctypes.c_int), ('compress_scale', ctypes.c_int),
                ('publish', ctypes.c_int)]


class ChanVfo(ctypes.Structure):
    _fields_ = [('frequency', ctypes.c_int), ('data_rate', ctypes.c_int), ('out_rate', ctypes.c_int),
                ('filter_bandwidth', ctypes.c_int), ('gain', ctypes.c_float), ('skip', ctypes.c_int)]


CHAN_F_HOST_OUT = 0x1


class ChannelEvents(ctypes.Structure):
    _fields_ = [('dcd_edges', ctypes.c_int64), ('hunter_steps', ctypes.c_int64), ('hunter_fc', ctypes.c_double * 8)]


# every entry point declared in include/aero_engine.h and include/aero_chan.h (tests/test_abi.py checks the header)
_SIGS = {
    'aero_engine_create': (ctypes.c_int, [ctypes.POINTER(EngineCfg), ctypes.POINTER(ctypes.c_void_p)]),
    'aero_engine_destroy': (None, [ctypes.c_void_p]),
    'aero_channel_open': (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ChannelCfg), ctypes.POINTER(ctypes.c_int)]),
    'aero_push_pcm': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_uint32]),
    'aero_push_pcm_batch': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_int, ctypes.c_int]),
    'aero_push_pcm_dev': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_uint32]),
    'aero_run': (ctypes.c_int, [ctypes.c_void_p]),
    'aero_flush': (ctypes.c_int, [ctypes.c_void_p]),
    'aero_pop_softbits': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_items': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(AcarsItem), ctypes.c_size_t,
                                      ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_items_all': (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(AcarsItem), ctypes.POINTER(ctypes.c_int),
                                          ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_hops': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_size_t)]),
    'aero_trace_select': (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    'aero_pop_pt': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_blocks': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_frames': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_rt_tests': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_c_units': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_voice': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_rt_packets': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_size_t)]),
    'aero_timing': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_long)]),
    'aero_timing_reset': (None, [ctypes.c_void_p]),
    'aero_samples_processed': (ctypes.c_uint64, [ctypes.c_void_p]),
    'aero_stat': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]),
    'aero_channel_stat': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p,
                                         ctypes.POINTER(ctypes.c_int64)]),
    'aero_channel_get_events': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ChannelEvents)]),
    'aero_sync': (ctypes.c_int, [ctypes.c_void_p]),
    'aero_device_math': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_size_t]),
    'aero_strerror': (ctypes.c_char_p, [ctypes.c_int]),
    # include/aero_chan.h
    'aero_chan_create': (ctypes.c_int, [ctypes.POINTER(ChanCfg), ctypes.POINTER(ChanMain), ctypes.c_int,
                                        ctypes.POINTER(ChanVfo), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    'aero_chan_destroy': (None, [ctypes.c_void_p]),
    'aero_chan_block_len': (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    'aero_chan_vfo_info': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    'aero_chan_main_info': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    'aero_chan_push': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]),
    'aero_chan_run': (ctypes.c_int, [ctypes.c_void_p]),
    'aero_chan_sync': (ctypes.c_int, [ctypes.c_void_p]),
    'aero_chan_vfo_output': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.POINTER(ctypes.c_size_t)]),
    'aero_chan_pop_audio': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_size_t)]),
    'aero_chan_pop_iq': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.c_size_t)]),
    'aero_chan_feed': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
}

_lib = None


def _torch_hip_runtime():
    """Paths of the HIP/HSA runtime copies a PyTorch-ROCm wheel bundles
    (torch/lib), or [] when torch is not installed.  Found without importing
    torch (no HIP initialisation happens here)."""
    import importlib.util
    spec = importlib.util.find_spec('torch')
    if spec is None or not spec.origin:
        return []
    tlib = os.path.join(os.path.dirname(spec.origin), 'lib')
    return [p for p in (os.path.join(tlib, 'libhsa-runtime64.so'), os.path.join(tlib, 'libamdhip64.so'))
            if os.path.exists(p)]


def load_library(path=None):
    """Loads libaero_engine.so (or $AERO_ENGINE_SO, an experimental build of
    the same sources); raises when the HIP build is missing.

    One HIP runtime per process: the PyTorch-ROCm wheel bundles its own
    libamdhip64 / libhsa-runtime64 (SONAME libamdhip64.so.7, the same as
    /opt/rocm's, which the engine links).  Loaded after torch, the engine
    binds to torch's copy by SONAME; loaded first, it would pull in
    /opt/rocm's copy and torch would then load a second runtime from
    torch/lib, and a device pointer allocated by one runtime is unknown to
    the other (aero_push_pcm_dev / aero_chan_push(dev) fail).  So torch's
    copy, when torch is installed, is loaded first by its absolute path:
    torch's later load of the same file reuses it (same inode) and the engine
    binds to it by SONAME, in either import order.  Without torch (the C++
    host) the engine uses /opt/rocm's runtime."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get('AERO_ENGINE_SO') or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError('libaero_engine.so not built (%s); run aero-cli_amd/build.py' % path)
    for rt in _torch_hip_runtime():
        ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if path == LIB_PATH:
                raise
            continue  # an older experimental build (A/B) without a newer entry point
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class AeroError(RuntimeError):
    def __init__(self, rc, what):
        lib = load_library()
        super().__init__('%s failed: %s (%d)' % (what, lib.aero_strerror(rc).decode(), rc))
        self.rc = rc


def _check(rc, what):
    if rc != AERO_OK:
        raise AeroError(rc, what)


def item_line(it):
    """Canonical text of one ACARSItem, identical to the oracle's emit_item."""
    def hx(b):
        return b.hex()
    kind = 'F' if it.fragment else 'A'
    head = ('%s aes=%06X ges=%02X qno=%02X refno=%02X mode=%02X tak=%02X bi=%02X '
            'nonacars=%d downlink=%d valid=%d hastext=%d more=%d' % (
                kind, it.aesid, it.gesid, it.qno, it.refno, it.mode, it.tak, it.bi, it.nonacars,
                it.downlink, it.valid, it.hastext, it.moretocome))
    label = bytes(it.label)[:it.label_len]
    reg = bytes(it.reg)[:it.reg_len]
    msg = ctypes.string_at(ctypes.addressof(it) + AcarsItem.msg.offset, it.msg_len)
    return head + ' label=' + hx(label) + ' reg=' + hx(reg) + ' msg=' + hx(msg)


class Engine:
    """Batched MI355X Aero demodulator (one engine per GPU)."""

    def __init__(self, max_channels, device=0, flags=0):
        self.lib = load_library()
        cfg = EngineCfg(device, max_channels, flags)
        h = ctypes.c_void_p()
        _check(self.lib.aero_engine_create(ctypes.byref(cfg), ctypes.byref(h)), 'aero_engine_create')
        self.h = h
        self.flags = flags
        self._fs = {}

    def close(self):
        if self.h:
            self.lib.aero_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # sample rate aero-decode feeds each bit rate (decode/decode.cpp:142-159)
    RATE = {10500: 48000, 600: 12000, 1200: 24000, 8400: 48000}

    def open_channel(self, bitrate=10500, fs=None, disable_reassembly=False, burst=False):
        fs = fs or self.RATE.get(bitrate, 48000)
        cfg = ChannelCfg(bitrate, int(burst), fs, int(disable_reassembly))
        ch = ctypes.c_int()
        _check(self.lib.aero_channel_open(self.h, ctypes.byref(cfg), ctypes.byref(ch)), 'aero_channel_open')
        self._fs[ch.value] = fs
        return ch.value

    def push(self, ch, pcm, fs=None):
        pcm = np.ascontiguousarray(pcm, dtype=np.int16)
        fs = fs or self._fs.get(ch, 48000)
        _check(self.lib.aero_push_pcm(self.h, ch, pcm.ctypes.data, pcm.size, fs), 'aero_push_pcm')

    def push_batch(self, pcm, nch=None):
        """pcm: int16 [n, ld] host array (time-major) for channels 0..nch-1."""
        pcm = np.ascontiguousarray(pcm, dtype=np.int16)
        n, ld = pcm.shape
        _check(self.lib.aero_push_pcm_batch(self.h, pcm.ctypes.data, n, ld, nch or ld, 0), 'aero_push_pcm_batch')

    def push_device(self, ch, ptr, n, fs=None):
        """ptr: HIP device pointer of n int16 samples for channel ch."""
        fs = fs or self._fs.get(ch, 48000)
        _check(self.lib.aero_push_pcm_dev(self.h, ch, ctypes.c_void_p(ptr), n, fs), 'aero_push_pcm_dev')

    def push_batch_host(self, ptr, n, ld, nch):
        """ptr: host pointer of int16 [n, ld]; pinned memory (e.g. a torch
        pin_memory() tensor) is DMA'd straight into HBM."""
        _check(self.lib.aero_push_pcm_batch(self.h, ctypes.c_void_p(ptr), n, ld, nch, 0), 'aero_push_pcm_batch')

    def push_batch_device(self, ptr, n, ld, nch):
        """ptr: HIP device pointer of int16 [n, ld] (e.g. torch tensor.data_ptr())."""
        _check(self.lib.aero_push_pcm_batch(self.h, ctypes.c_void_p(ptr), n, ld, nch, 1), 'aero_push_pcm_batch')

    def trace_select(self, channels):
        """Keeps traces (soft bits, hops, pt, blocks, frames) of these
        continuous channels only; [] keeps every channel's again."""
        arr = (ctypes.c_int * max(1, len(channels)))(*[int(c) for c in channels])
        _check(self.lib.aero_trace_select(self.h, arr, len(channels)), 'aero_trace_select')

    def run(self):
        _check(self.lib.aero_run(self.h), 'aero_run')

    def flush(self):
        _check(self.lib.aero_flush(self.h), 'aero_flush')

    def sync(self):
        _check(self.lib.aero_sync(self.h), 'aero_sync')

    def _pop(self, fn, ch, dtype, rec=1):
        out = []
        cap = 1 << 20
        while True:
            buf = np.empty(cap * rec, dtype=dtype)
            n = ctypes.c_size_t()
            _check(fn(self.h, ch, buf.ctypes.data, cap, ctypes.byref(n)), fn.__name__)
            out.append(buf[:n.value * rec].copy())
            if n.value < cap:
                break
        r = np.concatenate(out)
        return r.reshape(-1, rec) if rec > 1 else r

    def softbits(self, ch):
        return self._pop(self.lib.aero_pop_softbits, ch, np.int16).astype(np.uint8)

    def softbits16(self, ch):
        """burst channels: delivered soft bits with -1 start-of-packet markers"""
        return self._pop(self.lib.aero_pop_softbits, ch, np.int16)

    def rt_tests(self, ch):
        """burst channels: (blockptr, result code) of every R/T test"""
        return self._pop(self.lib.aero_pop_rt_tests, ch, np.uint8).view(np.uint32).reshape(-1, 2)

    def rt_packets(self, ch):
        """burst channels: [(kind 'R'/'T', infofield bytes)] of every decoded R/T packet"""
        raw = self._pop(self.lib.aero_pop_rt_packets, ch, np.uint8)
        out, i = [], 0
        while i < len(raw):
            kind, ln = np.frombuffer(raw[i:i + 8].tobytes(), np.uint32)
            out.append((chr(kind), bytes(raw[i + 8:i + 8 + int(ln)])))
            i += 8 + int(ln)
        return out

    def c_units(self, ch):
        """C channel: every CRC-valid Call_progress SU, [n, 12] bytes"""
        return self._pop(self.lib.aero_pop_c_units, ch, np.uint8, 12)

    def voice(self, ch):
        """C channel: per frame (AES of its last Call_progress, 300 voice bytes)"""
        raw = self._pop(self.lib.aero_pop_voice, ch, np.uint8, 304)
        return [(int(np.frombuffer(r[:4].tobytes(), np.uint32)[0]), bytes(r[4:])) for r in raw]

    def hops(self, ch):
        return self._pop(self.lib.aero_pop_hops, ch, np.float64, 6)

    def pt(self, ch):
        return self._pop(self.lib.aero_pop_pt, ch, np.float64, 2)

    def blocks(self, ch):
        return self._pop(self.lib.aero_pop_blocks, ch, np.uint8)

    def frames(self, ch):
        return self._pop(self.lib.aero_pop_frames, ch, np.uint8)

    def items(self, ch):
        out = []
        arr = (AcarsItem * 64)()
        while True:
            n = ctypes.c_size_t()
            _check(self.lib.aero_pop_items(self.h, ch, arr, 64, ctypes.byref(n)), 'aero_pop_items')
            out.extend(item_line(arr[i]) for i in range(n.value))
            if n.value < 64:
                return out

    def drain_items(self, lines=False, cap=4096, keep=None):
        """Pops the items of every channel (aero_pop_items_all).  Returns the
        count, or (channel, canonical line) pairs with lines=True (only the
        channels in the set `keep`, when given)."""
        if getattr(self, '_drain_cap', 0) != cap:
            self._drain_buf = ((AcarsItem * cap)(), (ctypes.c_int * cap)())
            self._drain_cap = cap
        arr, chs = self._drain_buf
        total, out = 0, []
        while True:
            n = ctypes.c_size_t()
            _check(self.lib.aero_pop_items_all(self.h, arr, chs, cap, ctypes.byref(n)), 'aero_pop_items_all')
            total += n.value
            if lines:
                out.extend((chs[i], item_line(arr[i])) for i in range(n.value) if keep is None or chs[i] in keep)
            if n.value < cap:
                return out if lines else total

    def timing(self, name):
        ms = ctypes.c_double()
        k = ctypes.c_long()
        _check(self.lib.aero_timing(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(k)), 'aero_timing')
        return ms.value, k.value

    def timing_reset(self):
        self.lib.aero_timing_reset(self.h)

    def stat(self, name):
        """aero_stat counter: 'viterbi_jobs', 'frames', 'su_crc_ok' (and burst 'rt_*'), or the
        continuous groups' 'device_bytes' / 'groups'."""
        v = ctypes.c_uint64()
        _check(self.lib.aero_stat(self.h, name.encode(), ctypes.byref(v)), 'aero_stat')
        return int(v.value)

    def channel_stat(self, ch, name):
        """aero_channel_stat: 'hunter_scans' or 'freq_center'."""
        v = ctypes.c_int64()
        _check(self.lib.aero_channel_stat(self.h, ch, name.encode(), ctypes.byref(v)), 'aero_channel_stat')
        return int(v.value)

    def channel_events(self, ch):
        """aero_channel_get_events: (dcd_edges, hunter_steps, [centre of each
        of the last min(8, steps) steps, oldest first])."""
        ev = ChannelEvents()
        _check(self.lib.aero_channel_get_events(self.h, ch, ctypes.byref(ev)), 'aero_channel_get_events')
        n = int(ev.hunter_steps)
        fcs = [ev.hunter_fc[(k - 1) & 7] for k in range(max(1, n - 7), n + 1)]
        return int(ev.dcd_edges), n, fcs

    def samples_processed(self):
        return int(self.lib.aero_samples_processed(self.h))

    def device_math(self, fn, x, y=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros_like(x) if y is None else np.ascontiguousarray(y, dtype=np.float64)
        out = np.empty_like(x)
        _check(self.lib.aero_device_math(self.h, MATH_FN[fn], x.ctypes.data, y.ctypes.data, out.ctypes.data,
                                         x.size), 'aero_device_math')
        return out


# ------------------------------------------------------------------ channeliser
def vfo_out_rate(data_rate, out_rate=0):
    """[vfos] out_rate default by data_rate (publish/publisher.cpp:164-176)."""
    if out_rate or not data_rate:
        return out_rate
    return {600: 12000, 1200: 24000}.get(int(data_rate), 48000)


def vfo_bitrate(data_rate):
    """aero-decode bit rate of a [vfos] entry's audio (10500 unless 600/1200)."""
    return int(data_rate) if int(data_rate) in (600, 1200) else 10500


def parse_sdr_ini(text):
    """SDRReceiver INI as QSettings reads it for aero-publish
    (publish/publisher.cpp:55-227): returns (general, mains, vfos) dicts with
    the keys the publisher uses; arrays are QSettings' [name] size=N,
    i\\key=value entries."""
    sections, cur = {}, 'General'
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line[0] in ';#':
            continue
        if line.startswith('[') and line.endswith(']'):
            cur = line[1:-1]
            continue
        if '=' in line:
            k, v = line.split('=', 1)
            sections.setdefault(cur, {})[k.strip()] = v.strip()

    def to_int(v):  # QVariant::toInt: 0 when the text is not an integer
        try:
            return int(v)
        except (TypeError, ValueError):
            return 0

    def to_float(v):
        try:
            return float(v)
        except (TypeError, ValueError):
            return 0.0

    def array(name):
        sec = sections.get(name, {})
        out = []
        for i in range(1, to_int(sec.get('size')) + 1):
            pre = '%d\\' % i
            out.append({k[len(pre):]: v for k, v in sec.items() if k.startswith(pre)})
        return out

    g = sections.get('General', {})
    general = dict(sample_rate=to_int(g.get('sample_rate')), center_frequency=to_int(g.get('center_frequency')),
                   mix_offset=to_int(g.get('mix_offset')), correct_dc_bias=g.get('correct_dc_bias') == '1',
                   zmq_address=g.get('zmq_address', ''))
    mains = [dict(frequency=to_int(d.get('frequency')), out_rate=to_int(d.get('out_rate')),
                  compress_scale=to_int(d.get('compress_scale')),
                  publish=int(bool(d.get('zmq_address')) and bool(d.get('zmq_topic'))))
             for d in array('main_vfos')]
    vfos = [dict(frequency=to_int(d.get('frequency')), data_rate=to_int(d.get('data_rate')),
                 out_rate=to_int(d.get('out_rate')), filter_bandwidth=to_int(d.get('filter_bandwidth')),
                 gain=to_float(d.get('gain')), topic=d.get('topic', ''))
            for d in array('vfos')]
    return general, mains, vfos


class Channeliser:
    """aero-publish's channeliser on one GPU (include/aero_chan.h):
    Publisher::loadSettings + demodData (publish/publisher.cpp:55-306) and
    vfo::process (publish/vfo.cpp:154-313).  `mains` / `vfos` are the INI's
    [main_vfos] / [vfos] entries (dicts as parse_sdr_ini returns); `skip`
    marks [vfos] entries another process computes."""

    def __init__(self, sample_rate, center_frequency, mains, vfos, mix_offset=0, correct_dc_bias=False,
                 max_blocks=8, device=0, host_out=False, skip=None):
        self.lib = load_library()
        cfg = ChanCfg(device, int(sample_rate), int(center_frequency), int(mix_offset), int(bool(correct_dc_bias)),
                      int(max_blocks), CHAN_F_HOST_OUT if host_out else 0)
        m = (ChanMain * max(1, len(mains)))()
        for i, d in enumerate(mains):
            m[i] = ChanMain(int(d['frequency']), int(d.get('out_rate', 0)), int(d.get('compress_scale', 0)),
                            int(d.get('publish', 0)))
        v = (ChanVfo * max(1, len(vfos)))()
        for i, d in enumerate(vfos):
            v[i] = ChanVfo(int(d['frequency']), int(d.get('data_rate', 0)), int(d.get('out_rate', 0)),
                           int(d.get('filter_bandwidth', 0)), float(d.get('gain', 0.0)),
                           int(bool(skip[i])) if skip is not None else 0)
        h = ctypes.c_void_p()
        _check(self.lib.aero_chan_create(ctypes.byref(cfg), m, len(mains), v, len(vfos), ctypes.byref(h)),
               'aero_chan_create')
        self.h = h
        self.nmain, self.nvfo = len(mains), len(vfos)
        b = ctypes.c_int()
        _check(self.lib.aero_chan_block_len(h, ctypes.byref(b)), 'aero_chan_block_len')
        self.block_len = b.value

    def close(self):
        if self.h:
            self.lib.aero_chan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def vfo_info(self, v):
        i = (ctypes.c_int * 5)()
        _check(self.lib.aero_chan_vfo_info(self.h, v, i), 'aero_chan_vfo_info')
        return dict(main=i[0], out_rate=i[1], samples_per_block=i[2], halfbands=i[3], late=i[4])

    def main_info(self, m):
        i = (ctypes.c_int * 3)()
        _check(self.lib.aero_chan_main_info(self.h, m, i), 'aero_chan_main_info')
        return dict(out_rate=i[0], samples_per_block=i[1], halfbands=i[2])

    def push(self, iq):
        """iq: complex64 host samples, whole reads of block_len."""
        iq = np.ascontiguousarray(iq, dtype=np.complex64)
        nb = iq.size // self.block_len
        if nb * self.block_len != iq.size:
            raise ValueError('push whole reads of %d samples' % self.block_len)
        _check(self.lib.aero_chan_push(self.h, iq.ctypes.data, nb, 0), 'aero_chan_push')

    def push_device(self, ptr, nblocks):
        """ptr: HIP device pointer of nblocks * block_len interleaved CF32 samples."""
        _check(self.lib.aero_chan_push(self.h, ctypes.c_void_p(ptr), nblocks, 1), 'aero_chan_push')

    def run(self):
        _check(self.lib.aero_chan_run(self.h), 'aero_chan_run')

    def sync(self):
        _check(self.lib.aero_chan_sync(self.h), 'aero_chan_sync')

    def output_device(self, v):
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        _check(self.lib.aero_chan_vfo_output(self.h, v, ctypes.byref(p), ctypes.byref(n)), 'aero_chan_vfo_output')
        return p.value, n.value

    def _pop(self, fn, i, dtype):
        out, cap = [], 1 << 20
        while True:
            buf = np.empty(cap, dtype=dtype)
            n = ctypes.c_size_t()
            _check(fn(self.h, i, buf.ctypes.data, cap, ctypes.byref(n)), fn.__name__)
            out.append(buf[:n.value].copy())
            if n.value < cap:
                return np.concatenate(out)

    def audio(self, v):
        return self._pop(self.lib.aero_chan_pop_audio, v, np.int16)

    def iq(self, m):
        return self._pop(self.lib.aero_chan_pop_iq, m, np.int8)

    def feed(self, engine, channels):
        """channels[v]: engine channel of [vfos] entry v, or -1."""
        arr = (ctypes.c_int * max(1, self.nvfo))(*[int(c) for c in channels])
        _check(self.lib.aero_chan_feed(self.h, engine.h, arr), 'aero_chan_feed')
