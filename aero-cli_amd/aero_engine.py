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

F_TRACE_PT = 0x1
F_TRACE_BLOCKS = 0x2
F_TIMING = 0x4
F_TRACE_SOFT = 0x8
F_TRACE_HOPS = 0x10
F_TRACE_FRAMES = 0x20
F_TRACE_ALL = F_TRACE_PT | F_TRACE_BLOCKS | F_TRACE_SOFT | F_TRACE_HOPS | F_TRACE_FRAMES

MATH_FN = {'hypot': 0, 'atan2': 1, 'tanh': 2, 'sin': 3, 'cos': 4, 'log10': 5, 'sqrt': 6, 'fmod360': 7,
           'div': 8}


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


# every entry point declared in include/aero_engine.h (tests/test_abi.py checks the header)
_SIGS = {
    'aero_engine_create': (ctypes.c_int, [ctypes.POINTER(EngineCfg), ctypes.POINTER(ctypes.c_void_p)]),
    'aero_engine_destroy': (None, [ctypes.c_void_p]),
    'aero_channel_open': (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ChannelCfg), ctypes.POINTER(ctypes.c_int)]),
    'aero_push_pcm': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_uint32]),
    'aero_push_pcm_batch': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_int, ctypes.c_int]),
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
    'aero_pop_pt': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_blocks': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_size_t)]),
    'aero_pop_frames': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_size_t)]),
    'aero_timing': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_long)]),
    'aero_timing_reset': (None, [ctypes.c_void_p]),
    'aero_samples_processed': (ctypes.c_uint64, [ctypes.c_void_p]),
    'aero_sync': (ctypes.c_int, [ctypes.c_void_p]),
    'aero_device_math': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_size_t]),
    'aero_strerror': (ctypes.c_char_p, [ctypes.c_int]),
}

_lib = None


def load_library(path=None):
    """Loads libaero_engine.so (or $AERO_ENGINE_SO, an experimental build of
    the same sources); raises when the HIP build is missing."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get('AERO_ENGINE_SO') or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError('libaero_engine.so not built (%s); run aero-cli_amd/build.py' % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
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
    RATE = {10500: 48000, 600: 12000, 1200: 24000}

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

    def push_batch_device(self, ptr, n, ld, nch):
        """ptr: HIP device pointer of int16 [n, ld] (e.g. torch tensor.data_ptr())."""
        _check(self.lib.aero_push_pcm_batch(self.h, ctypes.c_void_p(ptr), n, ld, nch, 1), 'aero_push_pcm_batch')

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

    def drain_items(self, lines=False, cap=4096):
        """Pops the items of every channel (aero_pop_items_all).  Returns the
        count, or (channel, canonical line) pairs with lines=True."""
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
                out.extend((chs[i], item_line(arr[i])) for i in range(n.value))
            if n.value < cap:
                return out if lines else total

    def timing(self, name):
        ms = ctypes.c_double()
        k = ctypes.c_long()
        _check(self.lib.aero_timing(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(k)), 'aero_timing')
        return ms.value, k.value

    def timing_reset(self):
        self.lib.aero_timing_reset(self.h)

    def samples_processed(self):
        return int(self.lib.aero_samples_processed(self.h))

    def device_math(self, fn, x, y=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros_like(x) if y is None else np.ascontiguousarray(y, dtype=np.float64)
        out = np.empty_like(x)
        _check(self.lib.aero_device_math(self.h, MATH_FN[fn], x.ctypes.data, y.ctypes.data, out.ctypes.data,
                                         x.size), 'aero_device_math')
        return out
