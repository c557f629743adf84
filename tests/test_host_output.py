"""aero-decode's console / forwarder formats (decode/output.cpp:12-171) as
the drop-in host produces them (aero-cli_amd/host/output.cpp, through
libaero_host.so), against tests/golden/output_golden.json, which Qt itself
(QString::arg / mid / replace, QJsonDocument compact writer; conda Qt 5.9.7)
produced from the same items (tests/golden/make_output_golden.sh).  Also the
host's command-line surface (decode/main.cpp:17-92) where it ends before the
engine starts (no GPU needed)."""
import ctypes
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, 'tests', 'golden')
BIN = os.path.join(ROOT, 'aero-cli_amd', 'bin')


@pytest.fixture(scope='module')
def host_lib(engine_lib):
    import build
    build.build_host()
    L = ctypes.CDLL(os.path.join(BIN, 'libaero_host.so'))
    for f in (L.aero_host_format, L.aero_host_format_latin1):
        f.restype = ctypes.c_long
        f.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
                      ctypes.c_char_p, ctypes.c_size_t]
    return L


def to_item(d):
    import aero_engine as ae
    it = ae.AcarsItem()
    it.aesid, it.gesid, it.qno, it.refno = d['aesid'], d['gesid'], d['qno'], d['refno']
    it.mode, it.tak, it.bi = d['mode'], d['tak'], d['bi']
    it.nonacars, it.downlink, it.moretocome = d['nonacars'], d['downlink'], d['moretocome']
    lab, reg, msg = (bytes.fromhex(d[k]) for k in ('label', 'reg', 'msg'))
    it.label_len, it.reg_len, it.msg_len = len(lab), len(reg), len(msg)
    it.label, it.reg = lab, reg
    ctypes.memmove(ctypes.addressof(it) + ae.AcarsItem.msg.offset, msg, len(msg))
    return it


def fmt(L, f, station, dr, it, ms):
    buf = ctypes.create_string_buffer(65536)
    n = L.aero_host_format(f, station.encode(), dr, ctypes.byref(it), ms, buf, len(buf))
    assert n >= 0
    return buf.raw[:n].decode('utf-8')


def test_formats_match_qt_fixture(host_lib):
    items = json.load(open(os.path.join(GOLD, 'output_items.json')))
    gold = json.load(open(os.path.join(GOLD, 'output_golden.json')))['cases']
    assert len(gold) == len(items['items'])
    for d, g in zip(items['items'], gold):
        it = to_item(d)
        ms, st = items['time_ms'], items['station']
        assert fmt(host_lib, 1, st, 0, it, ms) == g['text'], d
        assert fmt(host_lib, 1, st, 1, it, ms) == g['text_fragments'], d
        assert fmt(host_lib, 2, st, 0, it, ms) == g['jaero'], d
        assert fmt(host_lib, 3, st, 0, it, ms) == g['jsondump'], d


def test_forwarded_bytes_are_latin1(host_lib):
    items = json.load(open(os.path.join(GOLD, 'output_items.json')))
    gold = json.load(open(os.path.join(GOLD, 'output_golden.json')))['cases']
    for d, g in zip(items['items'], gold):
        it = to_item(d)
        buf = ctypes.create_string_buffer(65536)
        n = host_lib.aero_host_format_latin1(1, items['station'].encode(), 0, ctypes.byref(it), items['time_ms'],
                                             buf, len(buf))
        assert buf.raw[:n] == g['text'].encode('latin-1', 'replace')


def _decode(*args, env=None):
    exe = os.path.join(BIN, 'aero-decode')
    return subprocess.run([exe] + list(args), capture_output=True, text=True, timeout=60,
                          env=dict(os.environ, **(env or {})))


def test_cli_surface(host_lib):
    r = _decode('--help')
    assert r.returncode == 0 and '--bit-rate' in r.stdout and '--no-signal-exit' in r.stdout
    r = _decode('-t', 'VFO01')
    assert r.returncode == 1 and 'Required publisher option is missing' in r.stderr
    r = _decode('-p', 'tcp://127.0.0.1:1')
    assert r.returncode == 1 and 'Required topic option is missing' in r.stderr
    r = _decode('--bogus')
    assert r.returncode == 1 and "Unknown option 'bogus'" in r.stderr
    r = _decode('-p', 'tcp://127.0.0.1:1', '-t', 'VFO01', '-b')
    assert r.returncode == 1 and 'Missing value' in r.stderr
    # Decoder ctor refusals complete with status 0 (decode/decode.cpp:87-104)
    r = _decode('-p', 'tcp://127.0.0.1:1', '-t', 'VFO01', '-b', '8400', '-s', 'X')
    assert r.returncode == 0 and 'Unsupported bit rate: 8400' in r.stderr
    r = _decode('-p', 'tcp://127.0.0.1:1', '-t', 'VFO01', '--bit-rate=600', '--format', 'xml', '-s', 'X')
    assert r.returncode == 0 and 'Invalid output format provided: xml' in r.stderr
    for bad in ('text', 'json=tcp://h:1', 'text=', 'text=http://h:1', 'text=tcp://h', 'text=tcp://:5'):
        r = _decode('-p', 'tcp://127.0.0.1:1', '-t', 'VFO01', '-b10500', '-f', bad, '-s', 'X')
        assert r.returncode == 0 and 'Some forwarders configuration may be malformed' in r.stderr, bad
    r = _decode('-p', 'tcp://127.0.0.1:1', '-t', 'VFO01', '-b', '600', '-v')
    assert 'No station ID provided, using generated default' in r.stderr and '-AERO-INMARSAT' in r.stderr
