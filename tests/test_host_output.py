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
BIN = os.environ.get('AERO_HOST_BIN') or os.path.join(ROOT, 'aero-cli_amd', 'bin')  # asan_check.sh: sanitizer builds


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


def _publish(*args):
    exe = os.path.join(BIN, 'aero-publish')
    return subprocess.run([exe] + list(args), capture_output=True, text=True, timeout=60)


def test_publish_cli_surface(host_lib, tmp_path):
    """aero-publish's command line and settings checks (publish/main.cpp:17-49,
    publish/publisher.cpp:55-80), all before the GPU is touched."""
    r = _publish('--help')
    assert r.returncode == 0 and '--enable-dcc' in r.stdout and 'settings' in r.stdout
    r = _publish('x.ini')
    assert r.returncode == 1 and 'Required device option missing' in r.stderr
    r = _publish('-d', 'driver=file,path=/dev/null')
    assert r.returncode == 1 and 'Required settings path missing' in r.stderr
    r = _publish('-d', 'driver=file,path=/dev/null', str(tmp_path / 'missing.ini'))
    assert r.returncode == 0 and "doesn't exist or isn't a file" in r.stderr
    ini = tmp_path / 'bad_rate.ini'
    ini.write_text('[General]\nsample_rate=250000\n')
    r = _publish('-d', 'driver=file,path=/dev/null', str(ini))
    assert r.returncode == 0 and 'Provided sample rate is not supported: 250000' in r.stderr
    ini.write_text('sample_rate=abc\n')
    r = _publish('-d', 'driver=file,path=/dev/null', str(ini))
    assert r.returncode == 0 and "either doesn't exist or isn't an integer" in r.stderr
    import aero_testlib as tl
    ini.write_text(tl.c5_ini(tl.c5_config()))
    r = _publish('-d', 'driver=rtlsdr', str(ini))
    assert r.returncode == 0 and '[ERROR] failed to find device: driver=rtlsdr' in r.stderr


def test_publish_reads_the_ini_like_qsettings(host_lib, tmp_path):
    """The host's QSettings restatement (host/ini.cpp) on the generated C5
    INI: every main VFO and [vfos] entry as Publisher::loadSettings reads it
    (publish/publisher.cpp:115-222), dumped with -v before the device opens."""
    import re
    import aero_testlib as tl
    cfg = tl.c5_config()
    ini = tmp_path / 'c5.ini'
    ini.write_text(tl.c5_ini(cfg))
    r = _publish('-v', '-d', 'driver=none', str(ini))
    mains = re.findall(r'main (\d+) frequency (-?\d+) out_rate (\d+)', r.stderr)
    vfos = re.findall(r'vfo (\d+) topic (\S+) frequency (-?\d+) data_rate (\d+) out_rate (\d+) '
                      r'filter_bandwidth (\d+) gain ([0-9.e+-]+)', r.stderr)
    assert [(int(f), int(o)) for _, f, o in mains] == [(m['frequency'], m['out_rate']) for m in cfg['mains']]
    assert len(vfos) == 64
    for (i, topic, f, dr, orate, fb, g), w in zip(vfos, cfg['vfos']):
        assert topic == 'VFO%02d' % (int(i) + 1) and int(f) == w['frequency'] and int(dr) == w['data_rate']
        assert int(orate) == 0 and int(fb) == w.get('filter_bandwidth', 0) and float(g) == w['gain']
