"""The drop-in aero-decode host (aero-cli_amd/bin/aero-decode) end to end on
the GPU: synthetic P-channel PCM published over ZeroMQ in aero-publish's wire
format (tools/zmq_pcm_pub, [topic][u32 rate][int16 PCM] in 12000-sample
messages) -> ZMQ SUB -> engine -> console lines in --format jsondump, a TCP
forwarder in text and a UDP forwarder in jaero.  Every line must equal the
oracle's ACARS items for the same PCM, formatted by the Qt-pinned formatter
(tests/test_host_output.py), at a pinned wall clock."""
import ctypes
import os
import re
import signal
import socket
import subprocess
import threading
import time

import numpy as np
import pytest

import aero_testlib as tl

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, 'aero-cli_amd', 'bin')
PUB = os.path.join(ROOT, 'tools', 'zmq_pcm_pub')
FIXED_MS = 1714558496789
STATION = 'GPU-TEST'


def free_port(kind=socket.SOCK_STREAM):
    with socket.socket(socket.AF_INET, kind) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def parse_line(line):
    """oracle / engine canonical item line -> aero_acars_item"""
    import aero_engine as ae
    f = dict(kv.split('=', 1) for kv in line.split()[1:])
    it = ae.AcarsItem()
    it.aesid, it.gesid = int(f['aes'], 16), int(f['ges'], 16)
    it.qno, it.refno, it.mode = int(f['qno'], 16), int(f['refno'], 16), int(f['mode'], 16)
    it.tak, it.bi = int(f['tak'], 16), int(f['bi'], 16)
    it.nonacars, it.downlink, it.valid = int(f['nonacars']), int(f['downlink']), int(f['valid'])
    it.hastext, it.moretocome = int(f['hastext']), int(f['more'])
    it.fragment = 1 if line.startswith('F') else 0
    lab, reg, msg = bytes.fromhex(f['label']), bytes.fromhex(f['reg']), bytes.fromhex(f['msg'])
    it.label_len, it.reg_len, it.msg_len = len(lab), len(reg), len(msg)
    it.label, it.reg = lab, reg
    ctypes.memmove(ctypes.addressof(it) + ae.AcarsItem.msg.offset, msg, len(msg))
    return it


def expected(lines, fmt_id, station=STATION):
    L = ctypes.CDLL(os.path.join(BIN, 'libaero_host.so'))
    L.aero_host_format.restype = ctypes.c_long
    L.aero_host_format.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong,
                                   ctypes.c_char_p, ctypes.c_size_t]
    out = []
    for ln in lines:
        it = parse_line(ln)
        buf = ctypes.create_string_buffer(65536)
        n = L.aero_host_format(fmt_id, station.encode(), 0, ctypes.byref(it), FIXED_MS, buf, len(buf))
        out.append(buf.raw[:n].decode())
    return out


class TcpSink(threading.Thread):
    def __init__(self):
        super().__init__(daemon=True)
        self.srv = socket.socket()
        self.srv.bind(('127.0.0.1', 0))
        self.srv.listen(4)
        self.port = self.srv.getsockname()[1]
        self.data = b''

    def run(self):
        self.srv.settimeout(120)
        try:
            conn, _ = self.srv.accept()
        except OSError:
            return
        conn.settimeout(120)
        while True:
            try:
                b = conn.recv(65536)
            except OSError:
                break
            if not b:
                break
            self.data += b


class UdpSink(threading.Thread):
    def __init__(self):
        super().__init__(daemon=True)
        self.s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.s.bind(('127.0.0.1', 0))
        self.port = self.s.getsockname()[1]
        self.msgs = []

    def run(self):
        self.s.settimeout(1.0)
        self.stop = False
        while not self.stop:
            try:
                self.msgs.append(self.s.recv(65536))
            except OSError:
                continue


def _start_decoder(args, env):
    p = subprocess.Popen([os.path.join(BIN, 'aero-decode')] + args, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         env=dict(os.environ, AERO_DECODE_FIXED_TIME_MS=str(FIXED_MS), **env))
    lines = []

    def pump():
        for raw in p.stderr:
            lines.append(raw.decode('utf-8', 'replace').rstrip('\n'))
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    t0 = time.time()
    while not any('Listening for samples' in l for l in lines):
        assert p.poll() is None, '\n'.join(lines)
        assert time.time() - t0 < 120, 'decoder did not start'
        time.sleep(0.1)
    return p, lines, th


def test_zmq_to_acars_json_end_to_end(engine_lib, cpu_libs, tmp_path):
    import build
    build.build_host()
    pcm = tl.synth(seconds=20.0, seed=0xAE70, carrier=12041.0, ebn0=12.0)
    ref = tl.Oracle(dcd_tick=True)  # aero-decode runs the DCD timer (AERO_F_DCD_TICK)
    ref.push_chunked(pcm, 12000)
    want = ref.item_lines('A')
    assert len(want) >= 5
    f = tmp_path / 'vfo.pcm'
    pcm.astype('<i2').tofile(str(f))
    port = free_port()
    tcp, udp = TcpSink(), UdpSink()
    tcp.start()
    udp.start()
    dec, lines, th = _start_decoder(
        ['-p', 'tcp://127.0.0.1:%d' % port, '-t', 'VFO01', '-b', '10500', '--format', 'jsondump', '-s', STATION,
         '-v', '-f', 'text=tcp://127.0.0.1:%d,jaero=udp://127.0.0.1:%d' % (tcp.port, udp.port)], {})
    try:
        r = subprocess.run([PUB, '--bind', 'tcp://127.0.0.1:%d' % port, '--topic', 'VFO01', '--rate', '48000',
                            '--chunk', '12000', '--wait-ms', '1500', str(f)], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        # every message queued in the SUB socket is taken before SIGTERM (the
        # reference stops reading on a signal too); the tail hop is flushed
        t0 = time.time()
        while sum(l.startswith('{') for l in lines) < len(want) - 4 and time.time() - t0 < 90:
            time.sleep(0.2)
        time.sleep(1.0)
    finally:
        dec.send_signal(signal.SIGTERM)
        rc = dec.wait(timeout=120)
    th.join(timeout=10)
    tcp.join(timeout=10)
    udp.stop = True
    udp.join(timeout=5)
    assert rc == 0, '\n'.join(lines[-20:])
    console = [l for l in lines if l.startswith('{')]
    assert console == expected(want, 3)
    # -v: Decoder::handleDcdChange once the first frame synchronises (decode/decode.cpp:429-435)
    assert sum('Data carrier detected: no signal => signal' in l for l in lines) == 1
    assert tcp.data.decode('latin-1').splitlines() == [s for s in expected(want, 1)]
    assert [m.decode('latin-1').rstrip('\n') for m in udp.msgs] == expected(want, 2)


def test_no_signal_exit(engine_lib, tmp_path):
    """--no-signal-exit: a full hunter scan without a signal ends the decoder
    (decode/decode.cpp:418-427; 4 x 15 hops of 4096 samples at 10500 bps)."""
    import build
    build.build_host()
    rng = np.random.default_rng(5)
    noise = (rng.normal(0, 300, 48000 * 8)).astype('<i2')
    f = tmp_path / 'noise.pcm'
    noise.tofile(str(f))
    port = free_port()
    dec, lines, th = _start_decoder(['-p', 'tcp://127.0.0.1:%d' % port, '-t', 'VFO07', '-b', '10500', '-s', 'X',
                                     '--no-signal-exit', '-v'], {})
    try:
        subprocess.run([PUB, '--bind', 'tcp://127.0.0.1:%d' % port, '--topic', 'VFO07', '--rate', '48000',
                        '--chunk', '4800', '--pace-ms', '30', '--wait-ms', '1500', str(f)], capture_output=True,
                       timeout=120)
        rc = dec.wait(timeout=60)
    finally:
        if dec.poll() is None:
            dec.kill()
    th.join(timeout=10)
    text = '\n'.join(lines)
    # -v: Decoder::handleNewFreqCenter, SignalHunter's unclamped centres (decode/hunter.cpp:31-40)
    steps = re.findall(r'Trying frequency center ([0-9.]+) in search of signal', text)
    assert steps[:4] == ['5250.0', '10500.0', '15750.0', '0.0'], steps
    assert 'Scanned entire VFO bandwidth and could not find a signal.' in text
    assert 'Exiting because of no signal' in text
    assert rc == 0


def test_publish_to_decode_pipeline(engine_lib, cpu_libs, tmp_path):
    """aero-publish (GPU channeliser, CF32 file source, the generated C5 INI,
    64 VFOs) -> ZeroMQ -> two aero-decode processes (a 10500 and a 600 bps
    topic) -> jsondump lines equal to the oracle publisher's audio through
    the oracle decoder (publish/vfo.cpp -> decode/decode.cpp, config C5)."""
    import build
    build.build_host()
    cfg = tl.c5_config()
    x = tl.c5_wideband(cfg, 8.0)
    ref = tl.OraclePublisher(cfg['sample_rate'], cfg['center_frequency'], cfg['mains'], cfg['vfos'])
    nb = len(x) // ref.block_len
    ref.process(x[:nb * ref.block_len])
    wb = tmp_path / 'wideband.cf32'
    x[:nb * ref.block_len].astype(np.complex64).tofile(str(wb))
    port = free_port()
    ini = tmp_path / 'c5.ini'
    ini.write_text(tl.c5_ini(cfg).replace('tcp://*:6004', 'tcp://127.0.0.1:%d' % port))
    picks = [0, 7]  # VFO01 (10500 bps), VFO08 (600 bps)
    wants = []
    for v in picks:
        import aero_engine as ae
        o = tl.Oracle(bitrate=ae.vfo_bitrate(cfg["vfos"][v]["data_rate"]), dcd_tick=True)
        o.push_chunked(ref.usb(v), ref.info(v)['samples_per_block'])
        wants.append(o.item_lines('A'))
    assert len(wants[0]) >= 5
    decs = []
    for v in picks:
        br = str(cfg['vfos'][v]['data_rate'])
        decs.append(_start_decoder(['-p', 'tcp://127.0.0.1:%d' % port, '-t', 'VFO%02d' % (v + 1), '-b', br,
                                    '--format', 'jsondump', '-s', STATION, '-v'], {}))
    try:
        r = subprocess.run([os.path.join(BIN, 'aero-publish'), '-d',
                            'driver=file,path=%s,start_delay_ms=1500' % wb, str(ini)],
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-3000:]
        t0 = time.time()
        while any(sum(l.startswith('{') for l in d[1]) < len(w) - 4 for d, w in zip(decs, wants)) \
                and time.time() - t0 < 90:
            time.sleep(0.2)
        time.sleep(1.0)
    finally:
        for p, _, _ in decs:
            p.send_signal(signal.SIGTERM)
        rcs = [p.wait(timeout=120) for p, _, _ in decs]
    for (p, lines, th), want, rc in zip(decs, wants, rcs):
        th.join(timeout=10)
        assert rc == 0, '\n'.join(lines[-10:])
        console = [l for l in lines if l.startswith('{')]
        assert console == expected(want, 3)


def test_multi_topic_decoder(engine_lib, cpu_libs, tmp_path):
    """One aero-decode process for all 64 VFO topics of the C5 receiver
    (repeated -t, per-topic -b and -s): aero-publish (GPU channeliser) ->
    ZeroMQ -> one SUB socket with 64 subscriptions -> one engine channel per
    topic, one aero_run per batch of queued messages.  Each topic's jsondump
    lines (told apart by their station id) equal what a separate reference
    aero-decode would print: the oracle publisher's audio through the oracle
    decoder (publish/vfo.cpp -> decode/decode.cpp, config C5)."""
    import build
    import aero_engine as ae
    build.build_host()
    cfg = tl.c5_config()
    x = tl.c5_wideband(cfg, 8.0)
    ref = tl.OraclePublisher(cfg['sample_rate'], cfg['center_frequency'], cfg['mains'], cfg['vfos'])
    nb = len(x) // ref.block_len
    ref.process(x[:nb * ref.block_len])
    wb = tmp_path / 'wideband.cf32'
    x[:nb * ref.block_len].astype(np.complex64).tofile(str(wb))
    port = free_port()
    ini = tmp_path / 'c5.ini'
    ini.write_text(tl.c5_ini(cfg).replace('tcp://*:6004', 'tcp://127.0.0.1:%d' % port))
    nv = len(cfg['vfos'])
    wants = []
    for v in range(nv):
        o = tl.Oracle(bitrate=ae.vfo_bitrate(cfg["vfos"][v]["data_rate"]), dcd_tick=True)
        o.push_chunked(ref.usb(v), ref.info(v)['samples_per_block'])
        wants.append(o.item_lines('A'))
    assert sum(len(w) for w in wants) >= 40
    args = ['-p', 'tcp://127.0.0.1:%d' % port, '--format', 'jsondump', '-v']
    for v in range(nv):
        args += ['-t', 'VFO%02d' % (v + 1), '-b', str(cfg['vfos'][v]['data_rate']), '-s', 'ST%02d' % (v + 1)]
    # unpaced file source: unbounded ZeroMQ queues (AERO_ZMQ_HWM=0) so no message is dropped
    dec, lines, th = _start_decoder(args, {'AERO_ZMQ_HWM': '0'})
    try:
        r = subprocess.run([os.path.join(BIN, 'aero-publish'), '-d',
                            'driver=file,path=%s,start_delay_ms=1500' % wb, str(ini)],
                           capture_output=True, text=True, timeout=180, env=dict(os.environ, AERO_ZMQ_HWM='0'))
        assert r.returncode == 0, r.stderr[-3000:]
        # messages still queued at SIGTERM are dropped (as the reference
        # does): wait until the decoder has taken them all, i.e. its output
        # has stopped growing for a few seconds
        t0 = time.time()
        last, t_last = -1, time.time()
        while time.time() - t0 < 150:
            n_now = sum(l.startswith('{') for l in lines)
            if n_now != last:
                last, t_last = n_now, time.time()
            elif time.time() - t_last > 6.0:
                break
            time.sleep(0.2)
    finally:
        dec.send_signal(signal.SIGTERM)
        rc = dec.wait(timeout=120)
    th.join(timeout=10)
    assert rc == 0, '\n'.join(lines[-10:])
    console = [l for l in lines if l.startswith('{')]
    for v in range(nv):
        st = '"ST%02d"' % (v + 1)
        got = [l for l in console if st in l]
        assert got == expected(wants[v], 3, 'ST%02d' % (v + 1)), 'VFO%02d' % (v + 1)
    # every topic's data carrier came up once, each line naming its topic
    for v in range(nv):
        if wants[v]:
            assert sum(('Data carrier detected' in l and '[VFO%02d]' % (v + 1) in l) for l in lines) == 1


def test_msk_vfo_at_explicit_out_rate(engine_lib, cpu_libs, tmp_path):
    """aero-decode -b 600 subscribed to a VFO that aero-publish emits at an
    explicit INI out_rate (publish/publisher.cpp:160-176), here 24000 Hz: the
    MSK demodulator re-applies its settings at the message rate
    (decode/mskdemodulator.cpp:473-481) and the topic decodes; the console
    lines equal the oracle fed the same messages at that rate."""
    import build
    build.build_host()
    pcm = tl.synth_msk(seconds=30.0, bitrate=600, baud=600, seed=0xE104, carrier=1800.0, ebn0=16.0, fs=24000)
    ref = tl.Oracle(bitrate=600)
    ref.push_chunked(pcm, 6000, fs=24000)
    want = ref.item_lines('A')
    assert len(want) >= 1
    f = tmp_path / 'vfo.pcm'
    pcm.astype('<i2').tofile(str(f))
    port = free_port()
    dec, lines, th = _start_decoder(['-p', 'tcp://127.0.0.1:%d' % port, '-t', 'VFO03', '-b', '600', '--format',
                                     'jsondump', '-s', STATION, '-v'], {})
    try:
        r = subprocess.run([PUB, '--bind', 'tcp://127.0.0.1:%d' % port, '--topic', 'VFO03', '--rate', '24000',
                            '--chunk', '6000', '--wait-ms', '1500', str(f)], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        t0 = time.time()
        while sum(l.startswith('{') for l in lines) < len(want) and time.time() - t0 < 90:
            time.sleep(0.2)
        time.sleep(1.0)
    finally:
        dec.send_signal(signal.SIGTERM)
        rc = dec.wait(timeout=120)
    th.join(timeout=10)
    assert rc == 0, '\n'.join(lines[-20:])
    assert not any('CRIT' in l for l in lines), '\n'.join(lines[-20:])
    assert [l for l in lines if l.startswith('{')] == expected(want, 3)
