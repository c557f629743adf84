"""Writes tests/golden/output_items.json: ACARS items that exercise every
branch and escape of aero-decode's console/forwarder formats
(decode/output.cpp:12-171): up/downlink, non-ACARS, NAK (0x15) TAK, DEL
label, CR/LF/TAB/BEL/quote/backslash/control and Latin-1 bytes in the text,
short downlink texts (QString::mid past the end), '%n' sequences that
QString::arg chains re-substitute, fragments (moretocome).  The expected
lines are produced by make_output_golden.cpp (Qt's own QString/QJsonDocument)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def item(**kw):
    d = dict(aesid=0x4CA7E1, gesid=0x42, qno=0x3, refno=0x1A, mode=ord('2'), tak=ord('A'), bi=ord('5'),
             nonacars=0, downlink=0, moretocome=0, label=b'H1', reg=b'.EI-DEF', msg=b'HELLO WORLD')
    d.update(kw)
    for k in ('label', 'reg', 'msg'):
        d[k] = d[k].hex()
    return d


ITEMS = [
    item(),
    item(downlink=1, msg=b'M12AEI1234/REPORT 12:00\r\nPOS N53 W008\r\n'),
    item(tak=0x15, label=b'_\x7f', msg=b''),
    item(nonacars=1, msg=b'0A0B0C0D0E0F', reg=b''),
    item(msg=b'quote " backslash \\ tab\t bell\x07 ff\x0c bs\x08 nul-free ctl\x01\x1f del\x7f'),
    item(msg=bytes(range(0xA0, 0x100)) + b' latin1'),
    item(downlink=1, msg=b'AB'),
    item(downlink=1, msg=b'M12A%1%2 FLT %3 text %10'),
    item(label=b'%1', msg=b'100% done %L1 %99 %0'),
    item(moretocome=1, bi=ord('Z'), mode=ord('E'), reg=b'N123AB'),
    item(msg=b'\n\nleading and trailing newlines\n\n', downlink=0),
    item(gesid=0xC5, aesid=0xABCDEF, qno=0xF, refno=0xFF, downlink=1, msg=b'\r\r\rX'),
]

if __name__ == '__main__':
    with open(os.path.join(HERE, 'output_items.json'), 'w') as f:
        json.dump({'time_ms': 1714558496789, 'station': 'TEST-STATION-\u00c9', 'items': ITEMS}, f, indent=1)
