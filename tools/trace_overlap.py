"""Concurrency in a rocprofv3 kernel trace (--kernel-trace --output-format
csv): per kernel name the launches and device time, per queue the busy time,
and over the traced window the time any kernel ran and the time two or more
ran at once.  Usage: python tools/trace_overlap.py kernel_trace.csv [t0_frac]
(t0_frac: skip the first fraction of the window, e.g. a pre-roll)."""
import csv
import sys
from collections import defaultdict


def main(path, skip=0.0):
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        name = r.get('Kernel_Name') or r.get('Name')
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        q = r.get('Queue_Id') or r.get('Stream_Id') or '?'
        ev.append((s, e, name, q))
    ev.sort()
    t0, t1 = ev[0][0], max(e for _, e, _, _ in ev)
    t0 = t0 + int((t1 - t0) * skip)
    ev = [x for x in ev if x[0] >= t0]
    per = defaultdict(lambda: [0, 0])
    perq = defaultdict(int)
    for s, e, n, q in ev:
        per[n][0] += 1
        per[n][1] += e - s
        perq[q] += e - s
    pts = sorted([(s, 1) for s, _, _, _ in ev] + [(e, -1) for _, e, _, _ in ev])
    busy = multi = 0
    depth, last = 0, pts[0][0]
    for t, d in pts:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            multi += t - last
        depth += d
        last = t
    win = t1 - t0
    print('window %.1f ms, any kernel %.1f ms (%.0f%%), >= 2 kernels %.1f ms' % (win / 1e6, busy / 1e6,
                                                                                 100.0 * busy / win, multi / 1e6))
    for n, (k, d) in sorted(per.items(), key=lambda x: -x[1][1])[:15]:
        print('  %-70s %5d launches %9.1f ms' % (n[:70], k, d / 1e6))
    for q, d in sorted(perq.items(), key=lambda x: -x[1]):
        print('  queue %-10s %9.1f ms' % (q, d / 1e6))


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
