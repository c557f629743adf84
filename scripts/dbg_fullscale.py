"""Diagnostic for tests/test_gpu_fullscale.py: decode the bench pool at C
channels, keep soft bits / hops / pt for a sample of channels, and report
per channel the first hop record and the first pt symbol that differ from
the oracle.  Usage: python scripts/dbg_fullscale.py C [HOPS [ch,ch,...]]"""
import concurrent.futures as cf
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'aero-cli_amd'))
import aero_testlib as tl  # noqa: E402

P, HOP = 64, 4096


def main():
    C = int(sys.argv[1])
    HOPS = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    import torch
    import aero_engine as ae
    import bench
    import shard
    M = bench.MODES['oqpsk10500']
    offsets = shard.channel_offsets(C, P)
    span = HOPS * HOP
    length = span + int(offsets.max()) + 1
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        pool_host = np.stack(list(ex.map(lambda k: bench.synth_one(M, length / 48000.0, 0xAE20 + k, k), range(P))))
    stride = max(1, C // 32)
    sel = sorted(set([stride * k + k for k in range(32) if stride * k + k < C] + [C - 1]))
    if len(sys.argv) > 3:
        sel = sorted(int(v) for v in sys.argv[3].split(','))
    eng = ae.Engine(max_channels=C, flags=ae.F_TRACE_SOFT | ae.F_TRACE_HOPS | ae.F_TRACE_PT)
    for _ in range(C):
        eng.open_channel(10500, 48000)
    eng.trace_select(sel)
    pool = torch.from_numpy(pool_host).to('cuda')
    pts = {c: [] for c in sel}
    for s in range(HOPS):
        views = [pool[:, int(o) + s * HOP:int(o) + (s + 1) * HOP] for o in offsets]
        x = torch.stack(views).permute(2, 0, 1).reshape(HOP, C).contiguous()
        torch.cuda.synchronize()
        eng.push_batch_device(x.data_ptr(), HOP, C, C)
        eng.run()
        for c in sel:
            pts[c].append(eng.pt(c))
        eng.drain_items(lines=True, keep=set())
    eng.flush()
    for c in sel:
        pts[c].append(eng.pt(c))
    got = {c: (eng.softbits(c), eng.hops(c), np.concatenate(pts[c])) for c in sel}
    eng.close()

    def orc(c):
        pcm = pool_host[c % P, int(offsets[c // P]):int(offsets[c // P]) + span]
        o = tl.Oracle(trace_pt=True)
        o.push_chunked(pcm, HOP)
        return o.softbits(), o.hops(), o.pt()
    with cf.ThreadPoolExecutor(max_workers=16) as ex:
        refs = dict(zip(sel, ex.map(orc, sel)))
    bad = 0
    for c in sel:
        sb, hops, pt = got[c]
        rsb, rhops, rpt = refs[c]
        line = 'ch %6d  sb %s' % (c, 'eq' if np.array_equal(sb, rsb) else 'DIFF(%d/%d)' % (len(sb), len(rsb)))
        hv, rv = hops.view(np.int64), rhops.view(np.int64)
        if hv.shape != rv.shape:
            line += '  hops shape %s vs %s' % (hv.shape, rv.shape)
            bad += 1
        else:
            d = np.argwhere(hv != rv)
            if len(d):
                bad += 1
                r, k = d[0]
                line += '  hops first diff row %d col %d (%r vs %r), %d cells' % (r, k, hops[r, k], rhops[r, k], len(d))
            else:
                line += '  hops eq'
        n = min(len(pt), len(rpt))
        pv, rpv = pt[:n].view(np.int64), rpt[:n].view(np.int64)
        d = np.argwhere(pv != rpv)
        if len(d):
            i = d[0][0]
            line += '  pt first diff %d of %d/%d (%r vs %r) maxabs %.3g' % (
                i, len(pt), len(rpt), tuple(pt[i]), tuple(rpt[i]), float(np.abs(pt[:n] - rpt[:n]).max()))
        else:
            line += '  pt eq (%d/%d)' % (len(pt), len(rpt))
        print(line, flush=True)
    print('channels with hop diffs: %d of %d' % (bad, len(sel)), flush=True)


if __name__ == '__main__':
    main()
