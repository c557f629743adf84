"""The two oracle builds (aero_oracle.cpp header, ORACLE_CR_LIBM): glibc's
per-sample atan2/sin/cos/log10/cexp against correctly rounded ones.  They
may differ only by the libm's last-ulp rounding: identical decoded outputs
on a synthetic stream, pt_qpsk within a few ulps, the hop decisions equal."""
import numpy as np

import aero_testlib as tl


def _run(cr, pcm, bitrate=10500):
    o = tl.Oracle(trace_pt=True, bitrate=bitrate, cr=cr)
    o.push_chunked(pcm, 4096)
    return o


def test_cr_oracle_same_decode_as_glibc_oracle():
    pcm = tl.synth(seconds=10.0, seed=0xAE51)
    g, c = _run(False, pcm), _run(True, pcm)
    assert len(g.softbits()) > 1000
    assert np.array_equal(g.softbits(), c.softbits())
    assert np.array_equal(g.frames(), c.frames())
    assert g.item_lines('A') == c.item_lines('A') and g.item_lines('A')
    pg, pc = g.pt(), c.pt()
    assert pg.shape == pc.shape
    assert np.allclose(pg, pc, rtol=0, atol=1e-12)
    hg, hc = g.hops(), c.hops()
    assert hg.shape == hc.shape
    assert np.array_equal(hg[:, [0, 1, 2, 3, 5]], hc[:, [0, 1, 2, 3, 5]])
    assert np.allclose(hg[:, 4], hc[:, 4], rtol=1e-12, atol=0)


def test_cr_oracle_msk_same_decode():
    pcm = tl.synth_msk(seconds=8.0, seed=0xAE52, bitrate=1200)
    g, c = _run(False, pcm, 1200), _run(True, pcm, 1200)
    assert len(g.softbits()) > 1000
    assert np.array_equal(g.softbits(), c.softbits())
    assert g.item_lines('A') == c.item_lines('A')
