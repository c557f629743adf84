"""Builds profiles/pmc_<mode>.json (the HBM traffic bench.py reports as
roofline.traffic) from one FETCH_SIZE and one WRITE_SIZE rocprofv3 --pmc
capture of the same bench configuration (scripts/profile_round.sh).
FETCH_SIZE is doubled (MI355X_MICROARCH.md: gfx950 FETCH_SIZE reports half
the bytes of wide reads); both counters are in KiB.
Usage: python tools/pmc_json.py FETCH.csv WRITE.csv OUT.json [mode channels source-note]"""
import json
import sys

import pmc_summary

ALGO_BYTES = {'oqpsk10500': 18.22}  # bytes per input sample of the demod
HOP = {'oqpsk10500': 4096}


def main():
    fetch, write, out = sys.argv[1:4]
    mode = sys.argv[4] if len(sys.argv) > 4 else 'oqpsk10500'
    channels = int(sys.argv[5]) if len(sys.argv) > 5 else 65536
    note = sys.argv[6] if len(sys.argv) > 6 else ''
    s = pmc_summary.summary(pmc_summary.load([fetch, write]))
    kern = {}
    for k, d in s.items():
        fb = 2.0 * d.get('FETCH_SIZE', 0.0) * 1024
        wb = d.get('WRITE_SIZE', 0.0) * 1024
        kern[k] = {'fetch_bytes_x2': int(fb), 'write_bytes': int(wb), 'hbm_bytes_per_launch': int(fb + wb),
                   'dispatches': d['dispatches'], 'avg_ns': int(d['avg_ns'])}
    dom = next(k for k in kern if k.startswith('demod_oqpsk_kernel'))
    algo = int(ALGO_BYTES[mode] * channels * HOP[mode])
    res = {'source': note, 'config': {'mode': mode, 'channels': channels},
           'correction': 'FETCH_SIZE doubled (gfx950 reports half the bytes); counters in KiB; both count '
                         'Infinity-Cache traffic',
           'kernels': kern, 'kernel': 'demod_oqpsk_kernel', 'hbm_bytes_per_launch': kern[dom]['hbm_bytes_per_launch'],
           'algorithmic_bytes_per_launch': algo,
           'ratio_to_algorithmic': round(kern[dom]['hbm_bytes_per_launch'] / algo, 2)}
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
