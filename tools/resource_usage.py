"""Per-kernel register / spill / occupancy table of the engine's HIP sources
(the compiler's kernel-resource-usage remarks, with the product build's
per-file flags).  Usage: python tools/resource_usage.py [file.hip ...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'aero-cli_amd'))
import build  # noqa: E402

FIELDS = [('VGPRs', 'vgpr'), ('AGPRs', 'agpr'), ('ScratchSize [bytes/lane]', 'scratch'),
          ('Occupancy [waves/SIMD]', 'occ'), ('SGPRs Spill', 'sspill'), ('VGPRs Spill', 'vspill'),
          ('LDS Size [bytes/block]', 'lds')]


def usage(src, extra=()):
    name = os.path.basename(src)
    with tempfile.TemporaryDirectory() as td:
        cmd = ([build.HIPCC] + build.HIP_FLAGS + build.FILE_FLAGS.get(name, []) + list(extra) +
               ['-Rpass-analysis=kernel-resource-usage', '-c', src, '-o', os.path.join(td, 'o.o')])
        r = subprocess.run(cmd, capture_output=True, text=True)
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r'remark: (.*?) \[-Rpass-analysis', line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith('Function Name:'):
            cur = {'kernel': t.split(':', 1)[1].strip()}
            out.append(cur)
            continue
        for label, key in FIELDS:
            if cur is not None and t.startswith(label + ':'):
                cur[key] = int(t.split(':', 1)[1])
    return out


def main(argv):
    srcs = argv or [os.path.join(build.CSRC, s) for s in build.HIP_SRCS]
    print('%-62s %5s %5s %7s %4s %6s %6s %6s' % ('kernel', 'vgpr', 'agpr', 'scratch', 'occ', 'sspill', 'vspill', 'lds'))
    for s in srcs:
        for k in usage(s if os.path.isabs(s) else os.path.join(build.CSRC, s)):
            n = re.sub(r'^_ZN4aero\d+', '', k['kernel'])[:62]
            print('%-62s %5d %5d %7d %4d %6d %6d %6d' % (n, k.get('vgpr', 0), k.get('agpr', 0), k.get('scratch', 0),
                                                        k.get('occ', 0), k.get('sspill', 0), k.get('vspill', 0),
                                                        k.get('lds', 0)))


if __name__ == '__main__':
    main(sys.argv[1:])
