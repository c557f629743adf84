"""Static instruction mix of one kernel in a gfx950 assembly listing, split
into the sections of its AERO_X_STAMPS build (each s_memtime closes one).

  python tools/isa_split.py coarse_stamps.s coarse_kernelILi0E [--sections NAMES]

Categories: FP64 arithmetic (add/mul/fma), FP64 special (division and
square-root sequences, frexp/ldexp/class), moves (v_mov, v_cndmask, AGPR
moves), lane permutes (permlane, DPP, bpermute, v_perm), integer/other VALU,
compares, LDS, global/scratch memory, SALU, waits/barriers.  The counts are
static (most of the coarse kernel is unrolled; its log10 pass and fold
search are loops, listed once)."""
import re
import sys
from collections import Counter, OrderedDict

CATS = OrderedDict([
    ('fp64_arith', re.compile(r'^v_(add|mul|fma|fmac|sub)_f64')),
    ('fp64_special', re.compile(r'^v_(div_|rcp_f64|rsq_f64|sqrt_f64|frexp|ldexp_f64|cmp_class_f64|trig_preop|fract_f64|'
                                r'rndne_f64|floor_f64|trunc_f64|ceil_f64|max_f64|min_f64|cvt_f64|cvt_i32_f64|'
                                r'cvt_u32_f64)')),
    ('moves', re.compile(r'^v_(mov|cndmask|accvgpr|swap)')),
    ('permutes', re.compile(r'^(v_permlane|v_perm_b32|ds_bpermute|ds_permute|ds_swizzle|v_readlane|v_writelane|'
                            r'v_readfirstlane)|_dpp')),
    ('compare', re.compile(r'^v_cmp')),
    ('int_valu', re.compile(r'^v_')),
    ('lds', re.compile(r'^ds_')),
    ('memory', re.compile(r'^(global_|buffer_|flat_|scratch_|s_load|s_buffer_load)')),
    ('wait_barrier', re.compile(r'^(s_waitcnt|s_barrier|s_sleep|s_nop)')),
    ('salu', re.compile(r'^s_')),
])


def classify(op):
    for k, rx in CATS.items():
        if rx.search(op):
            return k
    return 'other'


def kernel_lines(path, name):
    out, on = [], False
    for line in open(path):
        if not on and re.match(r'^_ZN\w*%s\w*:' % re.escape(name), line):
            on = True
            continue
        if on:
            if line.startswith('.Lfunc_end') or re.match(r'^\s*\.size\s', line):
                break
            out.append(line)
    return out


def split(lines):
    secs, cur = [], Counter()
    for line in lines:
        s = line.strip()
        if not s or s.startswith(('.', ';', '//')) or s.endswith(':'):
            continue
        op = s.split()[0]
        if op == 's_memtime':
            secs.append(cur)
            cur = Counter()
            continue
        cur[classify(op)] += 1
    secs.append(cur)
    return secs


def main(argv):
    path, name = argv[0], argv[1]
    names = argv[3].split(',') if len(argv) > 3 and argv[2] == '--sections' else None
    secs = split(kernel_lines(path, name))
    cols = list(CATS) + ['other']
    print('%-26s' % 'section' + ''.join('%13s' % c for c in cols) + '%9s' % 'total')
    tot = Counter()
    for i, c in enumerate(secs):
        label = names[i] if names and i < len(names) else 'section %d' % i
        print('%-26s' % label[:26] + ''.join('%13d' % c[k] for k in cols) + '%9d' % sum(c.values()))
        tot += c
    print('%-26s' % 'kernel' + ''.join('%13d' % tot[k] for k in cols) + '%9d' % sum(tot.values()))


if __name__ == '__main__':
    main(sys.argv[1:])
